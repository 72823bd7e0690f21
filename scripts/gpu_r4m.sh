#!/bin/bash
# round-4: decoder backward in two launches per step -- kernel + engine tests, the model oracle
# tests, then bench / phase A/B against the three-launch loop
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-r4m}; mkdir -p $OUT
export TMPDIR=/tmp
step() { local n=$1; shift; echo "== $n"; timeout -k 10 ${T:-300} "$@" > $OUT/$n.log 2>&1; local rc=$?; tail -${TL:-3} $OUT/$n.log; return $rc; }
step kt python -u -m pytest tests/test_gpu_attention_ops.py -x -q --timeout 100 --timeout-method thread -k "rowp" &&
T=400 step et python -u -m pytest tests/test_gpu_production.py -x -q --timeout 200 --timeout-method thread -k "two_launches or oracle or split_streams or deterministic" &&
step ph2 python -u tools/phase_micro.py &&
TSAMD_DEC_BWD_2L=0 step ph3 python -u tools/phase_micro.py &&
step b2 python -u bench.py --decode-batches 0 --config5-steps 0 &&
TSAMD_DEC_BWD_2L=0 step b3 python -u bench.py --decode-batches 0 --config5-steps 0 &&
step b2b python -u bench.py --decode-batches 0 --config5-steps 0 &&
step ph5 python -u tools/phase_micro.py --batch 1024 --hidden 512 --enc 800 --layers 2 --iters 3 &&
TSAMD_DEC_BWD_2L=0 step ph5o python -u tools/phase_micro.py --batch 1024 --hidden 512 --enc 800 --layers 2 --iters 3
