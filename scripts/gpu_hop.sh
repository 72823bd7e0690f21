#!/bin/bash
# step_frame_hop: config #5 phases and bench twice, then the whole tier
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-hop2}; mkdir -p $OUT
export TMPDIR=/tmp
step() { local n=$1; shift; echo "== $n"; timeout -k 10 ${T:-300} "$@" > $OUT/$n.log 2>&1; local rc=$?; grep -h -o '"ms_per_step": [0-9.]*\|"config5_ms_per_step": [0-9.]*\|"backward_tail": [0-9.]*\|"total": [0-9.]*\|[0-9]* passed' $OUT/$n.log | tr '\n' ' '; echo; return $rc; }
step ph5 python -u tools/phase_micro.py --batch 1024 --hidden 512 --enc 800 --layers 2 --iters 3 &&
T=600 step bench1 python -u bench.py --decode-batches 0 &&
T=600 step bench2 python -u bench.py --decode-batches 0 &&
T=900 step tier python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread
