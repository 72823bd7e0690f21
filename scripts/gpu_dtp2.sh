#!/bin/bash
# decode with trained / random weights after the vocab_select group bound; decode tests first
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-dtp2}; mkdir -p $OUT
export TMPDIR=/tmp
step() { local n=$1; shift; echo "== $n"; timeout -k 10 ${T:-300} "$@" > $OUT/$n.log 2>&1; local rc=$?; grep -h '^{' $OUT/$n.log | cut -c1-300; tail -2 $OUT/$n.log; return $rc; }
T=600 step tests python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_decode_parity.py -q -x --timeout 300 --timeout-method thread &&
step tr python -u tools/decode_trained_prof.py --train-steps 80 --batches 10 &&
step rnd python -u tools/decode_trained_prof.py --train-steps 0 --batches 10 &&
step tr2 python -u tools/decode_trained_prof.py --train-steps 300 --batches 10 &&
step dec python -u bench_decode.py --batches 10
