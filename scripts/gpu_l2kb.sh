#!/bin/bash
# linear2 k-batch by K: linear2 tests, decode and bench (B = 256 + config #5) twice
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-l2kb}; mkdir -p $OUT
export TMPDIR=/tmp
step() { local n=$1; shift; echo "== $n"; timeout -k 10 ${T:-300} "$@" > $OUT/$n.log 2>&1; local rc=$?; grep -h -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"config5_ms_per_step": [0-9.]*\|"beam4_summaries_per_sec": [0-9.]*\|[0-9]* passed' $OUT/$n.log | tr '\n' ' '; echo; return $rc; }
step tests python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_model.py -q -x --timeout 300 --timeout-method thread &&
step dec1 python -u bench_decode.py --batches 10 &&
step dec2 python -u bench_decode.py --batches 10 &&
T=600 step bench1 python -u bench.py --decode-batches 4 &&
T=600 step bench2 python -u bench.py --decode-batches 4
