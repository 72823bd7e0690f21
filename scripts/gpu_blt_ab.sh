#!/bin/bash
# blt_mm: numerics tests, then bench.py with TSAMD_BLT=1 / 0 (B = 256 + config #5), back to back
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-bltab}; mkdir -p $OUT
export TMPDIR=/tmp
step() { local n=$1; shift; echo "== $n"; timeout -k 10 ${T:-300} "$@" > $OUT/$n.log 2>&1; local rc=$?; tail -${TL:-3} $OUT/$n.log; return $rc; }
T=300 step blt_tests python -u -m pytest tests/test_gpu_blt.py -v -x --timeout 120 --timeout-method thread &&
T=600 step tests python -u -m pytest tests/test_gpu_model.py tests/test_gpu_production.py -q -x --timeout 300 --timeout-method thread &&
T=600 step bench_blt1 env TSAMD_BLT=1 python -u bench.py --decode-batches 4 &&
T=600 step bench_blt0 env TSAMD_BLT=0 python -u bench.py --decode-batches 4 &&
T=600 step bench_blt1b env TSAMD_BLT=1 python -u bench.py --decode-batches 4
