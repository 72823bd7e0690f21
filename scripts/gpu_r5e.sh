#!/bin/bash
# round 5: 4-stage BK=32 gemm_bt (TSAMD_GEMM_V=4) against the 2-stage BK=64 one and hipBLASLt:
# numerics under both, the micro shapes under both, and the headline bench under both.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-r5e}; mkdir -p $OUT
export TMPDIR=/tmp
step() { local n=$1; shift; echo "== $n"; timeout -k 10 ${T:-300} "$@" > $OUT/$n.log 2>&1; local rc=$?; tail -${TL:-3} $OUT/$n.log; return $rc; }
TSAMD_GEMM_V=4 step gemmt4 python -u -m pytest tests/test_gpu_gemm.py -q -x --timeout 120 --timeout-method thread || exit 1
TL=10 step gemm3 python -u tools/gemm_micro.py || exit 1
TSAMD_GEMM_V=4 TL=10 step gemm4 python -u tools/gemm_micro.py || exit 1
T=400 TL=1 step b3 python -u bench.py --steps 20 --warmup 3 --decode-batches 0 --config5-steps 0 || exit 1
TSAMD_GEMM_V=4 T=400 TL=1 step b4 python -u bench.py --steps 20 --warmup 3 --decode-batches 0 --config5-steps 0 || exit 1
echo done
