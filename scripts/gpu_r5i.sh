#!/bin/bash
# round 5: gemm_bt with a three-deep A pipeline (TSAMD_GEMM_V=5) against the two-stage kernel and
# hipBLASLt: numerics under V=5, micro shapes both ways, headline and config #5 bench both ways.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-r5i}; mkdir -p $OUT
export TMPDIR=/tmp
step() { local n=$1; shift; echo "== $n"; timeout -k 10 ${T:-300} "$@" > $OUT/$n.log 2>&1; local rc=$?; tail -${TL:-3} $OUT/$n.log; return $rc; }
TSAMD_GEMM_V=5 step gemmt5 python -u -m pytest tests/test_gpu_gemm.py -q -x --timeout 120 --timeout-method thread || exit 1
TL=10 step gemm3 python -u tools/gemm_micro.py || exit 1
TSAMD_GEMM_V=5 TL=10 step gemm5 python -u tools/gemm_micro.py || exit 1
TSAMD_GEMM_V=5 T=600 step orc5 python -u -m pytest tests/test_gpu_production.py -q -x --timeout 300 --timeout-method thread -k "config5_shape or bench_shape" || exit 1
TSAMD_GEMM_V=5 T=500 TL=1 step c5 python -u bench.py --steps 20 --warmup 3 --decode-batches 0 --config5-steps 3 || exit 1
T=500 TL=1 step c3 python -u bench.py --steps 20 --warmup 3 --decode-batches 0 --config5-steps 3 || exit 1
echo done
