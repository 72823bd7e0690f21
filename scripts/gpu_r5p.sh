#!/bin/bash
# round 5: closing tier on the current tree, then the staggered gemm_bt (TSAMD_GEMM_V=6) A/B:
# numerics, micro shapes, headline + config #5 bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUTD=r5final2 bash scripts/gpu_r5final.sh || exit 1
OUT=gpurun_out/r5p; mkdir -p $OUT
export TMPDIR=/tmp
step() { local n=$1; shift; echo "== $n"; timeout -k 10 ${T:-300} "$@" > $OUT/$n.log 2>&1; local rc=$?; tail -${TL:-3} $OUT/$n.log; return $rc; }
T=120 step gemmt6 env TSAMD_GEMM_V=6 python -u -m pytest tests/test_gpu_gemm.py -q -x --timeout 60 --timeout-method thread || exit 1
TL=10 step gemm6 env TSAMD_GEMM_V=6 python -u tools/gemm_micro.py || exit 1
T=600 step orc6 env TSAMD_GEMM_V=6 python -u -m pytest tests/test_gpu_production.py -q -x --timeout 300 --timeout-method thread -k "config5_shape or bench_shape" || exit 1
T=500 TL=1 step c6 env TSAMD_GEMM_V=6 python -u bench.py --steps 20 --warmup 3 --decode-batches 0 --config5-steps 5 || exit 1
T=500 TL=1 step c3 python -u bench.py --steps 20 --warmup 3 --decode-batches 0 --config5-steps 5 || exit 1
echo done
