#!/bin/bash
# round 5: decoder RT-kernel diagnostics, then the RT / vocab A/Bs (gpu_r5h minus its first step) and the
# three-deep-A gemm_bt A/B (gpu_r5i).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-r5j}; mkdir -p $OUT
export TMPDIR=/tmp
step() { local n=$1; shift; echo "== $n"; timeout -k 10 ${T:-300} "$@" > $OUT/$n.log 2>&1; local rc=$?; tail -${TL:-3} $OUT/$n.log; return $rc; }
TL=12 step rt python -u -m pytest tests/test_gpu_decoder_rt.py -q --timeout 120 --timeout-method thread
rc=$?; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
TSAMD_GEMM_V=5 step gemmt5 python -u -m pytest tests/test_gpu_gemm.py -q -x --timeout 120 --timeout-method thread || exit 1
TL=10 step gemm5 env TSAMD_GEMM_V=5 python -u tools/gemm_micro.py || exit 1
TL=10 step gemm3 python -u tools/gemm_micro.py || exit 1
T=600 step orc python -u -m pytest tests/test_gpu_production.py -q -x --timeout 300 --timeout-method thread -k "config5_shape" || exit 1
TSAMD_VL_RH=4 step dect4 python -u -m pytest tests/test_gpu_decode.py -q -x --timeout 300 --timeout-method thread -k "topk or vocab" || exit 1
T=500 TL=1 step c1 python -u bench.py --steps 20 --warmup 3 --decode-batches 0 --config5-steps 3 || exit 1
TSAMD_DEC_RT=0 T=500 TL=1 step c0 python -u bench.py --steps 1 --warmup 1 --decode-batches 0 --config5-steps 3 || exit 1
TSAMD_GEMM_V=5 T=500 TL=1 step c5 python -u bench.py --steps 20 --warmup 3 --decode-batches 0 --config5-steps 3 || exit 1
TL=1 step d2 python -u bench_decode.py --batches 10 || exit 1
TSAMD_VL_RH=4 TL=1 step d4 python -u bench_decode.py --batches 10 || exit 1
TL=1 step d2b python -u bench_decode.py --batches 10 || exit 1
TSAMD_VL_RH=4 TL=1 step d4b python -u bench_decode.py --batches 10 || exit 1
echo done
