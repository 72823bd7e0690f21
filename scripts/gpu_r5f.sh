#!/bin/bash
# round 5: 64-row forward LSTM teams at H = 512 (TSAMD_LSTM_FWD64) and the merged encoder
# input-gradient GEMM (TSAMD_DX_MERGE): kernel tests, config #5 oracle, micro timings and
# config #5 / headline bench on both sides of each switch.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-r5f}; mkdir -p $OUT
export TMPDIR=/tmp
step() { local n=$1; shift; echo "== $n"; timeout -k 10 ${T:-300} "$@" > $OUT/$n.log 2>&1; local rc=$?; tail -${TL:-3} $OUT/$n.log; return $rc; }
step kt python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_lstm.py -q -x --timeout 200 --timeout-method thread || exit 1
T=600 step orc python -u -m pytest tests/test_gpu_production.py -q -x --timeout 300 --timeout-method thread -k "config5_shape or bench_shape" || exit 1
step m1 python -u tools/lstm_micro.py 512:1024:800 512:2048:800 512:768:800 || exit 1
TSAMD_LSTM_FWD64=0 step m0 python -u tools/lstm_micro.py 512:1024:800 512:2048:800 512:768:800 || exit 1
T=500 TL=1 step c11 python -u bench.py --steps 1 --warmup 1 --decode-batches 0 --config5-steps 3 || exit 1
TSAMD_LSTM_FWD64=0 T=500 TL=1 step c01 python -u bench.py --steps 1 --warmup 1 --decode-batches 0 --config5-steps 3 || exit 1
TSAMD_DX_MERGE=0 T=500 TL=1 step c10 python -u bench.py --steps 1 --warmup 1 --decode-batches 0 --config5-steps 3 || exit 1
T=400 TL=1 step b1 python -u bench.py --steps 20 --warmup 3 --decode-batches 0 --config5-steps 0 || exit 1
TSAMD_DX_MERGE=0 T=400 TL=1 step b0 python -u bench.py --steps 20 --warmup 3 --decode-batches 0 --config5-steps 0 || exit 1
echo done
