#!/bin/bash
# round 5: 64-row forward LSTM teams at H = 512 (TSAMD_LSTM_FWD64): persistent-vs-step-kernel
# tests, per-launch-sequence micro timings on both sides, config #5 bench on both sides.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-r5f}; mkdir -p $OUT
export TMPDIR=/tmp
step() { local n=$1; shift; echo "== $n"; timeout -k 10 ${T:-300} "$@" > $OUT/$n.log 2>&1; local rc=$?; tail -${TL:-3} $OUT/$n.log; return $rc; }
step lstmt python -u -m pytest tests/test_gpu_lstm.py -q -x --timeout 200 --timeout-method thread || exit 1
TL=3 step m1 python -u tools/lstm_micro.py 512:1024:800 512:2048:800 512:768:800 || exit 1
TSAMD_LSTM_FWD64=0 TL=3 step m0 python -u tools/lstm_micro.py 512:1024:800 512:2048:800 512:768:800 || exit 1
T=500 TL=1 step c1 python -u bench.py --steps 1 --warmup 1 --decode-batches 0 --config5-steps 3 || exit 1
TSAMD_LSTM_FWD64=0 T=500 TL=1 step c0 python -u bench.py --steps 1 --warmup 1 --decode-batches 0 --config5-steps 3 || exit 1
echo done
