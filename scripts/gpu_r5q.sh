#!/bin/bash
# round 5: encoder layer 0's input projection inside the persistent recurrence (FX) --
# kernel numerics, engine oracles, then the headline + config #5 bench with TSAMD_LSTM_FX=0 / 1.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5q; mkdir -p $OUT
export TMPDIR=/tmp
step() { local n=$1; shift; echo "== $n"; timeout -k 10 ${T:-300} "$@" > $OUT/$n.log 2>&1; local rc=$?; tail -${TL:-3} $OUT/$n.log; return $rc; }
T=300 step lstm python -u -m pytest tests/test_gpu_lstm.py -q -x --timeout 120 --timeout-method thread || exit 1
T=700 step orc python -u -m pytest tests/test_gpu_production.py -q -x --timeout 300 --timeout-method thread || exit 1
T=500 TL=1 step fx1 python -u bench.py --steps 20 --warmup 3 --decode-batches 0 --config5-steps 5 || exit 1
T=500 TL=1 step fx0 env TSAMD_LSTM_FX=0 python -u bench.py --steps 20 --warmup 3 --decode-batches 0 --config5-steps 5 || exit 1
echo done
