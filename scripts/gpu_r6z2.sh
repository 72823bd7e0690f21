#!/bin/bash
# round 6: config #5 bench A/B of the 32-row BPTT's deferred dz stores (TSAMD_LSTM_DEFER_DZ), + LSTM tests
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-r6z2}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_lstm.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_lstm.log 2>&1; rc=$?; tail -1 $OUT/pytest_lstm.log; [ $rc -eq 0 ] || exit $rc
for df in 1 0 1 0; do
  TSAMD_LSTM_DEFER_DZ=$df timeout -k 10 400 python bench.py --steps 3 --warmup 1 --decode-batches 0 > $OUT/bench_df$df.log 2>&1 || exit 1
  python -c "import json;r=json.loads(open('$OUT/bench_df$df.log').read().strip().splitlines()[-1]);print('defer $df', r['ms_per_step'], r.get('config5_ms_per_step'), r.get('config5_tokens_per_sec'))"
done
echo done
