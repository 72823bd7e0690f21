#!/bin/bash
# round 6: BPTT with deferred dz stores + LDS-only barriers (16- and 32-row kernels) -- LSTM
# tests, micro A/B (TSAMD_LSTM_DEFER_DZ / _DZ16), stamps A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-r6z}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_lstm.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_lstm.log 2>&1; rc=$?; tail -2 $OUT/pytest_lstm.log; [ $rc -eq 0 ] || exit $rc
for df in 1 0 1 0; do
  TSAMD_LSTM_DEFER_DZ=$df TSAMD_LSTM_DEFER_DZ16=$df timeout -k 10 300 python tools/lstm_micro.py 256:256:400 512:256:400 512:1024:800 512:2048:800 > $OUT/micro_df$df.jsonl 2>&1 || exit 1
  python -c "import json;[print('defer $df', (r:=json.loads(l))['H'], r['B'], r['bwd_us'], r['bwd_us_per_step'], r['err']) for l in open('$OUT/micro_df$df.jsonl') if l.startswith('{')]"
done
TSAMD_LSTM_DEFER_DZ=1 timeout -k 10 200 python tools/lstm_bptt_stamps.py 512:1024:800 > $OUT/stamps_df1.jsonl 2>&1 || exit 1
TSAMD_LSTM_DEFER_DZ=0 timeout -k 10 200 python tools/lstm_bptt_stamps.py 512:1024:800 > $OUT/stamps_df0.jsonl 2>&1 || exit 1
cat $OUT/stamps_df*.jsonl | grep -o '"us_plain[^}]*}'
echo done
