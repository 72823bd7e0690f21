#!/bin/bash
# round 6: bf16 encoder-output gradient (TSAMD_DE_BF16) -- ctx / LSTM / oracle tests, A/B bench incl. config #5
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-r6de}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_ctx.py tests/test_gpu_lstm.py tests/test_gpu_production.py tests/test_gpu_model.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for de in 1 0 1 0; do
  TSAMD_DE_BF16=$de timeout -k 10 400 python bench.py --steps 10 --warmup 3 --decode-batches 0 > $OUT/bench_de$de.log 2>&1 || exit 1
  python -c "import json;r=json.loads(open('$OUT/bench_de$de.log').read().strip().splitlines()[-1]);print('de_bf16 $de', r['ms_per_step'], r.get('config5_ms_per_step'), r.get('config5_tokens_per_sec'), r.get('config5_search_peak_mem_gb'))"
done
echo done
