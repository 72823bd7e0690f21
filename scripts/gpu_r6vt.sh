#!/bin/bash
# round 6: vocab_train 128-column tiles at 3 workgroups per CU (TSAMD_VT_NI=2) vs 256 at 2
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-r6vt}; mkdir -p $OUT
for ni in 0 2; do
  TSAMD_VT_NI=$ni timeout -k 10 120 python tools/vocab_train_micro.py --rows 20480 > $OUT/micro_ni$ni.jsonl 2>&1 || { tail -5 $OUT/micro_ni$ni.jsonl; exit 1; }
  echo "ni=$ni $(tail -1 $OUT/micro_ni$ni.jsonl)"
  TSAMD_VT_NI=$ni timeout -k 10 120 python tools/vocab_train_micro.py --rows 20480 --hidden 128 > $OUT/micro128_ni$ni.jsonl 2>&1 || { tail -5 $OUT/micro128_ni$ni.jsonl; exit 1; }
  echo "H128 ni=$ni $(tail -1 $OUT/micro128_ni$ni.jsonl)"
done
TSAMD_VT_NI=2 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_model.py \
  -k "fused_vocab_head" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for ni in 0 2 0 2; do
  TSAMD_VT_NI=$ni timeout -k 10 300 python bench.py --steps 20 --warmup 5 --decode-batches 0 --config5-steps 0 > $OUT/b_ni$ni.log 2>&1 || { echo "ni=$ni failed"; tail -5 $OUT/b_ni$ni.log; exit 1; }
  python -c "import json;r=json.loads(open('$OUT/b_ni$ni.log').read().strip().splitlines()[-1]);print('ni=$ni', r['ms_per_step'], r.get('phase_ms_max_over_ranks'))"
done
echo done
