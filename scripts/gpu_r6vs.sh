#!/bin/bash
# round 6: vocab_train with scalar FP32 softmax epilogues (no packed ops in the MFMA gaps)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-r6vs}; mkdir -p $OUT
timeout -k 10 120 python tools/vocab_train_micro.py --rows 20480 > $OUT/micro.jsonl 2>&1 || { tail -5 $OUT/micro.jsonl; exit 1; }
echo "H256 $(tail -1 $OUT/micro.jsonl)"
timeout -k 10 120 python tools/vocab_train_micro.py --rows 20480 --hidden 512 > $OUT/micro512.jsonl 2>&1 || { tail -5 $OUT/micro512.jsonl; exit 1; }
echo "H512 $(tail -1 $OUT/micro512.jsonl)"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_model.py tests/test_gpu_production.py \
  -k "fused_vocab_head or bench_shape_matches or config5_shape_matches or deterministic_mode" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --decode-batches 0 --config5-steps 0 > $OUT/b$i.log 2>&1 || { echo "bench failed"; tail -5 $OUT/b$i.log; exit 1; }
  python -c "import json;r=json.loads(open('$OUT/b$i.log').read().strip().splitlines()[-1]);print('bench', r['ms_per_step'], r.get('phase_ms_max_over_ranks'))"
done
timeout -k 10 400 python bench.py --steps 1 --warmup 1 --decode-batches 0 --config5-steps 4 > $OUT/c5.log 2>&1 || { echo "c5 failed"; tail -5 $OUT/c5.log; exit 1; }
python -c "import json;r=json.loads(open('$OUT/c5.log').read().strip().splitlines()[-1]);print('c5', r['config5_ms_per_step'])"
echo done
