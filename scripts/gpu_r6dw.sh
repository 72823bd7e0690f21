#!/bin/bash
# round 6: vocab dW graph beside the decoder backward loop (TSAMD_VOCAB_DW_SIDE) -- tests, then A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-r6dw}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_production.py \
  -k "vocab_dw_beside or graph_replay_equals" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -4 $OUT/tests.log
for side in 0 1 0 1; do
  TSAMD_VOCAB_DW_SIDE=$side timeout -k 10 300 python bench.py --steps 20 --warmup 5 --decode-batches 0 --config5-steps 0 \
    > $OUT/b_side$side.log 2>&1 || { echo "side=$side failed"; tail -5 $OUT/b_side$side.log; exit 1; }
  python -c "import json;r=json.loads(open('$OUT/b_side$side.log').read().strip().splitlines()[-1]);print('side=$side', r['ms_per_step'], r.get('phase_ms_max_over_ranks'))"
done
for side in 0 1; do
  TSAMD_VOCAB_DW_SIDE=$side timeout -k 10 400 python bench.py --steps 1 --warmup 1 --decode-batches 0 --config5-steps 4 \
    > $OUT/c5_side$side.log 2>&1 || { echo "c5 side=$side failed"; tail -5 $OUT/c5_side$side.log; exit 1; }
  python -c "import json;r=json.loads(open('$OUT/c5_side$side.log').read().strip().splitlines()[-1]);print('c5 side=$side', {k:v for k,v in r.items() if 'config5' in k})"
done
echo done
