#!/bin/bash
# round 6: vocab dW beside the decoder backward loop -- side-stream CU masks / priorities vs the headline
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-r6dw2}; mkdir -p $OUT
timeout -k 10 120 python -c "from textsummarization_on_flink_amd.ops import ops; print('prio range', list(ops().stream_priority_range()))" || exit 1
for cfg in "TSAMD_VOCAB_DW_SIDE=0" "X=0" "TSAMD_VOCAB_DW_CUS=64:1" "TSAMD_VOCAB_DW_CUS=64:4" "TSAMD_VOCAB_DW_CUS=32:8" "TSAMD_VOCAB_DW_CUS=128:2" "TSAMD_VOCAB_DW_PRIO=1" "TSAMD_VOCAB_DW_PRIO=0" "TSAMD_VOCAB_DW_SIDE=0"; do
  tag=$(echo $cfg | tr '=:' '__')
  env $cfg timeout -k 10 300 python bench.py --steps 20 --warmup 5 --decode-batches 0 --config5-steps 0 > $OUT/b_$tag.log 2>&1 || { echo "$cfg failed"; tail -5 $OUT/b_$tag.log; exit 1; }
  python -c "import json;r=json.loads(open('$OUT/b_$tag.log').read().strip().splitlines()[-1]);print('$cfg', r['ms_per_step'], r.get('phase_ms_max_over_ranks'))"
done
echo done
