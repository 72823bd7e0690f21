#!/bin/bash
# round 6: HIP graph execution knobs vs the headline step (parallel row-group branches)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-r6gq}; mkdir -p $OUT
for cfg in "X=0" "DEBUG_HIP_FORCE_GRAPH_QUEUES=1" "DEBUG_HIP_FORCE_GRAPH_QUEUES=2" "DEBUG_HIP_FORCE_GRAPH_QUEUES=4" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=1" "X=0"; do
  tag=$(echo $cfg | tr '=' '_')
  env $cfg timeout -k 10 300 python bench.py --steps 20 --warmup 5 --decode-batches 0 --config5-steps 0 > $OUT/b_$tag.log 2>&1 || { echo "$cfg failed"; tail -3 $OUT/b_$tag.log; continue; }
  python -c "import json;r=json.loads(open('$OUT/b_$tag.log').read().strip().splitlines()[-1]);print('$cfg', r['ms_per_step'])"
done
echo done
