#!/bin/bash
# round 6: engine-switch sweep at the headline (same box, 20 timed steps each)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-r6sw}; mkdir -p $OUT
for cfg in "X=0" "TSAMD_SPLIT=4" "TSAMD_SPLIT_BWD=4" "TSAMD_SPLIT=4 TSAMD_SPLIT_BWD=4" "TSAMD_SPLIT=1" "TSAMD_DEFER_WGRAD=0" "X=0"; do
  tag=$(echo $cfg | tr '= ' '__')
  env $cfg timeout -k 10 300 python bench.py --steps 20 --warmup 5 --decode-batches 0 --config5-steps 0 > $OUT/b_$tag.log 2>&1 || { echo "$cfg failed"; tail -5 $OUT/b_$tag.log; exit 1; }
  python -c "import json;r=json.loads(open('$OUT/b_$tag.log').read().strip().splitlines()[-1]);print('$cfg', r['ms_per_step'])"
done
echo done
