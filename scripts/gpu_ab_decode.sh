#!/bin/bash
# bench_decode A/B: for each env assignment in $VARIANTS (":" joins several; "-" = none).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-abdec}; mkdir -p $OUT
i=0
for v in $VARIANTS; do
  i=$((i+1)); e=""; [ "$v" != "-" ] && e="${v//:/ }"
  timeout -k 10 300 env $e python bench_decode.py ${DEC_ARGS} > $OUT/v$i.log 2>&1 || { tail -20 $OUT/v$i.log; exit 1; }
  echo "[$v] $(tail -1 $OUT/v$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_batch"], d["ms_per_batch_median"])')"
done
echo done
