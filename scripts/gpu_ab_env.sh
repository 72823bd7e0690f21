#!/bin/bash
# Generic bench A/B: for each env assignment in $VARIANTS (space separated, ":" joins several; "-" = none) run
# bench.py $BENCH_ARGS and print ms/step + value.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-abenv}; mkdir -p $OUT
export TMPDIR=/tmp
i=0
for v in $VARIANTS; do
  i=$((i+1)); e=""; [ "$v" != "-" ] && e="${v//:/ }"
  timeout -k 10 400 env $e python bench.py ${BENCH_ARGS} > $OUT/v$i.log 2>&1 || { tail -20 $OUT/v$i.log; exit 1; }
  echo "[$v] $(tail -1 $OUT/v$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d.get("beam4_summaries_per_sec"))')"
done
echo done
