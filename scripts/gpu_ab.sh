#!/bin/bash
# A/B on one box: ENV_A vs ENV_B (env assignments), interleaved, B=$1.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/ab; mkdir -p $OUT
B=${1:-64}; A_ENV=${2:-X=1}; B_ENV=${3:-X=2}
for r in 1 2 3; do
  for v in A B; do
    if [ $v = A ]; then E=$A_ENV; else E=$B_ENV; fi
    env $E timeout -k 10 300 python bench.py --batch $B --steps 20 > $OUT/${v}_$r.log 2>&1 || { tail -20 $OUT/${v}_$r.log; exit 1; }
    echo "$v ($E) r=$r $(grep -o '"ms_per_step": [0-9.]*' $OUT/${v}_$r.log)"
  done
done
