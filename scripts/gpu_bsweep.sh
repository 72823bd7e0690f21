#!/bin/bash
# Batch sweep of the headline bench + B=256 profile.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/bsweep; mkdir -p $OUT
export TMPDIR=/tmp
for b in 128 256 384 512; do
  timeout -k 10 400 python bench.py --batch $b --steps 10 > $OUT/b$b.log 2>&1 || { tail -20 $OUT/b$b.log; exit 1; }
  echo "b=$b $(grep -o '"ms_per_step": [0-9.]*' $OUT/b$b.log) $(grep -o '"value": [0-9.]*' $OUT/b$b.log)"
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --batch 256 --no-graph > $OUT/prof.log 2>&1; echo "prof rc=$?"
