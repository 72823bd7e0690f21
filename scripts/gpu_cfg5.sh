#!/bin/bash
# Config #5 measurements on one MI355X: bench at batch 1024 and 2048 (phase times in the JSON),
# a rocprofv3 kernel-stats profile at batch 1024, and the default B=256 bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${OUTD:-cfg5}; mkdir -p $OUT
C5="--hidden 512 --layers 2 --enc 800 --decode-batches 0"
timeout -k 10 400 python bench.py $C5 --batch 1024 --steps 5 --warmup 2 > $OUT/b1024.log 2>&1 || { tail -20 $OUT/b1024.log; exit 1; }
tail -1 $OUT/b1024.log | cut -c1-900
timeout -k 10 500 python bench.py $C5 --batch 2048 --steps 4 --warmup 2 > $OUT/b2048.log 2>&1 || { tail -20 $OUT/b2048.log; exit 1; }
tail -1 $OUT/b2048.log | cut -c1-900
if [ -n "$PROF" ]; then
  timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py $C5 --batch 1024 --steps 2 --warmup 1 > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
  python scripts/kstats.py $(find $OUT/prof -name '*kernel_stats.csv' | head -1) 8 30 > $OUT/kstats.txt && head -40 $OUT/kstats.txt
fi
timeout -k 10 300 python bench.py > $OUT/b256.log 2>&1 || { tail -20 $OUT/b256.log; exit 1; }
tail -1 $OUT/b256.log | cut -c1-700
echo done
