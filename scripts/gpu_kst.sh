#!/bin/bash
# train-step kernel stats (B=256) + bench at 50 steps
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-kst}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 4 --warmup 1 > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
python scripts/kstats.py $OUT/prof/run_kernel_stats.csv 7 40 > $OUT/train_kstats.txt
head -12 $OUT/train_kstats.txt | cut -c1-110
timeout -k 10 300 python bench.py --steps 50 > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | cut -c1-200
