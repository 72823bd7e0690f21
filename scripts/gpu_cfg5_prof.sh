#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-cfg5p}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --hidden 512 --layers 2 --enc 800 --batch auto --steps 3 --warmup 1 --decode-batches 0 > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
python scripts/kstats.py $OUT/prof/run_kernel_stats.csv 5 40 > $OUT/kstats.txt
tail -1 $OUT/prof.log
