#!/bin/bash
# Kernel trace of the bench's training step (ordered per-dispatch view of the last step) and
# kernel stats of bench.py at the default config (train + decode).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-trace}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --decode-batches 2 ${BENCH_ARGS} > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
tail -1 $OUT/prof.log | cut -c1-300
python scripts/kstats.py $OUT/prof/run_kernel_stats.csv 1 45 > $OUT/kstats_all.txt
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/tr -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --decode-batches 0 ${BENCH_ARGS} > $OUT/tr.log 2>&1 || { tail -20 $OUT/tr.log; exit 1; }
python scripts/ktrace.py $OUT/tr/run_kernel_trace.csv > $OUT/ktrace.txt; head -3 $OUT/ktrace.txt
echo traced
