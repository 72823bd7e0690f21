#!/bin/bash
# decode with / without the XCD-aware attn_score order (10 timed batches + kernel stats)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-score2}; mkdir -p $OUT
export TMPDIR=/tmp
for x in 1 0; do
  TSAMD_SCORE_XCD=$x timeout -k 10 300 python bench_decode.py --batches 10 > $OUT/dec$x.log 2>&1 || { tail -20 $OUT/dec$x.log; exit 1; }
  echo "xcd=$x $(tail -1 $OUT/dec$x.log | cut -c1-120)"
  TSAMD_SCORE_XCD=$x timeout -k 10 300 python bench_decode.py --articles 128 --batches 10 > $OUT/dec128_$x.log 2>&1 || { tail -20 $OUT/dec128_$x.log; exit 1; }
  echo "xcd=$x a128 $(tail -1 $OUT/dec128_$x.log | cut -c1-120)"
done
TSAMD_SCORE_XCD=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/p1 -o run --output-format csv -- python3 bench_decode.py --batches 2 > $OUT/p1.log 2>&1 || { tail -20 $OUT/p1.log; exit 1; }
python scripts/kstats.py $OUT/p1/run_kernel_stats.csv 3 6
