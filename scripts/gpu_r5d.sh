#!/bin/bash
# round 5: decode kernel stats on the current tree (dot2 scores)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5d; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/dp -o run --output-format csv -- python3 bench_decode.py --batches 3 > $OUT/dec.log 2>&1 || { tail -5 $OUT/dec.log; exit 1; }
tail -2 $OUT/dec.log
python scripts/kstats.py $(ls $OUT/dp/*kernel_stats.csv | head -1) 3 16 > $OUT/decode_kstats.txt; cat $OUT/decode_kstats.txt
rm -rf $OUT/dp
echo done
