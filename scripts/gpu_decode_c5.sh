#!/bin/bash
# Config #5 decode alone (bench_decode.py --hidden 512 --layers 2 --enc 800): throughput and kernel stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-dc5}; mkdir -p $OUT
export TMPDIR=/tmp
C5="--hidden 512 --layers 2 --enc 800"
timeout -k 10 300 python bench_decode.py $C5 --batches 6 > $OUT/bd.log 2>&1 || { tail -20 $OUT/bd.log; exit 1; }
tail -1 $OUT/bd.log | cut -c1-300
timeout -k 10 300 python bench_decode.py $C5 --batches 6 --no-pipeline > $OUT/bd_np.log 2>&1 || { tail -20 $OUT/bd_np.log; exit 1; }
tail -1 $OUT/bd_np.log | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/p -o run --output-format csv -- python3 bench_decode.py $C5 --batches 2 > $OUT/p.log 2>&1 || { tail -20 $OUT/p.log; exit 1; }
python scripts/kstats.py $OUT/p/run_kernel_stats.csv 3 16 > $OUT/decode_c5_kstats.txt; head -18 $OUT/decode_c5_kstats.txt
rm -rf $OUT/p/*trace*
echo done
