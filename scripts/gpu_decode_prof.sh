#!/bin/bash
# Decode kernel stats: beam-4, 64 articles at hidden 256 (bench_decode.py) and config #5's decode
# (bench.py --hidden 512 --layers 2 --enc 800, decode only).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-dprof}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python bench_decode.py --batches 4 > $OUT/bd.log 2>&1 || { tail -20 $OUT/bd.log; exit 1; }
tail -1 $OUT/bd.log | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/p1 -o run --output-format csv -- python3 bench_decode.py --batches 2 > $OUT/p1.log 2>&1 || { tail -20 $OUT/p1.log; exit 1; }
python scripts/kstats.py $OUT/p1/run_kernel_stats.csv 3 16 > $OUT/decode_h256_kstats.txt; head -18 $OUT/decode_h256_kstats.txt
timeout -k 10 400 python bench.py --hidden 512 --layers 2 --enc 800 --batch 64 --steps 1 --warmup 1 --decode-batches 4 > $OUT/c5d.log 2>&1 || { tail -20 $OUT/c5d.log; exit 1; }
tail -1 $OUT/c5d.log | cut -c1-400
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/p2 -o run --output-format csv -- python3 bench.py --hidden 512 --layers 2 --enc 800 --batch 64 --steps 1 --warmup 1 --decode-batches 2 > $OUT/p2.log 2>&1 || { tail -20 $OUT/p2.log; exit 1; }
python scripts/kstats.py $OUT/p2/run_kernel_stats.csv 1 24 > $OUT/decode_c5_kstats.txt; head -26 $OUT/decode_c5_kstats.txt
rm -rf $OUT/p1/*trace* $OUT/p2/*trace*
echo done
