#!/bin/bash
# round 6, final tree: kernel windows (timed steps; the 3 phase-timed diagnostic steps skipped) and idle gaps
# of the headline step and of config #5 at batch 2048, plus the decode kernel stats
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-r6kw}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d $OUT/t1 -o run --output-format csv -- python3 bench.py --steps 6 --warmup 3 --decode-batches 0 --config5-steps 0 > $OUT/b256.log 2>&1 || exit 1
python scripts/kwin.py $OUT/t1/run_kernel_trace.csv 4 45 adagrad_kernel 3 > $OUT/train_kwin_b256.txt && python scripts/kgaps.py $OUT/t1/run_kernel_trace.csv 4 30 adagrad_kernel 3 > $OUT/train_gaps_b256.txt && head -2 $OUT/train_kwin_b256.txt
rm -rf $OUT/t1
timeout -k 10 600 rocprofv3 --kernel-trace -d $OUT/t2 -o run --output-format csv -- python3 bench.py --hidden 512 --enc 800 --layers 2 --batch 2048 --steps 3 --warmup 2 --decode-batches 0 --config5-steps 0 > $OUT/c5.log 2>&1 || exit 1
python scripts/kwin.py $OUT/t2/run_kernel_trace.csv 2 45 adagrad_kernel 3 > $OUT/cfg5_kwin_b2048.txt && python scripts/kgaps.py $OUT/t2/run_kernel_trace.csv 2 30 adagrad_kernel 3 > $OUT/cfg5_gaps_b2048.txt && head -2 $OUT/cfg5_kwin_b2048.txt
rm -rf $OUT/t2
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/dp -o run --output-format csv -- python3 bench_decode.py --batches 3 > $OUT/dec.log 2>&1 || exit 1
python scripts/kstats.py $(ls $OUT/dp/*kernel_stats.csv | head -1) 3 16 > $OUT/decode_kstats.txt; head -4 $OUT/decode_kstats.txt
rm -rf $OUT/dp
echo done
