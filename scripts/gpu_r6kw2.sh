#!/bin/bash
# round 6: config #5 kernel window + gaps on the current tree
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-r6kw2}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace -d $OUT/t2 -o run --output-format csv -- python3 bench.py --hidden 512 --enc 800 --layers 2 --batch 2048 --steps 3 --warmup 2 --decode-batches 0 --config5-steps 0 > $OUT/c5.log 2>&1 || exit 1
python scripts/kwin.py $OUT/t2/run_kernel_trace.csv 2 60 adagrad_kernel 3 > $OUT/cfg5_kwin_b2048.txt && python scripts/kgaps.py $OUT/t2/run_kernel_trace.csv 2 40 adagrad_kernel 3 > $OUT/cfg5_gaps_b2048.txt && head -2 $OUT/cfg5_kwin_b2048.txt
rm -rf $OUT/t2
echo done
