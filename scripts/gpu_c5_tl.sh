#!/bin/bash
# Config #5: bench at batch 1024 / 2048 and a kernel-trace timeline of the batch-1024 step.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-c5tl}; mkdir -p $OUT
export TMPDIR=/tmp
C5="--hidden 512 --layers 2 --enc 800"
timeout -k 10 400 python bench.py $C5 --batch 2048 --steps 3 --warmup 1 --decode-batches 0 > $OUT/b2048.log 2>&1 || { tail -20 $OUT/b2048.log; exit 1; }
tail -1 $OUT/b2048.log | cut -c1-200
timeout -k 10 400 python tools/phase_micro.py --hidden 512 --layers 2 --enc 800 --batch 1024 --iters 2 > $OUT/phase.log 2>&1 || { tail -20 $OUT/phase.log; exit 1; }
tail -1 $OUT/phase.log
timeout -k 10 400 rocprofv3 --kernel-trace -d $OUT/tr -o run --output-format csv -- python3 bench.py $C5 --batch 1024 --steps 1 --warmup 1 --decode-batches 0 > $OUT/tr.log 2>&1 || { tail -20 $OUT/tr.log; exit 1; }
python tools/timeline.py $OUT/tr/run_kernel_trace.csv 40 > $OUT/timeline.txt; head -45 $OUT/timeline.txt
rm -rf $OUT/tr
echo done
