#!/bin/bash
# round 5: config #5 (batch 2048) kernel windows of the TIMED steps (bench.py's last 3 steps are
# the phase-timed diagnostics, which synchronise every step: skipped) -- kernels and idle gaps
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5v; mkdir -p $OUT
export TMPDIR=/tmp
T=600; echo "== c5tr"
timeout -k 10 $T rocprofv3 --kernel-trace -d $OUT/tr -o run --output-format csv -- python3 bench.py --hidden 512 --enc 800 --layers 2 --batch 2048 --steps 3 --warmup 2 --decode-batches 0 --config5-steps 0 > $OUT/c5tr.log 2>&1 || exit 1
grep -o '"ms_per_step": [0-9.]*' $OUT/c5tr.log
python scripts/kwin.py $OUT/tr/run_kernel_trace.csv 2 45 adagrad_kernel 3 > $OUT/cfg5_kwin.txt; head -3 $OUT/cfg5_kwin.txt
python scripts/kgaps.py $OUT/tr/run_kernel_trace.csv 2 30 adagrad_kernel 3 > $OUT/cfg5_gaps.txt 2>&1; head -1 $OUT/cfg5_gaps.txt; grep -A12 "^idle" $OUT/cfg5_gaps.txt
rm -rf $OUT/tr
echo done
