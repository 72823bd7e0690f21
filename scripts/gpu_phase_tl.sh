#!/bin/bash
# Phase wall times (proj on / off) and a kernel-trace timeline of the B=256 step.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-ptl}; mkdir -p $OUT
export TMPDIR=/tmp
for p in 1 0; do
  timeout -k 10 300 env TSAMD_PROJ_ATTN=$p python tools/phase_micro.py ${PHASE_ARGS} > $OUT/phase_p$p.log 2>&1 || { tail -20 $OUT/phase_p$p.log; exit 1; }
  echo "proj=$p $(tail -1 $OUT/phase_p$p.log)"
done
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/tr -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --decode-batches 0 ${BENCH_ARGS} > $OUT/tr.log 2>&1 || { tail -20 $OUT/tr.log; exit 1; }
python tools/timeline.py $OUT/tr/run_kernel_trace.csv 30 > $OUT/timeline.txt; head -40 $OUT/timeline.txt
rm -rf $OUT/tr
echo done
