#!/bin/bash
# round 6: headline kernel windows + overlap (kgaps) with TSAMD_VOCAB_PAD=1 and 0
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-r6w}; mkdir -p $OUT
export TMPDIR=/tmp
for pad in 1 0; do
  TSAMD_VOCAB_PAD=$pad timeout -k 10 400 rocprofv3 --kernel-trace -d $OUT/t$pad -o run --output-format csv -- python3 bench.py --steps 6 --warmup 3 --decode-batches 0 --config5-steps 0 > $OUT/b256_pad$pad.log 2>&1 || exit 1
  python scripts/kwin.py $OUT/t$pad/run_kernel_trace.csv 4 45 adagrad_kernel 3 > $OUT/kwin_pad$pad.txt && python scripts/kgaps.py $OUT/t$pad/run_kernel_trace.csv 4 30 adagrad_kernel 3 > $OUT/gaps_pad$pad.txt
  head -1 $OUT/kwin_pad$pad.txt; grep -i "vocab_train\|cijk\|gemm_bt" $OUT/gaps_pad$pad.txt | cut -c1-120
  rm -rf $OUT/t$pad
done
echo done
