#!/bin/bash
# round 5: headline bench x2 + phases + kernel window after the attn_bwd_rowp spill fix (the tests
# of gpu_r5l are in the closing tier), then the closing run (gpu_r5final).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5l; mkdir -p $OUT
export TMPDIR=/tmp
step() { local n=$1; shift; echo "== $n"; timeout -k 10 ${T:-300} "$@" > $OUT/$n.log 2>&1; local rc=$?; tail -${TL:-3} $OUT/$n.log; return $rc; }
T=400 TL=1 step b1 python -u bench.py --steps 20 --warmup 3 --decode-batches 0 --config5-steps 0 || exit 1
TL=2 step ph python -u tools/phase_micro.py || exit 1
T=400 step tr rocprofv3 --kernel-trace -d $OUT/tr -o run --output-format csv -- python3 bench.py --steps 3 --warmup 2 --decode-batches 0 --config5-steps 0 || exit 1
python scripts/kwin.py $OUT/tr/run_kernel_trace.csv 3 40 > $OUT/train_kwin_b256.txt; head -4 $OUT/train_kwin_b256.txt
rm -rf $OUT/tr
bash scripts/gpu_r5final.sh
