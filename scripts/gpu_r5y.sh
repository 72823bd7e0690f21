#!/bin/bash
# round 5: headline step (B = 256) by phase, by kernel and by idle gap on the current tree
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5y; mkdir -p $OUT
export TMPDIR=/tmp
step() { local n=$1; shift; echo "== $n"; timeout -k 10 ${T:-300} "$@" > $OUT/$n.log 2>&1; local rc=$?; tail -${TL:-2} $OUT/$n.log; return $rc; }
T=300 step ph python -u tools/phase_micro.py --iters 5 || exit 1
T=400 step tr rocprofv3 --kernel-trace -d $OUT/tr -o run --output-format csv -- python3 bench.py --steps 5 --warmup 3 --decode-batches 0 --config5-steps 0 || exit 1
python scripts/kwin.py $OUT/tr/run_kernel_trace.csv 4 45 adagrad_kernel 3 > $OUT/kwin_b256.txt; head -3 $OUT/kwin_b256.txt
python scripts/kgaps.py $OUT/tr/run_kernel_trace.csv 4 30 adagrad_kernel 3 > $OUT/gaps_b256.txt 2>&1; head -1 $OUT/gaps_b256.txt; grep -A16 "^idle" $OUT/gaps_b256.txt
rm -rf $OUT/tr
echo done
