#!/bin/bash
# config #5 kernel profile (bench.py's config5 part only: 2 warm-up + 5 timed steps at batch 1024)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-c5p}; mkdir -p $OUT
export TMPDIR=/tmp
step() { local n=$1; shift; echo "== $n"; timeout -k 10 ${T:-300} "$@" > $OUT/$n.log 2>&1; local rc=$?; tail -${TL:-3} $OUT/$n.log; return $rc; }
T=600 step c5prof rocprofv3 --kernel-trace --stats -d $OUT/c -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --decode-batches 0 --config5-steps 5 &&
python scripts/kstats.py $OUT/c/run_kernel_stats.csv 7 40 > $OUT/cfg5_kstats.txt
