#!/bin/bash
# decode kernel stats with trained (80 steps) vs random-init weights
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-dtp}; mkdir -p $OUT
export TMPDIR=/tmp
step() { local n=$1; shift; echo "== $n"; timeout -k 10 ${T:-300} "$@" > $OUT/$n.log 2>&1; local rc=$?; grep -h '^{' $OUT/$n.log | cut -c1-300; return $rc; }
step tr rocprofv3 --kernel-trace --stats -d $OUT/tr -o run --output-format csv -- python3 tools/decode_trained_prof.py --train-steps 80 &&
step rnd rocprofv3 --kernel-trace --stats -d $OUT/rnd -o run --output-format csv -- python3 tools/decode_trained_prof.py --train-steps 0
&& python scripts/kstats.py $OUT/tr/run_kernel_stats.csv 1 30 > $OUT/tr_kstats.txt && python scripts/kstats.py $OUT/rnd/run_kernel_stats.csv 1 30 > $OUT/rnd_kstats.txt
