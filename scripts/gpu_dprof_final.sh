#!/bin/bash
# closing decode kernel stats: random init (bench_decode) and an 80-step trained checkpoint
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-dpf}; mkdir -p $OUT
export TMPDIR=/tmp
step() { local n=$1; shift; echo "== $n"; timeout -k 10 ${T:-300} "$@" > $OUT/$n.log 2>&1; local rc=$?; grep -h '^{' $OUT/$n.log | cut -c1-200; return $rc; }
step drnd rocprofv3 --kernel-trace --stats -d $OUT/r -o run --output-format csv -- python3 bench_decode.py --batches 5 &&
python scripts/kstats.py $OUT/r/run_kernel_stats.csv 6 30 > $OUT/decode_kstats.txt &&
step dtr rocprofv3 --kernel-trace --stats -d $OUT/t -o run --output-format csv -- python3 tools/decode_trained_prof.py --train-steps 80 --batches 6 &&
python scripts/kstats.py $OUT/t/run_kernel_stats.csv 7 40 > $OUT/decode_trained_kstats.txt
