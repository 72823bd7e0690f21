#!/bin/bash
# round-4 A/B: non-temporal logits stores in the decode vocab head (TSAMD_VL_NTS)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-r4r}; mkdir -p $OUT
export TMPDIR=/tmp
step() { local n=$1; shift; echo "== $n"; timeout -k 10 ${T:-300} "$@" > $OUT/$n.log 2>&1; local rc=$?; tail -${TL:-3} $OUT/$n.log; return $rc; }
for v in 0 1 0 1; do
  TSAMD_VL_NTS=$v T=120 step vl$v rocprofv3 --kernel-trace --stats -d $OUT/v$v -o run --output-format csv -- python3 tools/vocab_micro.py || exit 1
  python scripts/kstats.py $OUT/v$v/run_kernel_stats.csv 1 3 | sed -n 2,3p
done
step d0 python -u bench_decode.py --batches 10 &&
TSAMD_VL_NTS=1 step d1 python -u bench_decode.py --batches 10 &&
step d0b python -u bench_decode.py --batches 10 &&
TSAMD_VL_NTS=1 step d1b python -u bench_decode.py --batches 10
