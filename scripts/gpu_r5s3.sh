#!/bin/bash
# round 5: headline bench, backward loop in 4 row groups (TSAMD_SPLIT_BWD=4) vs the default 2
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5s3; mkdir -p $OUT
export TMPDIR=/tmp
step() { local n=$1; shift; echo "== $n"; timeout -k 10 ${T:-300} "$@" > $OUT/$n.log 2>&1; local rc=$?; grep -o '"ms_per_step": [0-9.]*' $OUT/$n.log | head -1; return $rc; }
for r in 1 2 3; do
step d$r python -u bench.py --decode-batches 0 --config5-steps 0 || exit 1
step b$r env TSAMD_SPLIT_BWD=4 python -u bench.py --decode-batches 0 --config5-steps 0 || exit 1
done
echo done
