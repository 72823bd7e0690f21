#!/bin/bash
# round 5: decoder row groups at config #5 batch 2048 (forward / backward loop groups)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5t; mkdir -p $OUT
export TMPDIR=/tmp
C5="--hidden 512 --enc 800 --layers 2 --batch 2048 --steps 5 --warmup 2 --decode-batches 0 --config5-steps 0"
step() { local n=$1; shift; echo "== $n"; timeout -k 10 ${T:-300} "$@" > $OUT/$n.log 2>&1; local rc=$?; grep -o '"ms_per_step": [0-9.]*' $OUT/$n.log; return $rc; }
step s2 python -u bench.py $C5 || exit 1
step s4 env TSAMD_SPLIT=4 python -u bench.py $C5 || exit 1
step s4b2 env TSAMD_SPLIT=4 TSAMD_SPLIT_BWD=2 python -u bench.py $C5 || exit 1
step s2b4 env TSAMD_SPLIT=2 TSAMD_SPLIT_BWD=4 python -u bench.py $C5 || exit 1
step s2r python -u bench.py $C5 || exit 1
echo done
