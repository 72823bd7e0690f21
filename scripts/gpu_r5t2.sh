#!/bin/bash
# round 5: decoder row groups at config #5, second pass (8 groups; batch 1024)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5t2; mkdir -p $OUT
export TMPDIR=/tmp
C5="--hidden 512 --enc 800 --layers 2 --steps 5 --warmup 2 --decode-batches 0 --config5-steps 0"
step() { local n=$1; shift; echo "== $n"; timeout -k 10 ${T:-300} "$@" > $OUT/$n.log 2>&1; local rc=$?; grep -o '"ms_per_step": [0-9.]*' $OUT/$n.log; return $rc; }
step s4 env TSAMD_SPLIT=4 python -u bench.py $C5 --batch 2048 || exit 1
step s8 env TSAMD_SPLIT=8 python -u bench.py $C5 --batch 2048 || exit 1
step s8b4 env TSAMD_SPLIT=8 TSAMD_SPLIT_BWD=4 python -u bench.py $C5 --batch 2048 || exit 1
step s2 python -u bench.py $C5 --batch 2048 || exit 1
step k2 python -u bench.py $C5 --batch 1024 || exit 1
step k4 env TSAMD_SPLIT=4 python -u bench.py $C5 --batch 1024 || exit 1
echo done
