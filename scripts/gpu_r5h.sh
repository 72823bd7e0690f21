#!/bin/bash
# round 5: A/B of the tr01 / in-kernel bf16 a glue removal at config #5 (TSAMD_TR01_AB=0: the torch passes)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5h; mkdir -p $OUT
export TMPDIR=/tmp
C5="--hidden 512 --enc 800 --layers 2 --batch 2048 --steps 10 --warmup 2 --decode-batches 0 --config5-steps 0"
step() { local n=$1; shift; echo "== $n"; timeout -k 10 ${T:-300} "$@" > $OUT/$n.log 2>&1; local rc=$?; grep -o '"ms_per_step": [0-9.]*' $OUT/$n.log; return $rc; }
step new1 python -u bench.py $C5 || exit 1
step old1 env TSAMD_TR01_AB=0 python -u bench.py $C5 || exit 1
step new2 python -u bench.py $C5 || exit 1
step old2 env TSAMD_TR01_AB=0 python -u bench.py $C5 || exit 1
echo done
