#!/bin/bash
# round 5: HIP runtime launch knobs A/B on the driver-style bench (headline + decode, then config #5)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5x; mkdir -p $OUT
export TMPDIR=/tmp
step() { local n=$1; shift; echo "== $n"; timeout -k 10 ${T:-300} "$@" > $OUT/$n.log 2>&1; local rc=$?; grep -o '"ms_per_step": [0-9.]*\|"beam4_summaries_per_sec": [0-9.]*' $OUT/$n.log | tr '\n' ' '; echo; return $rc; }
step base python -u bench.py --config5-steps 0 || exit 1
step kern env HIP_FORCE_DEV_KERNARG=1 python -u bench.py --config5-steps 0 || exit 1
step base2 python -u bench.py --config5-steps 0 || exit 1
step kern2 env HIP_FORCE_DEV_KERNARG=1 python -u bench.py --config5-steps 0 || exit 1
echo done
