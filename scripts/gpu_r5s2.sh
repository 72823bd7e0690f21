#!/bin/bash
# round 5: decoder row groups at the headline shape on the current tree (phase times + bench)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5s2; mkdir -p $OUT
export TMPDIR=/tmp
step() { local n=$1; shift; echo "== $n"; timeout -k 10 ${T:-300} "$@" > $OUT/$n.log 2>&1; local rc=$?; tail -1 $OUT/$n.log | cut -c1-260; return $rc; }
step ph2 python -u tools/phase_micro.py --iters 5 || exit 1
step ph1 env TSAMD_SPLIT=1 python -u tools/phase_micro.py --iters 5 || exit 1
step ph4 env TSAMD_SPLIT=4 python -u tools/phase_micro.py --iters 5 || exit 1
echo done
