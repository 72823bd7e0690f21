#!/bin/bash
# round-4: the whole GPU tier (deterministic mode over decoder row groups, fork-safe loaders),
# per-phase step breakdown at the bench shape and config #5, then the bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-r4h}; mkdir -p $OUT
export TMPDIR=/tmp
step() { local n=$1; shift; echo "== $n"; timeout -k 10 ${T:-300} "$@" > $OUT/$n.log 2>&1; local rc=$?; tail -${TL:-3} $OUT/$n.log; return $rc; }
T=900 step tier python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread; rc=$?
# test failures (pytest exit 1) still let the measurements run; a fault, abort or timeout does not
[ $rc -le 1 ] &&
step ph256 python -u tools/phase_micro.py &&
step ph5 python -u tools/phase_micro.py --batch 1024 --hidden 512 --enc 800 --layers 2 --iters 3 &&
T=600 step bench python -u bench.py
