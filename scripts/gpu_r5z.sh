#!/bin/bash
# round 5: driver-style bench on the current tree (twice), config #5 steady state
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5z; mkdir -p $OUT
export TMPDIR=/tmp
step() { local n=$1; shift; echo "== $n"; timeout -k 10 ${T:-300} "$@" > $OUT/$n.log 2>&1; local rc=$?; tail -${TL:-1} $OUT/$n.log | cut -c1-400; return $rc; }
T=600 step bench python -u bench.py || exit 1
T=600 step bench2 python -u bench.py || exit 1
grep -o '"ms_per_step": [0-9.]*\|"beam4_summaries_per_sec": [0-9.]*\|"config5_tokens_per_sec": [0-9.]*\|"config5_ms_per_step": [0-9.]*\|"config5_beam4_summaries_per_sec": [0-9.]*' $OUT/bench.log $OUT/bench2.log
echo done
