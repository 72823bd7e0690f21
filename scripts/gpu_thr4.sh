#!/bin/bash
# stream fit + transform (the fit's trained checkpoint served) and transform alone (random init), each with the
# decoder-alone rate on the same checkpoint
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-thr4}; mkdir -p $OUT
export TMPDIR=/tmp
step() { local n=$1; shift; echo "== $n"; timeout -k 10 ${T:-300} "$@" > $OUT/$n.log 2>&1; local rc=$?; grep -h '^{' $OUT/$n.log | cut -c1-400; return $rc; }
step both python -u tools/stream_throughput.py --out $OUT/thr.jsonl &&
step tonly python -u tools/stream_throughput.py --only transform --out $OUT/thr.jsonl
