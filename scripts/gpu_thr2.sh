#!/bin/bash
# stream transform right after a stream fit in the same tool process, twice, then transform alone
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-thr2}; mkdir -p $OUT
export TMPDIR=/tmp
step() { local n=$1; shift; echo "== $n"; timeout -k 10 ${T:-300} "$@" > $OUT/$n.log 2>&1; local rc=$?; grep -h '^{' $OUT/$n.log | cut -c1-200; return $rc; }
step both1 python -u tools/stream_throughput.py &&
step both2 python -u tools/stream_throughput.py &&
step tonly python -u tools/stream_throughput.py --only transform
