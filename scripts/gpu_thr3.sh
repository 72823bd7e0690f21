#!/bin/bash
# is the slower transform after a fit the driver process's state or the GPU's?  fit and transform in separate
# driver processes back to back, then both in one process
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-thr3}; mkdir -p $OUT
export TMPDIR=/tmp
step() { local n=$1; shift; echo "== $n"; timeout -k 10 ${T:-300} "$@" > $OUT/$n.log 2>&1; local rc=$?; grep -h '^{' $OUT/$n.log | cut -c1-120; return $rc; }
step fit python -u tools/stream_throughput.py --only fit &&
step tr python -u tools/stream_throughput.py --only transform &&
step both python -u tools/stream_throughput.py
