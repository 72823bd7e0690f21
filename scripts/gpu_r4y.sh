#!/bin/bash
# round-4 closing check with blt_mm: the whole GPU tier, smoke(), bench.py, bench_decode, stream-fed fit and
# transform throughput at the full shape, request latency
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-r4y}; mkdir -p $OUT
export TMPDIR=/tmp
step() { local n=$1; shift; echo "== $n"; timeout -k 10 ${T:-300} "$@" > $OUT/$n.log 2>&1; local rc=$?; tail -${TL:-3} $OUT/$n.log; return $rc; }
T=900 step tier python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread &&
step smoke python -u -c "import __graft_entry__ as g; g.smoke()" &&
T=600 step bench python -u bench.py &&
step dec python -u bench_decode.py --batches 10 &&
T=600 step thr python -u tools/stream_throughput.py --out $OUT/stream_thr.jsonl &&
step lat python -u tools/stream_latency.py --requests 60 --waits 0
