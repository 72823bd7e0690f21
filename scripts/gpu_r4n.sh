#!/bin/bash
# round-4: the whole GPU tier after the serving-path changes (next batch prefetched during the
# current batch's last chunk, decode packs without the embedding sort, binary result records;
# beam bookkeeping ranked and selected in parallel (ballot prefix counts);
# colsum finish), then decode / stream throughput / latency
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-r4n}; mkdir -p $OUT
export TMPDIR=/tmp
step() { local n=$1; shift; echo "== $n"; timeout -k 10 ${T:-300} "$@" > $OUT/$n.log 2>&1; local rc=$?; tail -${TL:-3} $OUT/$n.log; return $rc; }
T=900 step tier python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread &&
step dec python -u bench_decode.py --batches 10 &&
step thr python -u tools/stream_throughput.py --only transform --out $OUT/stream_thr.jsonl &&
step lat python -u tools/stream_latency.py --requests 60 --waits 0 &&
step bench python -u bench.py
