#!/bin/bash
# round-4 iteration: decode attention kernel numerics + timing, decode tests, streaming throughput
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-r4}; mkdir -p $OUT
export TMPDIR=/tmp
step() { local n=$1; shift; echo "== $n"; timeout -k 10 ${T:-300} "$@" > $OUT/$n.log 2>&1; local rc=$?; tail -${TL:-3} $OUT/$n.log; return $rc; }
step attn_test python -u -m pytest tests/test_gpu_attention_ops.py -x -q --timeout 120 --timeout-method thread -k "beam or fwd_row" &&
step attn_micro python -u tools/decode_kernels_micro.py &&
step vocab_micro python -u tools/vocab_micro.py &&
step dec_test python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_decode_parity.py -x -q --timeout 200 --timeout-method thread &&
step bench_dec python -u bench_decode.py &&
step thr python -u tools/stream_throughput.py --only transform --out $OUT/stream_thr.jsonl &&
step lat python -u tools/stream_latency.py --requests 60 --waits 0 &&
step pipe python -u -m pytest tests/test_gpu_pipeline.py -x -q --timeout 200 --timeout-method thread
