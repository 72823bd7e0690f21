#!/bin/bash
# round-4: production-shape oracle tests (compacted vocab head, 4-phase DP buckets), decode vocab
# head numerics + timing, train + decode bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-r4b}; mkdir -p $OUT
export TMPDIR=/tmp
step() { local n=$1; shift; echo "== $n"; timeout -k 10 ${T:-300} "$@" > $OUT/$n.log 2>&1; local rc=$?; tail -${TL:-3} $OUT/$n.log; return $rc; }
step prod python -u -m pytest tests/test_gpu_production.py tests/test_gpu_dist.py -x -q --timeout 200 --timeout-method thread &&
step vtest python -u -m pytest tests/test_gpu_decode.py -x -q --timeout 100 --timeout-method thread -k "vocab_topk or fused_decode" &&
step bench python -u bench.py --config5-steps 0 &&
T=400 step vprof rocprofv3 --kernel-trace --stats -d $OUT/v -o run --output-format csv -- python3 tools/vocab_micro.py &&
python scripts/kstats.py $OUT/v/run_kernel_stats.csv 1 4 &&
step dec_fused python -u bench_decode.py --batches 10 &&
step dec_unfused python -u bench_decode.py --batches 10 --unfused-step &&
step thr python -u tools/stream_throughput.py --out $OUT/stream_thr.jsonl &&
step lat python -u tools/stream_latency.py --requests 60 --waits 0
