#!/bin/bash
# round-4: per-kernel profiles of the final defaults (train B = 256, beam-4 decode), then the stream
# paths with the restored decode vocab head
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-r4l}; mkdir -p $OUT
export TMPDIR=/tmp
step() { local n=$1; shift; echo "== $n"; timeout -k 10 ${T:-300} "$@" > $OUT/$n.log 2>&1; local rc=$?; tail -${TL:-3} $OUT/$n.log; return $rc; }
step tprof rocprofv3 --kernel-trace --stats -d $OUT/t -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --decode-batches 0 --config5-steps 0 &&
python scripts/kstats.py $OUT/t/run_kernel_stats.csv 13 40 > $OUT/train_kstats.txt &&
step dprof rocprofv3 --kernel-trace --stats -d $OUT/d -o run --output-format csv -- python3 bench_decode.py --batches 5 &&
python scripts/kstats.py $OUT/d/run_kernel_stats.csv 6 30 > $OUT/decode_kstats.txt &&
step thr python -u tools/stream_throughput.py --out $OUT/stream_thr.jsonl &&
step lat python -u tools/stream_latency.py --requests 60 --waits 0
