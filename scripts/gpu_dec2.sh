#!/bin/bash
# Decode tests + beam-4 throughput at 64/128 articles + kernel profile (eager, 1 batch).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/dec2; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_decode.py -x -q > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python bench_decode.py > $OUT/d64.log 2>&1 || { echo fail; tail -20 $OUT/d64.log; exit 1; }
tail -1 $OUT/d64.log
timeout -k 10 600 python bench_decode.py --articles 128 > $OUT/d128.log 2>&1 || exit 1
tail -1 $OUT/d128.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench_decode.py --batches 1 --warmup 1 --no-graph > $OUT/prof.log 2>&1; echo "prof rc=$?"
