#!/bin/bash
# Decode tests, decode bench, vocab-head micro-benchmark (+ rocprof split).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-dec5}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests/test_gpu_decode.py tests/test_gpu_pipeline.py -x -q > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/vocab_micro.py > $OUT/micro.log 2>&1 && tail -1 $OUT/micro.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/mprof -o run --output-format csv -- python3 tools/vocab_micro.py --iters 20 > $OUT/mprof.log 2>&1; echo "mprof rc=$?"
timeout -k 10 600 python bench_decode.py > $OUT/d64.log 2>&1 || { tail -20 $OUT/d64.log; exit 1; }
echo "64: $(grep -o '"value": [0-9.]*' $OUT/d64.log) $(grep -o '"ms_per_batch": [0-9.]*' $OUT/d64.log)"
timeout -k 10 600 python bench_decode.py --articles 128 > $OUT/d128.log 2>&1 && echo "128: $(grep -o '"value": [0-9.]*' $OUT/d128.log)"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench_decode.py --batches 1 --warmup 1 --no-graph > $OUT/prof.log 2>&1; echo "prof rc=$?"
