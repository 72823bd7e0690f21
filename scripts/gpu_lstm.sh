#!/bin/bash
# Persistent LSTM: correctness vs step kernels, model tests, bench with/without, profile.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/lstm; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_gpu_lstm.py -x -q > $OUT/pytest_lstm.log 2>&1
rc=$?; tail -15 $OUT/pytest_lstm.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -m pytest tests -m gpu -x -q > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for b in 64 256; do
  timeout -k 10 600 python bench.py --batch $b --steps 10 > $OUT/bench_b$b.log 2>&1 || { tail -20 $OUT/bench_b$b.log; exit 1; }
  tail -1 $OUT/bench_b$b.log
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --batch 64 --no-graph > $OUT/prof.log 2>&1; echo "prof rc=$?"
