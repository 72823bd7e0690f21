#!/bin/bash
# one GPU iteration: numerics tests, bench (batch sweep), kernel profile.
# usage: gpu_iter.sh TAG PROF_BATCH [BENCH_BATCHES...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-it}; PB=${2:-64}; shift 2; BATCHES=${@:-64}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests/ -m gpu -x -q > $OUT/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for b in $BATCHES; do
  timeout -k 10 600 python bench.py --steps 10 --warmup 3 --batch $b > $OUT/bench_b$b.log 2>&1 || { echo "bench b=$b failed"; tail -30 $OUT/bench_b$b.log; exit 1; }
  tail -1 $OUT/bench_b$b.log
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --batch $PB --no-graph > $OUT/prof.log 2>&1; echo "prof rc=$?"
