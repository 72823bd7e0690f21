#!/bin/bash
# one GPU iteration: numerics tests, bench, kernel profile.  usage: gpu_iter.sh TAG [BATCH]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-it}; BATCH=${2:-64}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests/test_gpu_model.py -x -q > $OUT/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --batch $BATCH > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -30 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --batch $BATCH --no-graph > $OUT/prof.log 2>&1; echo "prof rc=$?"
