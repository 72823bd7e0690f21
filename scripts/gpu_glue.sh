#!/bin/bash
# glue fusions: GPU tier (incl. frames kernels), train bench (50 steps), decode bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-glue}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python bench.py --steps 50 > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | cut -c1-200
timeout -k 10 300 python bench_decode.py --batches 10 > $OUT/dec64.log 2>&1 || { tail -20 $OUT/dec64.log; exit 1; }
tail -1 $OUT/dec64.log | cut -c1-200
