#!/bin/bash
# Iteration check on one MI355X: GPU test tier, default bench (train + beam-4 decode),
# 2-rank self-launched bench (gloo, both ranks on the one GPU: plumbing only).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-check}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $OUT/pytest.log 2>&1
rc=$?; tail -4 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
timeout -k 10 300 python bench.py --gpus 2 --backend gloo --batch 64 --steps 5 --warmup 2 --decode-batches 2 > $OUT/dp2.log 2>&1 || { tail -20 $OUT/dp2.log; exit 1; }
tail -1 $OUT/dp2.log | cut -c1-400
echo done
