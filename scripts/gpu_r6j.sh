#!/bin/bash
# round 6: wgrad_tt (deterministic split-K TN GEMM) -- tests then micro at the encoder shapes
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-r6j}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/wgrad_tt_micro.py $MICRO_ARGS > $OUT/micro.jsonl 2>&1; rc=$?; cat $OUT/micro.jsonl | cut -c1-400; [ $rc -eq 0 ] || exit $rc
echo done
