#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/dec1; mkdir -p $OUT
timeout -k 10 600 python -m pytest tests/test_gpu_decode.py -x -q > $OUT/pytest.log 2>&1; echo "rc=$?"; tail -30 $OUT/pytest.log
