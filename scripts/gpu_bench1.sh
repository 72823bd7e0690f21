#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests/test_gpu_model.py -x -q > gpurun_out/b1_pytest.log 2>&1; echo "pytest rc=$?"; tail -3 gpurun_out/b1_pytest.log
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --batch 64 > gpurun_out/b1_bench64.log 2>&1 || { echo "bench failed rc=$?"; tail -30 gpurun_out/b1_bench64.log; exit 1; }
cat gpurun_out/b1_bench64.log
timeout -k 10 600 python bench.py --steps 5 --warmup 2 --batch 64 --no-graph > gpurun_out/b1_bench64_nograph.log 2>&1; echo "nograph rc=$?"; tail -2 gpurun_out/b1_bench64_nograph.log
