#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof1
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof1 -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --batch 64 --no-graph > gpurun_out/prof1/bench.log 2>&1; echo "prof rc=$?"
tail -3 gpurun_out/prof1/bench.log
find gpurun_out/prof1 -name "*stats*" | head
