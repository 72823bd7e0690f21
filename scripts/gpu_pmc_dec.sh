#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmcd; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES --kernel-include-regex "vocab" -d $OUT/p1 -o run --output-format csv -- python3 bench_decode.py --batches 1 --warmup 0 --no-graph --articles 64 > $OUT/p1.log 2>&1; echo "p1 rc=$?"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc VALUBusy OccupancyPercent MemUnitStalled SQ_LDS_BANK_CONFLICT --kernel-include-regex "vocab" -d $OUT/p2 -o run --output-format csv -- python3 bench_decode.py --batches 1 --warmup 0 --no-graph --articles 64 > $OUT/p2.log 2>&1; echo "p2 rc=$?"
