#!/bin/bash
# PMC counters for the hand-written kernels (B=64 train step, eager).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmc; mkdir -p $OUT
export TMPDIR=/tmp
B=${1:-64}
timeout -k 10 600 rocprofv3 --kernel-trace --pmc VALUBusy VALUUtilization MemUnitStalled OccupancyPercent --kernel-include-regex "attn|lstm|dec_|ptr_loss|linear2" -d $OUT/p1 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --batch $B --no-graph > $OUT/p1.log 2>&1; echo "p1 rc=$?"
timeout -k 10 600 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VMEM SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES --kernel-include-regex "attn|lstm|dec_|ptr_loss|linear2" -d $OUT/p2 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --batch $B --no-graph > $OUT/p2.log 2>&1; echo "p2 rc=$?"
timeout -k 10 600 rocprofv3 --kernel-trace --pmc FETCH_SIZE WRITE_SIZE --kernel-include-regex "attn|lstm|dec_|ptr_loss|linear2" -d $OUT/p3 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --batch $B --no-graph > $OUT/p3.log 2>&1; echo "p3 rc=$?"
ls -R $OUT | head -30
