#!/bin/bash
# PMC counters of the attention kernels at the B=256 bench shape (tools/attn_micro.py).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmc_attn; mkdir -p $OUT
export TMPDIR=/tmp
R="attn_score|attn_bwd_step|attn_softmax"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU SQ_INSTS_VMEM_RD --kernel-include-regex "$R" -d $OUT/p1 -o run --output-format csv -- python3 tools/attn_micro.py > $OUT/p1.log 2>&1 || { tail -5 $OUT/p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum --kernel-include-regex "$R" -d $OUT/p2 -o run --output-format csv -- python3 tools/attn_micro.py > $OUT/p2.log 2>&1 || { tail -5 $OUT/p2.log; exit 1; }
python scripts/pmc_sum.py $(find $OUT/p1 -name "*counter_collection.csv")
python scripts/pmc_sum.py $(find $OUT/p2 -name "*counter_collection.csv")
