#!/bin/bash
# PMC counters of the decode vocab logits kernel (tools/vocab_micro.py, R=256, V=50k).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmc_vocab; mkdir -p $OUT
export TMPDIR=/tmp
R="vocab_logits"
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU SQ_INSTS_VMEM_RD --kernel-include-regex "$R" -d $OUT/p1 -o run --output-format csv -- python3 tools/vocab_micro.py --iters 10 > $OUT/p1.log 2>&1 || { tail -5 $OUT/p1.log; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum --kernel-include-regex "$R" -d $OUT/p2 -o run --output-format csv -- python3 tools/vocab_micro.py --iters 10 > $OUT/p2.log 2>&1 || { tail -5 $OUT/p2.log; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE --kernel-include-regex "$R" -d $OUT/p3 -o run --output-format csv -- python3 tools/vocab_micro.py --iters 10 > $OUT/p3.log 2>&1 || { tail -5 $OUT/p3.log; exit 1; }
for p in p1 p2 p3; do python scripts/pmc_sum.py $(find $OUT/$p -name "*counter_collection.csv"); done
