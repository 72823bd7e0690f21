#!/bin/bash
# PMC counters of the row-resident attention kernels and the feature-gradient pass at the
# B=256 bench shape (tools/attn_micro.py): waves / issue / stall counters, instruction mix
# (VALU, transcendental, VMEM), bytes fetched.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-pmc_row}; mkdir -p $OUT
export TMPDIR=/tmp
R="attn_fwd_row|attn_bwd_row|attn_bwd_feat|attn_bwd_step4"
PROG=${PROG:-tools/attn_micro.py}
p() {  # name counters...
  local n=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-include-regex "$R" -d $OUT/$n -o run --output-format csv -- python3 $PROG > $OUT/$n.log 2>&1 || { tail -5 $OUT/$n.log; return 1; }
  python scripts/pmc_sum.py $(find $OUT/$n -name "*counter_collection.csv") | tee $OUT/$n.txt
}
p p1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD &&
p p2 SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 &&
p p3 FETCH_SIZE TCC_HIT_sum &&
p p4 GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT32
echo pmc done
