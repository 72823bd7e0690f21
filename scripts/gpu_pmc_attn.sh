#!/bin/bash
# PMC record of the four attention kernels (attn_fwd_row, attn_bwd_row, attn_bwd_feat,
# attn_bwd_step4) at the bench shape (A = 512, T = 400) and config #5's (A = 1024, T = 800),
# 256 rows per launch, random operands (tools/attn_micro_c5.py), one counter group per pass.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-pmc_attn}; mkdir -p $OUT
export TMPDIR=/tmp
R="${PMC_REGEX:-attn_fwd_row|attn_bwd_row|attn_bwd_feat|attn_bwd_step4}"
p() {  # shape-tag pass counters...
  local n=$1; shift
  timeout -s KILL 150 rocprofv3 --pmc "$@" --kernel-include-regex "$R" -d $OUT/$n -o run --output-format csv -- python3 tools/attn_micro_c5.py > $OUT/$n.log 2>&1 || { tail -5 $OUT/$n.log; return 1; }
  python scripts/pmc_sum.py $(find $OUT/$n -name "*counter_collection.csv") > $OUT/$n.txt
}
for shape in a512 a1024; do
  if [ $shape = a512 ]; then export T=400 A=512 NG=4 D=100; else export T=800 A=1024 NG=4 D=100; fi
  p ${shape}_p1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD || exit 1
  p ${shape}_p2 SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 || exit 1
  p ${shape}_p3 FETCH_SIZE TCC_HIT_sum || exit 1
  p ${shape}_p4 GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT32 || exit 1
done
echo pmc done
