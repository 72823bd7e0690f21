#!/bin/bash
# PMC counters of the fused training vocab head (tools/vocab_train_micro.py, bench shape):
# issue / stall counters, instruction mix, bytes moved.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmc_vt; mkdir -p $OUT
export TMPDIR=/tmp
R="vocab_train"
p() {  # name counters...
  local n=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-include-regex "$R" -d $OUT/$n -o run --output-format csv -- python3 tools/vocab_train_micro.py --reps 1 --iters 2 > $OUT/$n.log 2>&1 || { tail -5 $OUT/$n.log; return 1; }
  python scripts/pmc_sum.py $(find $OUT/$n -name "*counter_collection.csv") | tee $OUT/$n.txt
}
p p1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD &&
p p2 SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 &&
p p3 FETCH_SIZE TCC_HIT_sum &&
p p4 GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT32 &&
p p5 SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_WR &&
p p6 WRITE_SIZE TCC_MISS_sum
echo pmc done
