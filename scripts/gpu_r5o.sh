#!/bin/bash
# round 5: PMC profile of gemm_bt on the config #5 encoder-projection shape (where do the waves
# wait: LDS conflicts, load latency, barriers?), with the available SQ counter list first.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-r5o}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --list-avail > $OUT/avail.txt 2>&1 || true
grep -o "SQ_[A-Z0-9_]*\|TCP_[A-Z0-9_]*\|TCC_[A-Z0-9_]*" $OUT/avail.txt | sort -u > $OUT/avail_names.txt || true
wc -l $OUT/avail_names.txt
R="gemm_bt_kernel"
PROG="tools/gemm_micro.py --only c5_gx_l1 --reps 3"
p() {  # name counters...
  local n=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-include-regex "$R" -d $OUT/$n -o run --output-format csv -- python3 $PROG > $OUT/$n.log 2>&1 || { tail -5 $OUT/$n.log; return 1; }
  python scripts/pmc_sum.py $(find $OUT/$n -name "*counter_collection.csv") | tee $OUT/$n.txt
}
p p1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM &&
p p2 SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_LDS_UNALIGNED_STALL SQ_INSTS_VALU &&
p p3 GRBM_GUI_ACTIVE GRBM_COUNT TCC_HIT_sum TCC_MISS_sum
echo pmc done
