#!/bin/bash
# round 6: attribution of the span decode logits kernel -- probe timings + PMC passes
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-r6b}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 python tools/vocab_span_probe.py > $OUT/probe.log 2>&1 || { tail -20 $OUT/probe.log; exit 1; }
tail -1 $OUT/probe.log
ROWS=128 timeout -k 10 120 python tools/vocab_span_probe.py > $OUT/probe128.log 2>&1 || { tail -20 $OUT/probe128.log; exit 1; }
tail -1 $OUT/probe128.log
R="vocab_logits_span"
p() {  # name counters...
  local n=$1; shift
  PMC=1 timeout -s KILL 60 rocprofv3 --pmc "$@" --kernel-include-regex "$R" -d $OUT/$n -o run --output-format csv -- python3 tools/vocab_span_probe.py > $OUT/$n.log 2>&1 || { tail -5 $OUT/$n.log; return 1; }
  python scripts/pmc_sum.py $(find $OUT/$n -name "*counter_collection.csv") | tee $OUT/$n.txt
}
p p1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD &&
p p3 FETCH_SIZE TCC_HIT_sum &&
p p4 GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_VALU SQ_INSTS_LDS &&
p p5 SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS &&
p p6 WRITE_SIZE TCC_MISS_sum
echo done
