#!/bin/bash
# blt_mm A/B by GEMM class: activation GEMMs only / + vocab dW / + long-K wgrads / torch.mm
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-bltab}; mkdir -p $OUT
export TMPDIR=/tmp
step() { local n=$1; shift; echo "== $n"; timeout -k 10 ${T:-300} "$@" > $OUT/$n.log 2>&1; local rc=$?; grep -o '"ms_per_step": [0-9.]*\|"phase_ms_max_over_ranks": {[^}]*}\|"config5_ms_per_step": [0-9.]*' $OUT/$n.log | tr '\n' ' '; echo; return $rc; }
B="python -u bench.py --decode-batches 0"
T=400 step act env TSAMD_BLT=1 $B &&
T=400 step act_vdw env TSAMD_BLT=1 TSAMD_BLT_VOCAB_DW=1 $B &&
T=400 step torch env TSAMD_BLT=0 $B &&
T=400 step act_wgrad env TSAMD_BLT=1 TSAMD_BLT_WGRAD=1 $B &&
T=400 step act2 env TSAMD_BLT=1 $B
