#!/bin/bash
# blt_mm candidate count A/B (24 default vs 64 vs 8)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-bltc}; mkdir -p $OUT
export TMPDIR=/tmp
step() { local n=$1; shift; echo "== $n"; timeout -k 10 ${T:-300} "$@" > $OUT/$n.log 2>&1; local rc=$?; grep -o '"ms_per_step": [0-9.]*\|"phase_ms_max_over_ranks": {[^}]*}\|"config5_ms_per_step": [0-9.]*' $OUT/$n.log | tr '\n' ' '; echo; return $rc; }
B="python -u bench.py --decode-batches 0"
T=400 step c24 env TSAMD_BLT_CANDIDATES=24 $B &&
T=400 step c64 env TSAMD_BLT_CANDIDATES=64 $B &&
T=400 step c8 env TSAMD_BLT_CANDIDATES=8 $B &&
T=400 step c64b env TSAMD_BLT_CANDIDATES=64 $B &&
T=400 step c24b env TSAMD_BLT_CANDIDATES=24 $B &&
T=300 step report python -u tools/blt_report.py && cat $OUT/report.log | grep '^{' > $OUT/report.jsonl &&
T=400 step report_c5 env C5=1 python -u tools/blt_report.py && cat $OUT/report_c5.log | grep '^{' > $OUT/report_c5.jsonl
