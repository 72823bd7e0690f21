#!/bin/bash
# Isolated kernel timings at the B=256 bench shape, one process per variant.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-micro2}; mkdir -p $OUT
for cfg in "base" "occ3 TSAMD_ATTN_OCC=3" "occ4 TSAMD_ATTN_OCC=4" "sw8 TSAMD_ATTN_SW=8"; do
  set -- $cfg
  env $2 timeout -k 10 240 python tools/attn_micro.py > $OUT/$1.log 2>&1 || { tail -20 $OUT/$1.log; exit 1; }
  echo "$1 $(tail -1 $OUT/$1.log)"
done
