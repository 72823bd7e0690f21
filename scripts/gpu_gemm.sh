#!/bin/bash
# vocab-head GEMM variants (tools/attn_micro.py) with kernel names
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-gemm}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python tools/attn_micro.py > $OUT/attn.log 2>&1 || { tail -20 $OUT/attn.log; exit 1; }
tail -1 $OUT/attn.log
