#!/bin/bash
# round 6: select-kernel phase stamps + the head micro
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-r6f}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 python tools/vocab_select_stamps.py > $OUT/stamps.log 2>&1 || { tail -20 $OUT/stamps.log; exit 1; }
tail -1 $OUT/stamps.log
timeout -k 10 120 python tools/vocab_micro.py --iters 200 2>&1 | tail -1
echo done
