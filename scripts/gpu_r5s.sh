#!/bin/bash
# round 5: F stored pre-scaled by 2 log2(e), score arguments through v_dot2 (attn_common.h
# fadd_bf2) -- full GPU tier, then the driver-style bench (headline, decode, config #5).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5s; mkdir -p $OUT
export TMPDIR=/tmp
step() { local n=$1; shift; echo "== $n"; timeout -k 10 ${T:-300} "$@" > $OUT/$n.log 2>&1; local rc=$?; tail -${TL:-3} $OUT/$n.log; return $rc; }
T=120 step attn python -u -m pytest tests/test_gpu_attention_ops.py -q -x --timeout 60 --timeout-method thread || exit 1
T=600 step tier python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread || exit 1
T=600 TL=1 step bench python -u bench.py || exit 1
echo done
