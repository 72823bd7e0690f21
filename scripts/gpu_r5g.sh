#!/bin/bash
# round 5: bf16 a written by attn_fwd_rowp, one-pass ctx transpose + cast (tr01) -- op tests, oracles, bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-r5g}; mkdir -p $OUT
export TMPDIR=/tmp
step() { local n=$1; shift; echo "== $n"; timeout -k 10 ${T:-300} "$@" > $OUT/$n.log 2>&1; local rc=$?; tail -${TL:-1} $OUT/$n.log | cut -c1-300; return $rc; }
T=120 step attn python -u -m pytest tests/test_gpu_attention_ops.py tests/test_gpu_frames.py -q -x --timeout 60 --timeout-method thread || exit 1
T=700 step orc python -u -m pytest tests/test_gpu_production.py tests/test_gpu_model.py -q -x --timeout 300 --timeout-method thread || exit 1
T=600 step bench python -u bench.py --decode-batches 0 || exit 1
grep -o '"ms_per_step": [0-9.]*\|"config5_ms_per_step": [0-9.]*' $OUT/bench.log
echo done
