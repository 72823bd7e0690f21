#!/bin/bash
# round 5: position-split attention backward (TSAMD_ATTN_PARTS) -- kernel / engine tests, then a
# back-to-back bench A/B (B = 256 headline and config #5 batch 1024)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-r5c}; mkdir -p $OUT
export TMPDIR=/tmp
step() { local n=$1; shift; echo "== $n"; timeout -k 10 ${T:-300} "$@" > $OUT/$n.log 2>&1; local rc=$?; tail -${TL:-3} $OUT/$n.log; return $rc; }
step ops python -u -m pytest tests/test_gpu_attention_ops.py -q -x --timeout 120 --timeout-method thread || exit 1
T=600 step prod python -u -m pytest tests/test_gpu_production.py tests/test_gpu_model.py -q -x --timeout 300 --timeout-method thread || exit 1
for v in 1 2 4 1 2 4; do
  TSAMD_ATTN_PARTS=$v TL=1 step b$v python -u bench.py --decode-batches 0 --config5-steps 0 || exit 1
done
for v in 1 2; do
  TSAMD_ATTN_PARTS=$v TL=1 step c$v python -u bench.py --decode-batches 0 --config5-steps 0 --hidden 512 --layers 2 --enc 800 --batch 1024 --steps 4 --warmup 2 || exit 1
done
echo done
