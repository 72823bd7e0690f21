#!/bin/bash
# round 5: vocab dW beside the decoder backward loop (TSAMD_VDW_LOOP) -- test, then a back-to-back
# bench A/B at B = 256 and config #5 (B = 1024)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-r5d}; mkdir -p $OUT
export TMPDIR=/tmp
step() { local n=$1; shift; echo "== $n"; timeout -k 10 ${T:-300} "$@" > $OUT/$n.log 2>&1; local rc=$?; tail -${TL:-3} $OUT/$n.log; return $rc; }
step t python -u -m pytest tests/test_gpu_production.py -q -x --timeout 300 --timeout-method thread -k "vocab_dw or deferred" || exit 1
for i in 1 2; do
  for v in 0 1; do
    TSAMD_VDW_LOOP=$v TL=1 step b${v}_$i python -u bench.py --decode-batches 0 --config5-steps 0 || exit 1
  done
done
for v in 0 1; do
  TSAMD_VDW_LOOP=$v TL=1 step c$v python -u bench.py --decode-batches 0 --config5-steps 0 --hidden 512 --layers 2 --enc 800 --batch 1024 --steps 4 --warmup 2 || exit 1
done
echo done
