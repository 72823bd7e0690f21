#!/bin/bash
# round 5: waves per workgroup of the beam-decode attention (TSAMD_DEC_AW, temporary A/B)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5aw; mkdir -p $OUT
export TMPDIR=/tmp
T=120 timeout -k 10 120 python -u -m pytest tests/test_gpu_attention_ops.py -q -x --timeout 60 --timeout-method thread > $OUT/t.log 2>&1 || { tail -5 $OUT/t.log; exit 1; }
for r in 1 2; do for w in 16 8 12; do
  TSAMD_DEC_AW=$w timeout -k 10 200 python -u bench_decode.py > $OUT/d${w}_$r.log 2>&1 || exit 1
  echo "aw $w run $r $(grep -o '"value": [0-9.]*' $OUT/d${w}_$r.log | tail -1)"
done; done
echo done
