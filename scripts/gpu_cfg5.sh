#!/bin/bash
# config #5 A/B: attention-backward numerics tests, then the config #5 bench with the default
# (256-position A=1024 kernel) and with the old 8-position kernel (TSAMD_ATTN_P4K2=0)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-cfg5}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_attention_ops.py tests/test_gpu_model.py -k "attn or attention" > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in 5 0; do
  TSAMD_ATTN_P4K2=$v timeout -k 10 300 python bench.py --hidden 512 --layers 2 --enc 800 --batch auto --steps 3 --warmup 1 --decode-batches 0 > $OUT/cfg5_$v.log 2>&1 || { tail -20 $OUT/cfg5_$v.log; exit 1; }
  tail -1 $OUT/cfg5_$v.log
done
