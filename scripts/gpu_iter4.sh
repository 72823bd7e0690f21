#!/bin/bash
# Fused attention-backward variants (NG=4 / NG=2 / two-kernel path) at B=256 and B=64.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-iter4}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for cfg in "ng4 " "ng2 TSAMD_ATTN_NG=2" "old TSAMD_ATTN_BWD_FUSED=0"; do
  set -- $cfg
  for B in 256 64; do
    env $2 timeout -k 10 200 python bench.py --batch $B --steps 20 --warmup 3 > $OUT/$1_b$B.log 2>&1 || { tail -20 $OUT/$1_b$B.log; exit 1; }
    echo "$1 B=$B $(python -c "import json,sys; d=json.loads(open('$OUT/$1_b$B.log').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['value'])")"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 4 --warmup 1 --batch 256 > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
python scripts/kstats.py $OUT/prof/run_kernel_stats.csv 7 12
