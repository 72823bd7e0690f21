#!/bin/bash
# Full GPU tier + bench A/B (dW overlap on/off) + 2-rank gloo DP plumbing + profile.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-iter7}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for cfg in "ovl " "noovl TSAMD_OVERLAP_DW=0"; do
  set -- $cfg
  for B in 256 64; do
    env $2 timeout -k 10 200 python bench.py --batch $B --steps 20 --warmup 3 > $OUT/$1_b$B.log 2>&1 || { tail -20 $OUT/$1_b$B.log; exit 1; }
    echo "$1 B=$B $(python -c "import json,sys; d=json.loads(open('$OUT/$1_b$B.log').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['value'])")"
  done
done
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --batch 64 --backend gloo > $OUT/dp2_gloo.log 2>&1 || { tail -20 $OUT/dp2_gloo.log; exit 1; }
tail -1 $OUT/dp2_gloo.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 4 --warmup 1 --batch 256 > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
python scripts/kstats.py $OUT/prof/run_kernel_stats.csv 7 16
