#!/bin/bash
# GPU tests, bench B=64/256, 2-rank DP plumbing check (gloo, one GPU), B=64 profile.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/it4; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for b in 64 256; do
  timeout -k 10 600 python bench.py --batch $b --steps 10 > $OUT/bench_b$b.log 2>&1 || { tail -20 $OUT/bench_b$b.log; exit 1; }
  tail -1 $OUT/bench_b$b.log
done
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --backend gloo --batch 16 --steps 3 --warmup 2 > $OUT/dp2.log 2>&1 || { tail -30 $OUT/dp2.log; exit 1; }
grep metric $OUT/dp2.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --batch 64 --no-graph > $OUT/prof.log 2>&1; echo "prof rc=$?"
