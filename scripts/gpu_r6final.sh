#!/bin/bash
# round-6 closing run: full GPU test tier, smoke, the driver's default bench (timed), decode bench,
# 2-rank DP plumbing over gloo on the one GPU.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-r6final}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
s=$(date +%s); timeout -k 10 600 python bench.py > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
echo "bench wall $(( $(date +%s) - s )) s"; tail -1 $OUT/bench.log > $OUT/bench.json; cut -c1-300 $OUT/bench.json
timeout -k 10 300 python bench_decode.py > $OUT/dec.log 2>&1 || { tail -20 $OUT/dec.log; exit 1; }
tail -1 $OUT/dec.log | cut -c1-200
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --batch 64 --backend gloo --config5-steps 0 --decode-batches 2 > $OUT/dp2_gloo.log 2>&1 || { tail -20 $OUT/dp2_gloo.log; exit 1; }
tail -1 $OUT/dp2_gloo.log | cut -c1-240
echo done
