#!/bin/bash
# Round check: GPU test tier, smoke, headline bench (default B=256, and B=64), decode bench,
# 2-rank DP plumbing (gloo, both ranks on the one GPU), rocprof kernel breakdown of a B=256
# train step and of the decode.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-round}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python bench.py > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
timeout -k 10 300 python bench.py --batch 64 --steps 20 --warmup 3 > $OUT/b64.log 2>&1 || { tail -20 $OUT/b64.log; exit 1; }
tail -1 $OUT/b64.log
timeout -k 10 300 python bench_decode.py > $OUT/dec.log 2>&1 || { tail -20 $OUT/dec.log; exit 1; }
tail -1 $OUT/dec.log
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --batch 64 --backend gloo > $OUT/dp2_gloo.log 2>&1 || { tail -20 $OUT/dp2_gloo.log; exit 1; }
tail -1 $OUT/dp2_gloo.log | cut -c1-240
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 4 --warmup 1 --batch 256 > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
python scripts/kstats.py $OUT/prof/run_kernel_stats.csv 5 30 > $OUT/train_kstats.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/dprof -o run --output-format csv -- python3 bench_decode.py --batches 2 > $OUT/dprof.log 2>&1 || { tail -20 $OUT/dprof.log; exit 1; }
echo done
