#!/bin/bash
# End-of-session numbers, part 1: GPU tier, smoke, headline bench (B=256, train + beam-4 decode),
# batch sweep, config #5, 2-rank self-launched DP plumbing (gloo, both ranks on the one GPU),
# rocprof kernel stats of the B=256 train step and of the decode.  Part 2: gpu_final2.sh.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-final}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
j() { python -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); print('$2', d.get('ms_per_step', d.get('ms_per_batch')), d['value'], d['unit'], d.get('beam4_summaries_per_sec', ''))"; }
timeout -k 10 300 python bench.py > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
j $OUT/bench.log "train B=256 (default) + decode"
for B in 64 128 512; do
  timeout -k 10 300 python bench.py --batch $B --steps 20 --warmup 3 --decode-batches 0 > $OUT/b$B.log 2>&1 || { tail -20 $OUT/b$B.log; exit 1; }
  j $OUT/b$B.log "train B=$B"
done
timeout -k 10 300 python bench.py --hidden 512 --layers 2 --enc 800 --batch auto --steps 3 --warmup 1 --decode-batches 2 > $OUT/cfg5.log 2>&1 || { tail -20 $OUT/cfg5.log; exit 1; }
j $OUT/cfg5.log "config5 H=512 L=2 enc=800 B=auto"
timeout -k 10 300 python bench.py --gpus 2 --backend gloo --batch 64 --steps 5 --warmup 2 --decode-batches 1 > $OUT/dp2_gloo.log 2>&1 || { tail -20 $OUT/dp2_gloo.log; exit 1; }
j $OUT/dp2_gloo.log "dp2 gloo plumbing (self-launched ranks)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 4 --warmup 1 --batch 256 --decode-batches 0 > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
python scripts/kstats.py $OUT/prof/run_kernel_stats.csv 7 30 > $OUT/train_kstats.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/dprof -o run --output-format csv -- python3 bench_decode.py --batches 2 > $OUT/dprof.log 2>&1 || { tail -20 $OUT/dprof.log; exit 1; }
python scripts/kstats.py $OUT/dprof/run_kernel_stats.csv 3 20 > $OUT/decode_kstats.txt
echo done
