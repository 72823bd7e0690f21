#!/bin/bash
# Round check: GPU test tier, smoke, headline bench (B=64 default and B=256), decode bench,
# rocprof kernel breakdown of a B=256 train step and of the decode.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-round}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -5 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python bench.py > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
timeout -k 10 300 python bench.py --batch 256 --steps 20 --warmup 3 > $OUT/b256.log 2>&1 || { tail -20 $OUT/b256.log; exit 1; }
tail -1 $OUT/b256.log
timeout -k 10 300 python bench_decode.py > $OUT/dec.log 2>&1 || { tail -20 $OUT/dec.log; exit 1; }
tail -1 $OUT/dec.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 4 --warmup 1 --batch 256 > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
python scripts/kstats.py $OUT/prof/run_kernel_stats.csv 5 30 > $OUT/train_kstats.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/dprof -o run --output-format csv -- python3 bench_decode.py --batches 2 > $OUT/dprof.log 2>&1 || { tail -20 $OUT/dprof.log; exit 1; }
echo done
