#!/bin/bash
# kslice_mma 8-step batches in the decoder kernels: GPU tier, train + decode bench, train kernel stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-kb}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python bench.py > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | cut -c1-200
timeout -k 10 300 python bench_decode.py --batches 10 > $OUT/dec64.log 2>&1 || { tail -20 $OUT/dec64.log; exit 1; }
tail -1 $OUT/dec64.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 4 --warmup 1 > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
python scripts/kstats.py $OUT/prof/run_kernel_stats.csv 7 16 > $OUT/train_kstats.txt
grep -E "dec_|linear2|total" $OUT/train_kstats.txt
