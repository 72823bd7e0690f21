#!/bin/bash
# fused LSTM gate-bias gradient: GPU tier, train profile (lstm bwd + reductions), bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-lstmdb}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 4 --warmup 1 > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
python scripts/kstats.py $OUT/prof/run_kernel_stats.csv 7 60 > $OUT/train_kstats.txt
grep -E "total|lstm_bwd|ReduceOp<c10::BFloat16|ReduceOp<float" $OUT/train_kstats.txt | cut -c1-120
timeout -k 10 300 python bench.py --steps 50 > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | cut -c1-200
