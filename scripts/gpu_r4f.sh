#!/bin/bash
# round-4: the 16-wave 32-row-team H = 512 BPTT (numerics vs the step kernels, per-step timing
# on/off), then config #5 on the bench (its --batch auto line)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-r4f}; mkdir -p $OUT
export TMPDIR=/tmp
step() { local n=$1; shift; echo "== $n"; timeout -k 10 ${T:-300} "$@" > $OUT/$n.log 2>&1; local rc=$?; tail -${TL:-3} $OUT/$n.log; return $rc; }
for m in 0 1 2 4 7; do
  TSAMD_VL_MODE=$m T=120 step vl_mode$m rocprofv3 --kernel-trace --stats -d $OUT/vl$m -o run --output-format csv -- python3 tools/vocab_micro.py || exit 1
  python scripts/kstats.py $OUT/vl$m/run_kernel_stats.csv 1 3 | tail -2
done
step lstm python -u -m pytest tests/test_gpu_lstm.py -x -q --timeout 100 --timeout-method thread &&
step micro32 python -u tools/lstm_micro.py 512:512:800 512:1024:800 512:2048:800 &&
TSAMD_LSTM_BWD32=0 step micro16 python -u tools/lstm_micro.py 512:512:800 512:1024:800 512:2048:800 &&
step cfg5test python -u -m pytest tests/test_gpu_production.py -x -q --timeout 200 --timeout-method thread -k config5 &&
T=600 step bench python -u bench.py --steps 10 --warmup 3
