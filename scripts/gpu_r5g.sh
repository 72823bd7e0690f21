#!/bin/bash
# round 5: config #5 (batch 2048, the bench sizing) kernel window + phase breakdown, and the headline
# bench, at the current state (merged upper-layer dX GEMM, batch-frame BPTT read).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-r5g}; mkdir -p $OUT
export TMPDIR=/tmp
step() { local n=$1; shift; echo "== $n"; timeout -k 10 ${T:-300} "$@" > $OUT/$n.log 2>&1; local rc=$?; tail -${TL:-3} $OUT/$n.log; return $rc; }
step kt python -u -m pytest tests/test_gpu_lstm.py tests/test_gpu_gemm.py -q -x --timeout 200 --timeout-method thread || exit 1
T=600 step orc python -u -m pytest tests/test_gpu_production.py -q -x --timeout 300 --timeout-method thread -k "config5_shape or bench_shape" || exit 1
T=400 TL=1 step b python -u bench.py --steps 20 --warmup 3 --decode-batches 0 --config5-steps 0 || exit 1
T=600 TL=1 step c5tr rocprofv3 --kernel-trace -d $OUT/tr -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --decode-batches 0 --config5-steps 2 || exit 1
python scripts/kwin.py $OUT/tr/run_kernel_trace.csv 2 45 > $OUT/cfg5_kwin_b2048.txt; head -3 $OUT/cfg5_kwin_b2048.txt
rm -rf $OUT/tr
T=500 TL=2 step ph python -u tools/phase_micro.py --hidden 512 --layers 2 --enc 800 --batch 2048 --iters 2 || exit 1
echo done
