#!/bin/bash
# round 5: encoder-output fill removed (LSTM writes zeros past lengths), attn_bwd_feat spill cut:
# kernel tests, oracles, headline + config #5 bench, kernel windows of both.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-r5n}; mkdir -p $OUT
export TMPDIR=/tmp
step() { local n=$1; shift; echo "== $n"; timeout -k 10 ${T:-300} "$@" > $OUT/$n.log 2>&1; local rc=$?; tail -${TL:-3} $OUT/$n.log; return $rc; }
step kt python -u -m pytest tests/test_gpu_lstm.py tests/test_gpu_attention_ops.py -q -x --timeout 200 --timeout-method thread || exit 1
T=600 step orc python -u -m pytest tests/test_gpu_production.py -q -x --timeout 300 --timeout-method thread -k "config5_shape or bench_shape or deterministic" || exit 1
T=500 TL=1 step b python -u bench.py --steps 20 --warmup 3 --decode-batches 0 --config5-steps 5 || exit 1
T=600 step c5tr rocprofv3 --kernel-trace -d $OUT/tr -o run --output-format csv -- python3 bench.py --steps 3 --warmup 2 --decode-batches 0 --config5-steps 2 || exit 1
python scripts/kwin.py $OUT/tr/run_kernel_trace.csv 2 45 > $OUT/cfg5_kwin_b2048.txt; head -3 $OUT/cfg5_kwin_b2048.txt
rm -rf $OUT/tr
echo done
