#!/bin/bash
# round 5: attn_bwd_rowp without spills -- attention op tests, production oracle (bench shape +
# deterministic), headline bench x2, kernel window.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-r5l}; mkdir -p $OUT
export TMPDIR=/tmp
step() { local n=$1; shift; echo "== $n"; timeout -k 10 ${T:-300} "$@" > $OUT/$n.log 2>&1; local rc=$?; tail -${TL:-3} $OUT/$n.log; return $rc; }
step at python -u -m pytest tests/test_gpu_attention_ops.py -q -x --timeout 200 --timeout-method thread || exit 1
T=600 step orc python -u -m pytest tests/test_gpu_production.py -q -x --timeout 300 --timeout-method thread -k "bench_shape or deterministic or graph_replay" || exit 1
T=400 TL=1 step b1 python -u bench.py --steps 20 --warmup 3 --decode-batches 0 --config5-steps 0 || exit 1
T=400 TL=1 step b2 python -u bench.py --steps 20 --warmup 3 --decode-batches 0 --config5-steps 0 || exit 1
TL=2 step ph python -u tools/phase_micro.py || exit 1
T=400 step tr rocprofv3 --kernel-trace -d $OUT/tr -o run --output-format csv -- python3 bench.py --steps 3 --warmup 2 --decode-batches 0 --config5-steps 0 || exit 1
python scripts/kwin.py $OUT/tr/run_kernel_trace.csv 3 40 > $OUT/train_kwin_b256.txt; head -4 $OUT/train_kwin_b256.txt
rm -rf $OUT/tr
echo done
