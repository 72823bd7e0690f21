#!/bin/bash
# Vocab-head micro-benchmark + rocprof split (pointer on / off).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-micro}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_gpu_decode.py -x -q -k "fused_vocab" > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/vocab_micro.py > $OUT/micro.log 2>&1 && tail -1 $OUT/micro.log
timeout -k 10 300 python tools/vocab_micro.py --no-pointer > $OUT/micro_np.log 2>&1 && tail -1 $OUT/micro_np.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/p1 -o run --output-format csv -- python3 tools/vocab_micro.py --iters 20 > $OUT/p1.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/p2 -o run --output-format csv -- python3 tools/vocab_micro.py --iters 20 --no-pointer > $OUT/p2.log 2>&1; echo "prof rc=$?"
python scripts/kstats.py $OUT/p1/run_kernel_stats.csv 1 8 2>/dev/null; python scripts/kstats.py $OUT/p2/run_kernel_stats.csv 1 8 2>/dev/null; true
