#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-pv}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_gpu_decode.py -x -q --timeout 100 --timeout-method thread -k "vocab_topk or fused_decode" > $OUT/t.log 2>&1; tail -3 $OUT/t.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/v -o run --output-format csv -- python3 tools/vocab_micro.py > $OUT/v.log 2>&1 && python scripts/kstats.py $OUT/v/run_kernel_stats.csv 1 4 > $OUT/vocab_kstats.txt && cat $OUT/vocab_kstats.txt &&
timeout -k 10 200 python -u bench_decode.py > $OUT/bd.log 2>&1; tail -1 $OUT/bd.log
