#!/bin/bash
# Decode vocab head: micro timing, decode GPU tests, decode bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-vmicro}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 python tools/vocab_micro.py > $OUT/base.log 2>&1 || { tail -20 $OUT/base.log; exit 1; }
tail -1 $OUT/base.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python bench_decode.py > $OUT/dec64.log 2>&1 || { tail -20 $OUT/dec64.log; exit 1; }
tail -1 $OUT/dec64.log
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $OUT/p0 -o run --output-format csv -- python3 tools/vocab_micro.py > $OUT/p0.log 2>&1 || { tail -20 $OUT/p0.log; exit 1; }
python scripts/kstats.py $OUT/p0/run_kernel_stats.csv 55 3
