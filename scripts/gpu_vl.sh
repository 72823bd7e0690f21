#!/bin/bash
# decode vocab logits epilogue: decode GPU tests, vocab micro + kernel stats, decode bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-vl}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $OUT/p0 -o run --output-format csv -- python3 tools/vocab_micro.py > $OUT/p0.log 2>&1 || { tail -20 $OUT/p0.log; exit 1; }
python scripts/kstats.py $OUT/p0/run_kernel_stats.csv 55 2
timeout -k 10 300 python bench_decode.py --batches 20 > $OUT/dec64.log 2>&1 || { tail -20 $OUT/dec64.log; exit 1; }
tail -1 $OUT/dec64.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_batch'], d['ms_per_batch_min'], d['ms_per_batch_median'])"
