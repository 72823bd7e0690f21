#!/bin/bash
# attn_score XCD-aware order: GPU tier, attention micro, FETCH_SIZE, train + decode bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-score}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python tools/attn_micro.py > $OUT/attn.log 2>&1 || { tail -20 $OUT/attn.log; exit 1; }
tail -1 $OUT/attn.log | cut -c1-200
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum --kernel-include-regex "attn_score|attn_softmax" -d $OUT/p2 -o run --output-format csv -- python3 tools/attn_micro.py > $OUT/p2.log 2>&1 || { tail -5 $OUT/p2.log; exit 1; }
python scripts/pmc_sum.py $(find $OUT/p2 -name "*counter_collection.csv")
timeout -k 10 300 python bench.py > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | cut -c1-200
timeout -k 10 300 python bench_decode.py > $OUT/dec64.log 2>&1 || { tail -20 $OUT/dec64.log; exit 1; }
tail -1 $OUT/dec64.log | cut -c1-200
