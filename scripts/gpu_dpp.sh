#!/bin/bash
# DPP / permlane cross-lane reductions: GPU tier, vocab head micro (occupancy 2 vs 4),
# attention micro, decode and train bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-dpp}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 120 python tools/vocab_micro.py > $OUT/v2.log 2>&1 || { tail -20 $OUT/v2.log; exit 1; }
tail -1 $OUT/v2.log
TSAMD_VL_OCC=4 timeout -k 10 120 python tools/vocab_micro.py > $OUT/v4.log 2>&1 || { tail -20 $OUT/v4.log; exit 1; }
tail -1 $OUT/v4.log
timeout -k 10 300 python tools/attn_micro.py > $OUT/attn.log 2>&1 || { tail -20 $OUT/attn.log; exit 1; }
tail -3 $OUT/attn.log
timeout -k 10 300 python bench_decode.py > $OUT/dec64.log 2>&1 || { tail -20 $OUT/dec64.log; exit 1; }
tail -1 $OUT/dec64.log
TSAMD_VL_OCC=4 timeout -k 10 300 python bench_decode.py > $OUT/dec64o4.log 2>&1 || { tail -20 $OUT/dec64o4.log; exit 1; }
tail -1 $OUT/dec64o4.log
timeout -k 10 300 python bench.py > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
