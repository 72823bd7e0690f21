#!/bin/bash
# round 6: span decode logits probe timings (+ exactness test of the head)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-r6c}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 python tools/vocab_span_probe.py > $OUT/probe.log 2>&1 || { tail -20 $OUT/probe.log; exit 1; }
tail -1 $OUT/probe.log
ROWS=128 timeout -k 10 120 python tools/vocab_span_probe.py > $OUT/probe128.log 2>&1 || { tail -20 $OUT/probe128.log; exit 1; }
tail -1 $OUT/probe128.log
timeout -k 10 200 python -u -m pytest tests/test_gpu_decode.py -k "vocab_topk" -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for m in "" 1; do TSAMD_VL_TILE=$m timeout -k 10 120 python tools/vocab_micro.py --iters 200 2>&1 | tail -1; done
timeout -k 10 120 python tools/vocab_micro.py --iters 100 --hidden 512 --enc 800 2>&1 | tail -1
echo done
