#!/bin/bash
# round 6: decode head -- exactness tests, select stamps, micro, bench_decode
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-r6g}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_decode_parity.py tests/test_device_beam_results.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/vocab_select_stamps.py > $OUT/stamps.log 2>&1 || { tail -20 $OUT/stamps.log; exit 1; }
tail -1 $OUT/stamps.log
timeout -k 10 120 python tools/vocab_micro.py --iters 200 2>&1 | tail -1
timeout -k 10 120 python tools/vocab_span_probe.py 2>&1 | tail -1
timeout -k 10 300 python bench_decode.py 2>&1 | tail -1 | cut -c1-200
timeout -k 10 300 python bench_decode.py 2>&1 | tail -1 | cut -c1-200
echo done
