#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/p4; mkdir -p $OUT
export TMPDIR=/tmp
TSAMD_ATTN_P4=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_decode.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in 0 1 2 3; do
  TSAMD_ATTN_P4=$v timeout -k 10 240 python tools/attn_micro.py > $OUT/m$v.log 2>&1 || { tail -20 $OUT/m$v.log; exit 1; }
  echo "p4=$v $(python -c "import json; d=json.loads(open('$OUT/m$v.log').read().strip().splitlines()[-1]); print(d['attn_bwd_step'])")"
done
timeout -k 10 300 python bench_decode.py > $OUT/dec.log 2>&1 || { tail -20 $OUT/dec.log; exit 1; }
tail -1 $OUT/dec.log | cut -c1-200
