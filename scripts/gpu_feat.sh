#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/feat; mkdir -p $OUT
export TMPDIR=/tmp
TSAMD_FEAT_V=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in 0 1 2; do
  TSAMD_FEAT_V=$v timeout -k 10 240 python tools/attn_micro.py > $OUT/m$v.log 2>&1 || { tail -20 $OUT/m$v.log; exit 1; }
  echo "feat_v=$v $(python -c "import json; d=json.loads(open('$OUT/m$v.log').read().strip().splitlines()[-1]); print(d['attn_bwd_feat'])")"
done
