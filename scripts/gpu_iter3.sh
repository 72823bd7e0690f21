#!/bin/bash
# Round-3 iteration: selected GPU tests (PYTEST_K), then optional attention micro + PMC passes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${OUTD:-iter3}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest ${PYTEST_FILES:-tests} -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $OUT/pytest.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR" $OUT/pytest.log | tail -30; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || [ -n "$CONTINUE" ] || exit $rc
if [ -n "$PMC" ]; then
  timeout -k 10 120 python tools/attn_micro.py > $OUT/attn_micro.json 2>&1 && tail -1 $OUT/attn_micro.json
  OUTD=${OUTD:-iter3}/pmc bash scripts/gpu_pmc_row.sh && PROG=tools/attn_bwd_a1024_micro.py OUTD=${OUTD:-iter3}/pmc1024 bash scripts/gpu_pmc_row.sh
fi
echo done
