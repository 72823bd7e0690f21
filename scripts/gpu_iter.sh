#!/bin/bash
# Quick iteration: selected GPU tests (PYTEST_K), then the default bench (and extra BENCH_ARGS variants).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-iter}; mkdir -p $OUT
export TMPDIR=/tmp
if [ -n "$PYTEST_K" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$PYTEST_K" > $OUT/pytest.log 2>&1
  rc=$?; tail -4 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
fi
i=0
for a in "" $BENCH_VARIANTS; do
  i=$((i+1))
  timeout -k 10 300 env $a python bench.py ${BENCH_ARGS} > $OUT/bench$i.log 2>&1 || { tail -20 $OUT/bench$i.log; exit 1; }
  echo "[$a] $(tail -1 $OUT/bench$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d.get("beam4_summaries_per_sec"), d.get("beam4_ms_per_batch"))')"
done
echo done
