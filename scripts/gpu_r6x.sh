#!/bin/bash
# round 6: batched attention-context GEMMs on ctx_bmm.hip -- kernel tests, micro (library vs
# native), oracle tests, A/B bench (TSAMD_CTX_NATIVE=1 / 0)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-r6x}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_ctx.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_ctx.log 2>&1; rc=$?; tail -3 $OUT/pytest_ctx.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/ctx_bmm_micro.py --native > $OUT/micro_b256.json 2>&1 || exit 1
timeout -k 10 200 python tools/ctx_bmm_micro.py --native --B 2048 --T 800 --A 1024 > $OUT/micro_c5.json 2>&1 || exit 1
cat $OUT/micro_b256.json $OUT/micro_c5.json | grep "{"
timeout -k 10 900 python -u -m pytest tests/test_gpu_production.py tests/test_gpu_model.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for nat in 1 0 1 0; do
  TSAMD_CTX_NATIVE=$nat timeout -k 10 300 python bench.py --steps 20 --warmup 5 --decode-batches 0 --config5-steps 0 > $OUT/bench_nat$nat.log 2>&1 || exit 1
  python -c "import json;r=json.loads(open('$OUT/bench_nat$nat.log').read().strip().splitlines()[-1]);print('native $nat', r['value'],r['ms_per_step'])"
done
echo done
