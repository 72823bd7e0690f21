#!/bin/bash
# round 6: rs_bwd over column groups, row-strided repack kind -- model / production tests, headline window
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-r6y}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_production.py tests/test_gpu_model.py tests/test_gpu_ctx.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --decode-batches 0 --config5-steps 0 > $OUT/bench$i.log 2>&1 || exit 1
  python -c "import json;r=json.loads(open('$OUT/bench$i.log').read().strip().splitlines()[-1]);print('bench', r['value'],r['ms_per_step'])"
done
timeout -k 10 400 rocprofv3 --kernel-trace -d $OUT/t1 -o run --output-format csv -- python3 bench.py --steps 6 --warmup 3 --decode-batches 0 --config5-steps 0 > $OUT/b256.log 2>&1 || exit 1
python scripts/kwin.py $OUT/t1/run_kernel_trace.csv 4 60 adagrad_kernel 3 > $OUT/train_kwin_b256.txt && python scripts/kgaps.py $OUT/t1/run_kernel_trace.csv 4 30 adagrad_kernel 3 > $OUT/train_gaps_b256.txt && head -1 $OUT/train_kwin_b256.txt
grep -i "rs_bwd\|pack_cast\|ctx_\|Cijk" $OUT/train_kwin_b256.txt | cut -c1-130
rm -rf $OUT/t1
echo done
