#!/bin/bash
# round 6: padded vocab gradients (dlogits rows / bf16 W at Vp = 128-aligned columns; dX on the
# split-K hand-written GEMM) -- kernel tests, oracle tests, A/B bench (TSAMD_VOCAB_PAD=0 / 1),
# headline kernel window
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-r6v}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm.py -m gpu -x -q --timeout 120 --timeout-method thread -k "splitk or narrow or wgrad" > $OUT/pytest_gemm.log 2>&1; rc=$?; tail -2 $OUT/pytest_gemm.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests/test_gpu_production.py tests/test_gpu_model.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for pad in 1 0 1 0; do
  TSAMD_VOCAB_PAD=$pad timeout -k 10 300 python bench.py --steps 20 --warmup 5 --decode-batches 0 --config5-steps 0 > $OUT/bench_pad$pad.log 2>&1 || exit 1
  python -c "import json;r=json.loads(open('$OUT/bench_pad$pad.log').read().strip().splitlines()[-1]);print('pad $pad', r['value'],r['ms_per_step'])"
done
timeout -k 10 400 rocprofv3 --kernel-trace -d $OUT/t1 -o run --output-format csv -- python3 bench.py --steps 6 --warmup 3 --decode-batches 0 --config5-steps 0 > $OUT/b256.log 2>&1 || exit 1
python scripts/kwin.py $OUT/t1/run_kernel_trace.csv 4 45 adagrad_kernel 3 > $OUT/train_kwin_b256.txt && head -2 $OUT/train_kwin_b256.txt
grep -i "cijk\|gemm_bt\|wgrad\|sum_kernel\|vocab" $OUT/train_kwin_b256.txt | cut -c1-150
rm -rf $OUT/t1
echo done
