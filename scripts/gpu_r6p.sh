#!/bin/bash
# round 6: decoder-side weight gradients on wgrad_tt -- oracle + kernel tests, config #5 kernel window, bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-r6p}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm.py -m gpu -x -q --timeout 120 --timeout-method thread -k wgrad > $OUT/pytest_gemm.log 2>&1; rc=$?; tail -2 $OUT/pytest_gemm.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests/test_gpu_production.py -m gpu -x -v --timeout 300 --timeout-method thread -k "oracle or wgrad_tt" > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace -d $OUT/t2 -o run --output-format csv -- python3 bench.py --hidden 512 --enc 800 --layers 2 --batch 2048 --steps 3 --warmup 2 --decode-batches 0 --config5-steps 0 > $OUT/c5.log 2>&1 || exit 1
python scripts/kwin.py $OUT/t2/run_kernel_trace.csv 2 45 adagrad_kernel 3 > $OUT/cfg5_kwin_b2048.txt && head -2 $OUT/cfg5_kwin_b2048.txt
grep -i "cijk\|reduce_kernel\|wgrad" $OUT/cfg5_kwin_b2048.txt | cut -c1-140
rm -rf $OUT/t2
timeout -k 10 600 python bench.py --steps 3 --warmup 2 --decode-batches 0 > $OUT/bench.log 2>&1 || exit 1
python -c "import json;r=json.loads(open('$OUT/bench.log').read().strip().splitlines()[-1]);print(r['value'],r['ms_per_step'],r.get('config5_tokens_per_sec'),r.get('config5_ms_per_step'))"
echo done
