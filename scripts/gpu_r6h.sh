#!/bin/bash
# round 6: decode A/B, span vs tile logits kernel (alternating), headline + config-5 decode shapes
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-r6h}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_decode_parity.py tests/test_device_beam_results.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for m in 0 1; do
    TSAMD_VL_TILE=$m timeout -k 10 300 python bench_decode.py > $OUT/dec_${m}_$i.log 2>&1 || exit 1
    echo "tile=$m $(grep -o '"value": [0-9.]*' $OUT/dec_${m}_$i.log | tail -1)" | tee -a $OUT/ab.txt
  done
done
for m in 0 1; do
  TSAMD_VL_TILE=$m timeout -k 10 300 python bench_decode.py --hidden 512 --layers 2 --enc 800 > $OUT/c5_${m}.log 2>&1 || exit 1
  echo "c5 tile=$m $(grep -o '"value": [0-9.]*' $OUT/c5_${m}.log | tail -1)" | tee -a $OUT/ab.txt
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench_decode.py --batches 5 > $OUT/prof.log 2>&1 &&
python scripts/kstats.py $OUT/prof/run_kernel_stats.csv 6 12 > $OUT/decode_kstats.txt && head -8 $OUT/decode_kstats.txt
echo done
