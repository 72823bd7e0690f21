#!/bin/bash
# Decode tests + A/B of the fused vocab head + profile.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/dec3; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_decode.py -x -q > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in 0 1; do
  TSAMD_FUSED_VOCAB=$v timeout -k 10 600 python bench_decode.py > $OUT/d64_f$v.log 2>&1 || { tail -20 $OUT/d64_f$v.log; exit 1; }
  echo "fused=$v $(grep -o '"value": [0-9.]*' $OUT/d64_f$v.log) $(grep -o '"ms_per_batch": [0-9.]*' $OUT/d64_f$v.log)"
done
timeout -k 10 600 python bench_decode.py --articles 128 > $OUT/d128.log 2>&1 && echo "128: $(grep -o '"value": [0-9.]*' $OUT/d128.log)"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench_decode.py --batches 1 --warmup 1 --no-graph > $OUT/prof.log 2>&1; echo "prof rc=$?"
