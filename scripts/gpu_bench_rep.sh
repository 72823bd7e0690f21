#!/bin/bash
# Repeated bench runs (variance check) at B=64 and 256.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/rep; mkdir -p $OUT
timeout -k 10 300 python -m pytest tests/test_gpu_model.py -x -q > $OUT/pytest.log 2>&1 || { tail -20 $OUT/pytest.log; exit 1; }
for r in 1 2 3; do for b in 64 256; do
  timeout -k 10 300 python bench.py --batch $b --steps 20 > $OUT/b${b}_$r.log 2>&1 || { tail -20 $OUT/b${b}_$r.log; exit 1; }
  echo "b=$b r=$r $(grep -o '"ms_per_step": [0-9.]*' $OUT/b${b}_$r.log) $(grep -o '"value": [0-9.]*' $OUT/b${b}_$r.log)"
done; done
