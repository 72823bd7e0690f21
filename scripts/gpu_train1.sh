#!/bin/bash
# Training-path tests + B=64/B=256 bench + profile.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-train1}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests/test_gpu_pipeline.py tests/test_gpu_lstm.py -x -q > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || { grep -E "^E " $OUT/pytest.log | head -30; exit $rc; }
timeout -k 10 600 python bench.py --batch 256 --steps 20 --warmup 3 > $OUT/b256.log 2>&1 || { tail -20 $OUT/b256.log; exit 1; }
tail -1 $OUT/b256.log | cut -c1-200
timeout -k 10 600 python bench.py --batch 64 --steps 20 --warmup 3 > $OUT/b64.log 2>&1 && tail -1 $OUT/b64.log | cut -c1-200
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 4 --warmup 1 --batch 256 > $OUT/prof.log 2>&1; echo "prof rc=$?"
python scripts/kstats.py $OUT/prof/run_kernel_stats.csv 7 30
