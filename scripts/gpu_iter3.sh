#!/bin/bash
# Fused attention-backward A/B + vocab GEMM micro + batch sweep.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-iter3}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --batch 256 --steps 20 --warmup 3 > $OUT/b256_fused.log 2>&1 || { tail -20 $OUT/b256_fused.log; exit 1; }
tail -1 $OUT/b256_fused.log
TSAMD_ATTN_BWD_FUSED=0 timeout -k 10 200 python bench.py --batch 256 --steps 20 --warmup 3 > $OUT/b256_old.log 2>&1 || { tail -20 $OUT/b256_old.log; exit 1; }
tail -1 $OUT/b256_old.log
timeout -k 10 200 python bench.py --batch 64 --steps 20 --warmup 3 > $OUT/b64.log 2>&1 || { tail -20 $OUT/b64.log; exit 1; }
tail -1 $OUT/b64.log
timeout -k 10 200 python tools/vocab_gemm_micro.py > $OUT/vgemm.log 2>&1 || { tail -20 $OUT/vgemm.log; exit 1; }
tail -1 $OUT/vgemm.log
for B in 384 512; do
  timeout -k 10 200 python bench.py --batch $B --steps 10 --warmup 3 > $OUT/b$B.log 2>&1 || { tail -20 $OUT/b$B.log; exit 1; }
  tail -1 $OUT/b$B.log
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 4 --warmup 1 --batch 256 > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
python scripts/kstats.py $OUT/prof/run_kernel_stats.csv 7 25
