#!/bin/bash
# round 6: column-span decode vocab_logits -- decode tests, micro A/B (span vs tile), kernel stats, bench_decode A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-r6a}; mkdir -p $OUT
export TMPDIR=/tmp
step() { local n=$1; shift; echo "== $n"; timeout -k 10 ${T:-300} "$@" > $OUT/$n.log 2>&1; local rc=$?; grep -h '^{' $OUT/$n.log | cut -c1-220; return $rc; }
step pytest python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_decode_parity.py tests/test_device_beam_results.py -m gpu -x -v --timeout 120 --timeout-method thread; rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
step micro_span python tools/vocab_micro.py --iters 200 &&
TSAMD_VL_TILE=1 step micro_tile python tools/vocab_micro.py --iters 200 &&
step micro_span512 python tools/vocab_micro.py --iters 100 --hidden 512 --enc 800 &&
TSAMD_VL_TILE=1 step micro_tile512 python tools/vocab_micro.py --iters 100 --hidden 512 --enc 800 &&
step prof_span rocprofv3 --kernel-trace --stats -d $OUT/ps -o run --output-format csv -- python3 tools/vocab_micro.py --iters 100 &&
python scripts/kstats.py $OUT/ps/run_kernel_stats.csv 1 8 > $OUT/kstats_span.txt &&
step dec_span python bench_decode.py &&
TSAMD_VL_TILE=1 step dec_tile python bench_decode.py &&
step dec_span2 python bench_decode.py
echo done
