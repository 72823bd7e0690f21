#!/bin/bash
# round 5: GEMM + decode-select tests, micro A/Bs, deterministic / oracle tests, decode A/B, bench,
# timeline trace.  Every GPU step has its own time limit; the first failure ends the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-r5b}; mkdir -p $OUT
export TMPDIR=/tmp
step() { local n=$1; shift; echo "== $n"; timeout -k 10 ${T:-300} "$@" > $OUT/$n.log 2>&1; local rc=$?; tail -${TL:-3} $OUT/$n.log; return $rc; }
step gemmt python -u -m pytest tests/test_gpu_gemm.py -q -x --timeout 120 --timeout-method thread || exit 1
step dect python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_decode_parity.py -q -x --timeout 300 --timeout-method thread || exit 1
TL=8 step gemm python -u tools/gemm_micro.py || exit 1
TL=12 step wgrad python -u tools/wgrad_tn_micro.py || exit 1
step det python -u -m pytest tests/test_gpu_production.py -q -x --timeout 300 --timeout-method thread -k "deterministic or oracle or held" || exit 1
for v in 1 0; do
  TSAMD_VS_ART=$v T=120 step vs$v rocprofv3 --kernel-trace --stats -d $OUT/vs$v -o run --output-format csv -- python3 tools/vocab_micro.py || exit 1
  python scripts/kstats.py $OUT/vs$v/run_kernel_stats.csv 1 3 | sed -n 2,3p
done
TSAMD_VS_ART=0 TL=1 step dec0 python -u bench_decode.py --batches 10 || exit 1
TL=1 step dec1 python -u bench_decode.py --batches 10 || exit 1
T=600 TL=1 step bench python -u bench.py || exit 1
step trace rocprofv3 --kernel-trace -d $OUT/tr -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --decode-batches 0 --config5-steps 0 || exit 1
python scripts/kwin.py $OUT/tr/run_kernel_trace.csv 1 40 > $OUT/kwin_b256.txt
python scripts/loop_tl.py $OUT/tr/run_kernel_trace.csv attn_bwd_rowp 60 30 > $OUT/tl_bwd.txt
python scripts/loop_tl.py $OUT/tr/run_kernel_trace.csv attn_fwd_rowp 60 30 > $OUT/tl_fwd.txt
rm -rf $OUT/tr
echo done
