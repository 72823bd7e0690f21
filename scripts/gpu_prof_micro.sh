#!/bin/bash
# decode micro benchmarks: attention variants (env knob), vocab head; kernel stats of each
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-pm}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 python -u -m pytest tests/test_gpu_attention_ops.py -x -q --timeout 60 --timeout-method thread -k beam > $OUT/attn_test.log 2>&1; tail -1 $OUT/attn_test.log
for v in 0 1 2; do
  TSAMD_ATTN_BEAM_VARIANT=$v timeout -k 10 120 python -u tools/decode_kernels_micro.py > $OUT/attn_v$v.log 2>&1 || exit 1
  echo "variant $v: $(tail -1 $OUT/attn_v$v.log)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/a -o run --output-format csv -- python3 tools/decode_kernels_micro.py --reps 20 > $OUT/a.log 2>&1 && python scripts/kstats.py $OUT/a/run_kernel_stats.csv 1 8 > $OUT/attn_kstats.txt && cat $OUT/attn_kstats.txt &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/v -o run --output-format csv -- python3 tools/vocab_micro.py > $OUT/v.log 2>&1 && python scripts/kstats.py $OUT/v/run_kernel_stats.csv 1 8 > $OUT/vocab_kstats.txt && cat $OUT/vocab_kstats.txt
