#!/bin/bash
# A/B and profiling runs used while tuning (one GPU).  Usage: bash scripts/gpu_ab.sh <what>
#   attn1024  attn_bwd_step at A = 1024, random and full lengths
#   cfg5      attention tests + config #5 bench
#   cfg5prof  rocprofv3 kernel stats of the config #5 bench
#   decode    bench_decode with $AB_ENV = 1 / 0 at 64 and 128 articles, twice
#   train     GPU tests matching $AB_K, then the B = 256 train bench for each $AB_ENV value in
#             $AB_VALUES (default "1 0 1 0"), and config #5 at B = 512 too when AB_CFG5=1
#             (e.g. AB_ENV=TSAMD_DEFER_WGRAD AB_K="model or decode" bash scripts/gpu_ab.sh train)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${OUTD:-ab_$1}; mkdir -p $OUT
CFG5="--hidden 512 --layers 2 --enc 800 --batch auto --steps 3 --warmup 1 --decode-batches 0"
case "$1" in
attn1024)
  for full in "" 1; do
    MICRO_FULL=$full timeout -k 10 120 python tools/attn_bwd_a1024_micro.py >> $OUT/a1024.jsonl || exit 1
  done; cat $OUT/a1024.jsonl ;;
cfg5)
  timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_attention_ops.py \
    tests/test_gpu_model.py -k "attn or attention" > $OUT/pytest.log 2>&1
  rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python bench.py $CFG5 > $OUT/cfg5.log 2>&1 || { tail -20 $OUT/cfg5.log; exit 1; }
  tail -1 $OUT/cfg5.log ;;
cfg5prof)
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py $CFG5 \
    > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
  python scripts/kstats.py $OUT/prof/run_kernel_stats.csv 4 40 > $OUT/kstats.txt; tail -1 $OUT/prof.log ;;
decode)
  for rep in 1 2; do for v in 1 0; do for a in 64 128; do
    L=$OUT/d_${v}_${a}_$rep.log
    env $AB_ENV=$v timeout -k 10 200 python bench_decode.py --articles $a --batches 10 --warmup 2 > $L 2>&1 || { tail -20 $L; exit 1; }
    echo "$AB_ENV=$v articles=$a $(python -c "import json;d=json.loads(open('$L').read().strip().splitlines()[-1]);print(d['value'], d.get('ms_per_batch'))")"
  done; done; done ;;
train)
  if [ -n "$AB_K" ]; then
    timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$AB_K" \
      > $OUT/pytest.log 2>&1
    rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
  fi
  j() { python -c "import json;d=json.loads(open('$1').read().strip().splitlines()[-1]);print('$2', d['ms_per_step'], d['value'])"; }
  i=0
  for v in ${AB_VALUES:-1 0 1 0}; do
    i=$((i+1))
    env $AB_ENV=$v timeout -k 10 300 python bench.py --decode-batches 0 --steps 40 --warmup 5 > $OUT/b$i.log 2>&1 \
      || { tail -20 $OUT/b$i.log; exit 1; }
    j $OUT/b$i.log "B=256 $AB_ENV=$v"
    if [ -n "$AB_CFG5" ]; then
      env $AB_ENV=$v timeout -k 10 300 python bench.py --hidden 512 --layers 2 --enc 800 --batch 512 --steps 4 \
        --warmup 1 --decode-batches 0 > $OUT/c$i.log 2>&1 || { tail -20 $OUT/c$i.log; exit 1; }
      j $OUT/c$i.log "cfg5 B=512 $AB_ENV=$v"
    fi
  done ;;
*) echo "unknown: $1"; exit 2 ;;
esac
