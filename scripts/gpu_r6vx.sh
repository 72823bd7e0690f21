#!/bin/bash
# round 6: vocab_train X image at a 2-slot row pad (conflict-free ds_read_b128 groups): probes, PMC, tests, bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-r6vx}; mkdir -p $OUT
export TMPDIR=/tmp
for p in 0 2 7; do
  TSAMD_VT_PROBE=$p timeout -k 10 120 python tools/vocab_train_micro.py --rows 20480 --reps 1 > $OUT/p$p.jsonl 2>&1 || { tail -5 $OUT/p$p.jsonl; exit 1; }
  echo "probe=$p $(tail -1 $OUT/p$p.jsonl)"
done
timeout -k 10 120 python tools/vocab_train_micro.py --rows 20480 --hidden 512 --reps 1 > $OUT/h512.jsonl 2>&1 || exit 1
echo "H512 $(tail -1 $OUT/h512.jsonl)"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_IDX_ACTIVE --kernel-include-regex vocab_train -d $OUT/pmc -o run --output-format csv -- python3 tools/vocab_train_micro.py --reps 1 --iters 2 > $OUT/pmc.log 2>&1 || { tail -5 $OUT/pmc.log; exit 1; }
python scripts/pmc_sum.py $(find $OUT/pmc -name "*counter_collection.csv") | tee $OUT/pmc.txt
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_model.py tests/test_gpu_production.py \
  -k "fused_vocab_head or bench_shape_matches or config5_shape_matches or deterministic_mode" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --decode-batches 0 --config5-steps 0 > $OUT/b$i.log 2>&1 || { echo "bench failed"; tail -5 $OUT/b$i.log; exit 1; }
  python -c "import json;r=json.loads(open('$OUT/b$i.log').read().strip().splitlines()[-1]);print('bench', r['ms_per_step'], r.get('phase_ms_max_over_ranks'))"
done
timeout -k 10 400 python bench.py --steps 1 --warmup 1 --decode-batches 0 --config5-steps 4 > $OUT/c5.log 2>&1 || { echo "c5 failed"; tail -5 $OUT/c5.log; exit 1; }
python -c "import json;r=json.loads(open('$OUT/c5.log').read().strip().splitlines()[-1]);print('c5', r['config5_ms_per_step'])"
echo done
