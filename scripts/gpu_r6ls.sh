#!/bin/bash
# round 6: persistent-LSTM LDS swizzle with the chunk bit-3 term (conflict-free MFMA fragment reads)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-r6ls}; mkdir -p $OUT
export TMPDIR=/tmp
[ -n "$SKIP_TESTS" ] || timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_lstm.py > $OUT/tests_lstm.log 2>&1 || { tail -30 $OUT/tests_lstm.log; exit 1; }
tail -1 $OUT/tests_lstm.log
[ -n "$SKIP_TESTS" ] || timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_production.py \
  -k "bench_shape_matches or config5_shape_matches or deterministic_mode or graph_replay_equals" > $OUT/tests_prod.log 2>&1 || { tail -30 $OUT/tests_prod.log; exit 1; }
tail -1 $OUT/tests_prod.log
timeout -k 10 300 python tools/lstm_bptt_stamps.py 512:1024:800 512:2048:800 > $OUT/stamps.jsonl 2>&1 || { tail -5 $OUT/stamps.jsonl; exit 1; }
python -c "
import json
for l in open('$OUT/stamps.jsonl'):
    if l.startswith('{'):
        r=json.loads(l); print(r['H'],r['B'],r['T'],'us',r['us_plain'],'per step',r['us_per_step_plain'],r['phases_cycles'])
"
timeout -s KILL 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-include-regex lstm -d $OUT/pmc -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --decode-batches 0 --config5-steps 0 > $OUT/pmc.log 2>&1 || { tail -5 $OUT/pmc.log; exit 1; }
python scripts/pmc_sum.py $(find $OUT/pmc -name "*counter_collection.csv") | tee $OUT/pmc.txt
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --decode-batches 0 --config5-steps 0 > $OUT/b$i.log 2>&1 || { echo "bench failed"; tail -5 $OUT/b$i.log; exit 1; }
  python -c "import json;r=json.loads(open('$OUT/b$i.log').read().strip().splitlines()[-1]);print('bench', r['ms_per_step'], r.get('phase_ms_max_over_ranks'))"
done
timeout -k 10 400 python bench.py --steps 1 --warmup 1 --decode-batches 0 --config5-steps 4 > $OUT/c5.log 2>&1 || { echo "c5 failed"; tail -5 $OUT/c5.log; exit 1; }
python -c "import json;r=json.loads(open('$OUT/c5.log').read().strip().splitlines()[-1]);print('c5', r['config5_ms_per_step'])"
echo done
