#!/bin/bash
# same-box A/B of two in-tree library builds: TSAMD_C_LIB=_C_ab.so (A) vs _C.so (B), headline bench
# alternating, then config #5
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-r6ab}; mkdir -p $OUT
i=0
for lib in _C_ab.so _C.so _C_ab.so _C.so _C_ab.so _C.so; do
  i=$((i+1))
  TSAMD_C_LIB=$lib timeout -k 10 300 python bench.py --steps 20 --warmup 5 --decode-batches 0 --config5-steps 0 > $OUT/b${i}_$lib.log 2>&1 || { echo "bench failed"; tail -5 $OUT/b${i}_$lib.log; exit 1; }
  python -c "import json;r=json.loads(open('$OUT/b${i}_$lib.log').read().strip().splitlines()[-1]);print('$lib', r['ms_per_step'], r.get('phase_ms_max_over_ranks'))"
done
if [ -z "$NO_C5" ]; then
for lib in _C_ab.so _C.so; do
  TSAMD_C_LIB=$lib timeout -k 10 400 python bench.py --steps 1 --warmup 1 --decode-batches 0 --config5-steps 4 > $OUT/c5_$lib.log 2>&1 || { echo "c5 failed"; tail -5 $OUT/c5_$lib.log; exit 1; }
  python -c "import json;r=json.loads(open('$OUT/c5_$lib.log').read().strip().splitlines()[-1]);print('c5 $lib', r['config5_ms_per_step'])"
done
fi
echo done
