#!/bin/bash
# Dead decoder step skipping: tests, then B=256 and config #5 benches with and without it.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-skip}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "${PYTEST_K:-rowp or projected or skip_pad or bench_shape or config5_shape or row_split or deterministic}" > $OUT/pytest.log 2>&1
rc=$?; tail -4 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
j() { python -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); print('$2', d['ms_per_step'], d['value'], d.get('beam4_summaries_per_sec'))"; }
for p in 1 0; do
  timeout -k 10 300 env TSAMD_SKIP_PAD_STEPS=$p python bench.py --steps 20 --warmup 3 --decode-batches 0 > $OUT/b256_p$p.log 2>&1 || { tail -20 $OUT/b256_p$p.log; exit 1; }
  j $OUT/b256_p$p.log "B=256 skip=$p"
done
for p in 1 0; do
  timeout -k 10 400 env TSAMD_SKIP_PAD_STEPS=$p python bench.py --hidden 512 --layers 2 --enc 800 --batch 1024 --steps 3 --warmup 1 --decode-batches 0 > $OUT/c5_p$p.log 2>&1 || { tail -20 $OUT/c5_p$p.log; exit 1; }
  j $OUT/c5_p$p.log "config5 B=1024 skip=$p"
done
echo done
