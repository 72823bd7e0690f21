#!/bin/bash
# A/B of the attention query projection fused into the row forward kernel (TSAMD_FUSED_SPROJ):
# GPU tests of the touched paths, then B = 256 and config #5 benches with and without it.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-sproj}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "sproj or fwd_row or production or graph or model" > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
j() { python -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); print('$2', d['ms_per_step'], d['value'])"; }
i=0
for v in 1 0 1 0; do
  i=$((i+1))
  TSAMD_FUSED_SPROJ=$v timeout -k 10 300 python bench.py --decode-batches 0 --steps 40 --warmup 5 > $OUT/b$i.log 2>&1 || { tail -20 $OUT/b$i.log; exit 1; }
  j $OUT/b$i.log "B=256 fused_sproj=$v"
done
for v in 1 0; do
  i=$((i+1))
  TSAMD_FUSED_SPROJ=$v timeout -k 10 300 python bench.py --hidden 512 --layers 2 --enc 800 --batch 512 --steps 4 --warmup 1 --decode-batches 0 > $OUT/b$i.log 2>&1 || { tail -20 $OUT/b$i.log; exit 1; }
  j $OUT/b$i.log "cfg5 B=512 fused_sproj=$v"
done
echo done
