#!/bin/bash
# A/B of the deeper load batches in dec_cell_fwd / dec_bwd_dz (TSAMD_DEC_KB): decoder GPU tests,
# the per-step kernel micro-benchmark, then B = 256 train and beam-4 decode with and without.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-deckb}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "model or production or decode or graph" > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in 0 1; do
  TSAMD_DEC_KB=$v timeout -k 10 200 python tools/dec_kernels_micro.py --rows 128,256 --hidden 256,512 > $OUT/micro$v.log 2>&1 || { tail -20 $OUT/micro$v.log; exit 1; }
  echo "DEC_KB=$v"; grep '^{' $OUT/micro$v.log
done
j() { python -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); print('$2', d['ms_per_step'], d['value'], d.get('beam4_summaries_per_sec'))"; }
i=0
for v in 1 0 1 0; do
  i=$((i+1))
  TSAMD_DEC_KB=$v timeout -k 10 300 python bench.py --steps 40 --warmup 5 --decode-batches 10 > $OUT/b$i.log 2>&1 || { tail -20 $OUT/b$i.log; exit 1; }
  j $OUT/b$i.log "B=256 dec_kb=$v"
done
echo done
