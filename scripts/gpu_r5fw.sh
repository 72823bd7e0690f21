#!/bin/bash
# round 5: waves per workgroup of the training projected attention forward at A = 512 (TSAMD_FWDP_W, temporary A/B)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5fw; mkdir -p $OUT
export TMPDIR=/tmp
for r in 1 2; do for w in 16 12 8; do
  TSAMD_FWDP_W=$w timeout -k 10 200 python -u bench.py --decode-batches 0 --config5-steps 0 > $OUT/b${w}_$r.log 2>&1 || exit 1
  echo "w $w run $r $(grep -o '"ms_per_step": [0-9.]*' $OUT/b${w}_$r.log | head -1)"
done; done
echo done
