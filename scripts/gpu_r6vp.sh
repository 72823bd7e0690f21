#!/bin/bash
# round 6: vocab_train pass-1 probes (TSAMD_VT_PROBE bits: 1 no X loads after the first unit, 2 no softmax
# epilogue, 4 no per-unit barrier) at the bench shape (20480 live rows, H = 256)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-r6vp}; mkdir -p $OUT
for p in 0 1 2 3 4 5 6 7 0; do
  TSAMD_VT_PROBE=$p timeout -k 10 120 python tools/vocab_train_micro.py --rows 20480 --reps 1 > $OUT/p$p.jsonl 2>&1 || { tail -5 $OUT/p$p.jsonl; exit 1; }
  echo "probe=$p $(tail -1 $OUT/p$p.jsonl)"
done
