#!/bin/bash
# round-4: restored round-3 decode vocab head (numerics + decode bench), 32-row BPTT variant sweep,
# then the deterministic-mode divergence hunt (whole GPU tier, then two deterministic trainers
# with 4 decoder row-group streams, per-step buffer checksums with row / column locations)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-r4g}; mkdir -p $OUT
export TMPDIR=/tmp
step() { local n=$1; shift; echo "== $n"; timeout -k 10 ${T:-300} "$@" > $OUT/$n.log 2>&1; local rc=$?; tail -${TL:-3} $OUT/$n.log; return $rc; }
step vtest python -u -m pytest tests/test_gpu_decode.py -x -q --timeout 100 --timeout-method thread &&
step dec python -u bench_decode.py --batches 10 &&
step dec5 python -u bench_decode.py --batches 6 --hidden 512 --layers 2 --enc 800 &&
for v in 0 1 2 3 4 5; do
  TSAMD_BWD32_VARIANT=$v step bwd32_v$v python -u tools/lstm_micro.py 512:1024:800 || exit 1
done &&
DSQ_SPLIT=4 T=1000 step det python -u tools/det_seq_after_suite.py
