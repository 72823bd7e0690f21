#!/bin/bash
# Decoder row-group count A/B (phase wall times + bench) with the current attention path.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-split}; mkdir -p $OUT
export TMPDIR=/tmp
for s in ${SPLITS:-1 2 4 8}; do
  timeout -k 10 300 env TSAMD_SPLIT=$s ${EXTRA_ENV} python tools/phase_micro.py ${PHASE_ARGS} > $OUT/phase_s$s.log 2>&1 || { tail -20 $OUT/phase_s$s.log; exit 1; }
  echo "split=$s $(tail -1 $OUT/phase_s$s.log)"
done
for s in ${BENCH_SPLITS:-2 4}; do
  timeout -k 10 300 env TSAMD_SPLIT=$s ${EXTRA_ENV} python bench.py --steps 20 --warmup 3 --decode-batches 0 ${BENCH_ARGS} > $OUT/bench_s$s.log 2>&1 || { tail -20 $OUT/bench_s$s.log; exit 1; }
  echo "bench split=$s $(tail -1 $OUT/bench_s$s.log | cut -c1-160)"
done
echo done
