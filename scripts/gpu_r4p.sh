#!/bin/bash
# round-4 final profiles: per-kernel stats of the train step (B = 256) and beam-4 decode, per-phase
# step breakdowns (B = 256, config #5 batch 1024)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-r4p}; mkdir -p $OUT
export TMPDIR=/tmp
step() { local n=$1; shift; echo "== $n"; timeout -k 10 ${T:-300} "$@" > $OUT/$n.log 2>&1; local rc=$?; tail -${TL:-3} $OUT/$n.log; return $rc; }
step tprof rocprofv3 --kernel-trace --stats -d $OUT/t -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --decode-batches 0 --config5-steps 0 &&
python scripts/kstats.py $OUT/t/run_kernel_stats.csv 13 40 > $OUT/train_kstats.txt &&
step dprof rocprofv3 --kernel-trace --stats -d $OUT/d -o run --output-format csv -- python3 bench_decode.py --batches 5 &&
python scripts/kstats.py $OUT/d/run_kernel_stats.csv 6 30 > $OUT/decode_kstats.txt &&
step ph256 python -u tools/phase_micro.py &&
step ph5 python -u tools/phase_micro.py --batch 1024 --hidden 512 --enc 800 --layers 2 --iters 3
