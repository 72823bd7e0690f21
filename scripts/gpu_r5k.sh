#!/bin/bash
# round 5 closing profiles: LSTM per-step latency vs team count (H = 256 / 512), headline kernel
# window, phase breakdown, decode kernel stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-r5k}; mkdir -p $OUT
export TMPDIR=/tmp
step() { local n=$1; shift; echo "== $n"; timeout -k 10 ${T:-300} "$@" > $OUT/$n.log 2>&1; local rc=$?; tail -${TL:-3} $OUT/$n.log; return $rc; }
TL=8 step lstm python -u tools/lstm_micro.py 256:64:400 256:128:400 256:256:400 256:512:400 512:128:400 512:256:400 || exit 1
TL=2 step ph python -u tools/phase_micro.py || exit 1
T=400 step tr rocprofv3 --kernel-trace -d $OUT/tr -o run --output-format csv -- python3 bench.py --steps 3 --warmup 2 --decode-batches 0 --config5-steps 0 || exit 1
python scripts/kwin.py $OUT/tr/run_kernel_trace.csv 3 40 > $OUT/train_kwin_b256.txt; head -3 $OUT/train_kwin_b256.txt
rm -rf $OUT/tr
T=300 step dp rocprofv3 --kernel-trace --stats -d $OUT/p1 -o run --output-format csv -- python3 bench_decode.py --batches 2 || exit 1
python scripts/kstats.py $OUT/p1/run_kernel_stats.csv 3 16 > $OUT/decode_h256_kstats.txt; head -12 $OUT/decode_h256_kstats.txt
rm -rf $OUT/p1
echo done
