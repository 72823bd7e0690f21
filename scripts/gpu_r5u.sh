#!/bin/bash
# round 5: config #5 (batch 2048) by phase and by kernel on the current tree (FX, dot2, 4 groups)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5u; mkdir -p $OUT
export TMPDIR=/tmp
step() { local n=$1; shift; echo "== $n"; timeout -k 10 ${T:-300} "$@" > $OUT/$n.log 2>&1; local rc=$?; tail -${TL:-2} $OUT/$n.log; return $rc; }
#T=400 step ph python -u tools/phase_micro.py --batch 2048 --hidden 512 --enc 800 --layers 2 --iters 3 || exit 1
T=600 step c5tr rocprofv3 --kernel-trace -d $OUT/tr -o run --output-format csv -- python3 bench.py --hidden 512 --enc 800 --layers 2 --batch 2048 --steps 2 --warmup 2 --decode-batches 0 --config5-steps 0 || exit 1
python scripts/kwin.py $OUT/tr/run_kernel_trace.csv 2 45 > $OUT/cfg5_kwin.txt; head -3 $OUT/cfg5_kwin.txt
python scripts/kgaps.py $OUT/tr/run_kernel_trace.csv 2 30 > $OUT/cfg5_gaps.txt 2>&1; tail -32 $OUT/cfg5_gaps.txt
rm -rf $OUT/tr
echo done
