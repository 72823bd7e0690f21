#!/bin/bash
# linear2 k-batch A/B on one box: bench_decode with TSAMD_L2_KB=0 (batches of 4) / default, alternating
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-l2ab}; mkdir -p $OUT
export TMPDIR=/tmp
step() { local n=$1; shift; echo "== $n"; timeout -k 10 ${T:-300} "$@" > $OUT/$n.log 2>&1; local rc=$?; grep -h -o '"value": [0-9.]*' $OUT/$n.log | tr '\n' ' '; echo; return $rc; }
step kb4a env TSAMD_L2_KB=0 python -u bench_decode.py --batches 12 &&
step kbKa python -u bench_decode.py --batches 12 &&
step kb4b env TSAMD_L2_KB=0 python -u bench_decode.py --batches 12 &&
step kbKb python -u bench_decode.py --batches 12 &&
step c5_kb4 env TSAMD_L2_KB=0 python -u bench_decode.py --hidden 512 --layers 2 --enc 800 --batches 4 &&
step c5_kbK python -u bench_decode.py --hidden 512 --layers 2 --enc 800 --batches 4
