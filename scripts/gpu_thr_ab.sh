#!/bin/bash
# stream transform throughput with blt_mm on / off (same box, alternating), plus bench_decode for each
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-thrab}; mkdir -p $OUT
export TMPDIR=/tmp
step() { local n=$1; shift; echo "== $n"; timeout -k 10 ${T:-300} "$@" > $OUT/$n.log 2>&1; local rc=$?; grep -h '^{' $OUT/$n.log | cut -c1-160; return $rc; }
step t_blt1 env TSAMD_BLT=1 python -u tools/stream_throughput.py --only transform &&
step t_blt0 env TSAMD_BLT=0 python -u tools/stream_throughput.py --only transform &&
step t_blt1b env TSAMD_BLT=1 python -u tools/stream_throughput.py --only transform &&
step t_blt0b env TSAMD_BLT=0 python -u tools/stream_throughput.py --only transform &&
step d_blt1 env TSAMD_BLT=1 python -u bench_decode.py --batches 10 &&
step d_blt0 env TSAMD_BLT=0 python -u bench_decode.py --batches 10
