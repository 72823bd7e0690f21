#!/bin/bash
# round-4 timing experiment: the 16-row BPTT without its dz stores (TSAMD_LSTM_NODZ=1, wrong
# results) -- how much of the step the store traffic's vmcnt coupling costs
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-r4q}; mkdir -p $OUT
export TMPDIR=/tmp
step() { local n=$1; shift; echo "== $n"; timeout -k 10 ${T:-300} "$@" > $OUT/$n.log 2>&1; local rc=$?; tail -${TL:-3} $OUT/$n.log; return $rc; }
step m0 python -u tools/lstm_micro.py 256:256:400 512:256:400 256:64:400 &&
TSAMD_LSTM_NODZ=1 step m1 python -u tools/lstm_micro.py 256:256:400 512:256:400 256:64:400 &&
step m0b python -u tools/lstm_micro.py 256:256:400 512:256:400 256:64:400 &&
TSAMD_LSTM_NODZ=1 step m1b python -u tools/lstm_micro.py 256:256:400 512:256:400 256:64:400
