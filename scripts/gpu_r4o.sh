#!/bin/bash
# round-4: BPTT dz stores issued before the hand-off (TSAMD_LSTM_EARLY_DZ) -- numerics, then timing A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-r4o}; mkdir -p $OUT
export TMPDIR=/tmp
step() { local n=$1; shift; echo "== $n"; timeout -k 10 ${T:-300} "$@" > $OUT/$n.log 2>&1; local rc=$?; tail -${TL:-3} $OUT/$n.log; return $rc; }
TSAMD_LSTM_EARLY_DZ=1 step lstm_early python -u -m pytest tests/test_gpu_lstm.py -x -q --timeout 100 --timeout-method thread &&
step m0 python -u tools/lstm_micro.py 256:256:400 512:256:400 512:1024:800 &&
TSAMD_LSTM_EARLY_DZ=1 step m1 python -u tools/lstm_micro.py 256:256:400 512:256:400 512:1024:800 &&
step m0b python -u tools/lstm_micro.py 256:256:400 512:256:400 512:1024:800 &&
TSAMD_LSTM_EARLY_DZ=1 step m1b python -u tools/lstm_micro.py 256:256:400 512:256:400 512:1024:800 &&
step smoke python -u -c "import __graft_entry__ as g; g.smoke()"
