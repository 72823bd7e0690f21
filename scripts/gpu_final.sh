#!/bin/bash
# end-of-round check at the committed state: the whole GPU tier, smoke(), bench.py (N = 1)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-final}; mkdir -p $OUT
export TMPDIR=/tmp
step() { local n=$1; shift; echo "== $n"; timeout -k 10 ${T:-300} "$@" > $OUT/$n.log 2>&1; local rc=$?; tail -${TL:-3} $OUT/$n.log; return $rc; }
T=900 step tier python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread &&
step smoke python -u -c "import __graft_entry__ as g; g.smoke()" &&
T=600 step bench python -u bench.py
