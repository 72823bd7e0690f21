#!/bin/bash
# deterministic-mode divergence hunt: the GPU tier (minus the deterministic test), then two
# deterministic GraphTrainers with 4 decoder row-group streams in the same process, per-step
# buffer checksums (tools/det_seq_after_suite.py)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-det}; mkdir -p $OUT
export TMPDIR=/tmp
DSQ_SPLIT=${SPLIT:-4} timeout -k 10 1000 python -u tools/det_seq_after_suite.py ${ARGS} > $OUT/det.log 2>&1; rc=$?
grep -E "suite rc|step" $OUT/det.log | tail -8
exit $rc
