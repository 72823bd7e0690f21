#!/bin/bash
# round 5: issue cost of v_dot2 bf16 unpack vs shift/and unpack (tools/micro/dot2_probe.cpp, prebuilt here)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5r; mkdir -p $OUT
timeout -k 10 60 ./tools/micro/dot2_probe > $OUT/dot2.jsonl 2>&1; rc=$?; cat $OUT/dot2.jsonl; exit $rc
