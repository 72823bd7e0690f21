#!/bin/bash
# hipBLASLt solution sweep for the config #5 encoder GEMM shapes, beside torch's own numbers
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-blt}; mkdir -p $OUT
export TMPDIR=/tmp
hipcc --offload-arch=gfx950 -O2 -std=c++17 tools/micro/hipblaslt_probe.cpp -lhipblaslt -o /tmp/hipblaslt_probe &&
echo "== torch" && timeout -k 10 300 python3 tools/gemm_c5.py > $OUT/torch.jsonl 2> $OUT/torch.err && cat $OUT/torch.jsonl &&
echo "== probe" && timeout -k 10 700 /tmp/hipblaslt_probe 819200 ${BUDGET:-40} > $OUT/probe.jsonl 2> $OUT/probe.err; rc=$?
cat $OUT/probe.jsonl; tail -3 $OUT/probe.err; exit $rc
