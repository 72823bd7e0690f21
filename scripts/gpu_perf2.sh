#!/bin/bash
# Config-5 bench + B=256 default-config bench and profile.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/perf2; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python bench.py --batch 256 --steps 10 > $OUT/b256.log 2>&1 || { tail -20 $OUT/b256.log; exit 1; }
tail -1 $OUT/b256.log
timeout -k 10 600 python bench.py --hidden 512 --enc 800 --layers 2 --batch 64 --steps 5 --warmup 2 > $OUT/c5_b64.log 2>&1 || { tail -20 $OUT/c5_b64.log; exit 1; }
tail -1 $OUT/c5_b64.log
timeout -k 10 600 python bench.py --hidden 512 --enc 800 --layers 2 --batch 256 --steps 5 --warmup 2 > $OUT/c5_b256.log 2>&1 || { tail -20 $OUT/c5_b256.log; exit 1; }
tail -1 $OUT/c5_b256.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --batch 256 --no-graph > $OUT/prof.log 2>&1; echo "prof rc=$?"
