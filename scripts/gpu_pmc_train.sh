#!/bin/bash
# HBM traffic per training kernel (FETCH_SIZE, WRITE_SIZE) at the B=256 bench shape.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmc_train; mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum -d $OUT/p1 -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 > $OUT/p1.log 2>&1 || { tail -5 $OUT/p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/p2 -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 > $OUT/p2.log 2>&1 || { tail -5 $OUT/p2.log; exit 1; }
python scripts/pmc_sum.py $(find $OUT/p1 -name "*counter_collection.csv") > $OUT/fetch.txt
python scripts/pmc_sum.py $(find $OUT/p2 -name "*counter_collection.csv") > $OUT/write.txt
cat $OUT/fetch.txt $OUT/write.txt | cut -c1-160
