#!/bin/bash
# decode A/B: env switch $AB_ENV in {0,1}, 64 and 128 articles, beam 4
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-decab}; mkdir -p $OUT
for rep in 1 2; do for v in 1 0; do for a in 64 128; do
  env $AB_ENV=$v timeout -k 10 200 python bench_decode.py --articles $a --batches 10 --warmup 2 > $OUT/d_${v}_${a}_$rep.log 2>&1 || { tail -20 $OUT/d_${v}_${a}_$rep.log; exit 1; }
  echo "$AB_ENV=$v articles=$a $(python -c "import json;d=json.loads(open('$OUT/d_${v}_${a}_$rep.log').read().strip().splitlines()[-1]);print(d['value'], d.get('ms_per_batch'))")"
done; done; done
