#!/bin/bash
# round 6: grouped decode encoder -- decode tests, bench_decode / bench.py decode A/B (TSAMD_DEC_GROUP_ENC 4 / 2 / 1)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-r6pe}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_pipeline.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for g in 4 2 1 4 2 1; do
  TSAMD_DEC_GROUP_ENC=$g timeout -k 10 300 python bench_decode.py --batches 8 > $OUT/dec_g$g.log 2>&1 || exit 1
  python -c "import json;r=json.loads(open('$OUT/dec_g$g.log').read().strip().splitlines()[-1]);print('group $g bench_decode', r['value'], r.get('ms_per_batch'))"
done
for g in 4 1; do
  TSAMD_DEC_GROUP_ENC=$g timeout -k 10 300 python bench.py --steps 3 --warmup 1 --config5-steps 0 > $OUT/bench_g$g.log 2>&1 || exit 1
  python -c "import json;r=json.loads(open('$OUT/bench_g$g.log').read().strip().splitlines()[-1]);print('group $g bench.py', r.get('beam4_summaries_per_sec'))"
done
echo done
