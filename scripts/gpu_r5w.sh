#!/bin/bash
# round 5: attention v / w_c gradients in the A = 1024 row backward (VW) -- op tests, model /
# production oracles, config #5 with TSAMD_VW_ROWP=1 / 0, headline
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5w; mkdir -p $OUT
export TMPDIR=/tmp
C5="--hidden 512 --enc 800 --layers 2 --batch 2048 --steps 5 --warmup 2 --decode-batches 0 --config5-steps 0"
step() { local n=$1; shift; echo "== $n"; timeout -k 10 ${T:-300} "$@" > $OUT/$n.log 2>&1; local rc=$?; tail -${TL:-2} $OUT/$n.log; return $rc; }
T=120 step attn python -u -m pytest tests/test_gpu_attention_ops.py -q -x --timeout 60 --timeout-method thread || exit 1
T=700 step orc python -u -m pytest tests/test_gpu_production.py tests/test_gpu_model.py -q -x --timeout 300 --timeout-method thread || exit 1
TL=0 step vw1 python -u bench.py $C5 || exit 1; grep -o '"ms_per_step": [0-9.]*' $OUT/vw1.log
TL=0 step vw0 env TSAMD_VW_ROWP=0 python -u bench.py $C5 || exit 1; grep -o '"ms_per_step": [0-9.]*' $OUT/vw0.log
TL=0 step vw1b python -u bench.py $C5 || exit 1; grep -o '"ms_per_step": [0-9.]*' $OUT/vw1b.log
TL=0 step vw0b env TSAMD_VW_ROWP=0 python -u bench.py $C5 || exit 1; grep -o '"ms_per_step": [0-9.]*' $OUT/vw0b.log
echo done
