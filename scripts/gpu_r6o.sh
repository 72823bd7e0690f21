#!/bin/bash
# round 6: wgrad_tt 4-wave (default) vs 8-wave kernel -- tests then micro
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-r6o}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm.py -m gpu -x -q --timeout 120 --timeout-method thread -k wgrad > $OUT/pytest.log 2>&1; rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/wgrad_tt_micro.py $MICRO_ARGS > $OUT/micro4.jsonl 2>&1 || { tail -5 $OUT/micro4.jsonl; exit 1; }
TSAMD_WGRAD_TT8=1 timeout -k 10 400 python tools/wgrad_tt_micro.py $MICRO_ARGS > $OUT/micro8.jsonl 2>&1 || { tail -5 $OUT/micro8.jsonl; exit 1; }
python - <<'PY'
import json,os
o=os.environ.get("OUTD","r6o")
for n in ("4","8"):
    for l in open(f"gpurun_out/{o}/micro{n}.jsonl"):
        if l.startswith("{"):
            r=json.loads(l); print(n, r["shape"], r["wgrad_tt_us"], r["wgrad_tt_TF"], "splitK", r["split_k_us"], r["split_k_TF"], "err", "%.1e"%r["err"], r["bitwise_repeat"])
PY
echo done
