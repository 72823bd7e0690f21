#!/bin/bash
# round 6: model oracle tests (new gradient bounds, wgrad_tt at config #5) + bench with the fixed
# GEMM table vs the timed "auto" dispatch
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-r6n}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_production.py tests/test_gpu_model.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
s=$(date +%s); timeout -k 10 600 python bench.py > $OUT/bench_table.log 2>&1 || { tail -20 $OUT/bench_table.log; exit 1; }
echo "bench wall $(( $(date +%s) - s )) s"; tail -1 $OUT/bench_table.log > $OUT/bench_table.json
TSAMD_GEMM_BT=auto timeout -k 10 600 python bench.py > $OUT/bench_auto.log 2>&1 || { tail -20 $OUT/bench_auto.log; exit 1; }
tail -1 $OUT/bench_auto.log > $OUT/bench_auto.json
python - <<'PY'
import json,os
o=os.environ.get("OUTD","r6n")
for n in ("table","auto"):
    r=json.load(open(f"gpurun_out/{o}/bench_{n}.json"))
    c=r["config"]
    print(n, r["value"], r["ms_per_step"], "c5", r.get("config5_tokens_per_sec"), r.get("config5_ms_per_step"),
          "dec", r.get("beam4_summaries_per_sec"), "c5dec", r.get("config5_beam4_summaries_per_sec"),
          "picks", c["gemm_dispatch"]["gemm_bt"], "/", c["gemm_dispatch"]["shapes"])
PY
echo done
