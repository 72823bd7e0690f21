#!/bin/bash
# round 6: LDS bank-conflict survey of every kernel of the headline training step (bench.py, 2 timed steps)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-pmc_lds}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT/run -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --decode-batches 0 --config5-steps 0 > $OUT/run.log 2>&1 || { tail -5 $OUT/run.log; exit 1; }
python scripts/pmc_sum.py $(find $OUT/run -name "*counter_collection.csv") > $OUT/lds.txt
python - <<'PY' "$OUT/lds.txt"
import re, sys
rows = []
for l in open(sys.argv[1]):
    m = dict(re.findall(r"(\w+)=([\d.e+-]+)", l))
    if "SQ_LDS_IDX_ACTIVE" in m and float(m["SQ_LDS_IDX_ACTIVE"]) > 0:
        rows.append((float(m.get("GRBM_GUI_ACTIVE", 0)), float(m["SQ_LDS_BANK_CONFLICT"]) / float(m["SQ_LDS_IDX_ACTIVE"]), l[:60]))
for g, f, k in sorted(rows, reverse=True)[:40]:
    print(f"{g:12.4g} conflict_share={f:.3f} {k}")
PY
echo done
