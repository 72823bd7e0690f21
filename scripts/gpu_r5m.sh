#!/bin/bash
# round 5: the attn_bwd_rowp spill fix A/B material (gpu_r5l) followed by the closing run (gpu_r5final).
cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_r5l.sh || exit 1
bash scripts/gpu_r5final.sh
