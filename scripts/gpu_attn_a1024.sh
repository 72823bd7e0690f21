set -e
for full in "" 1; do for v in 0 2 4 5; do MICRO_FULL=$full TSAMD_ATTN_P4K2=$v timeout -k 10 120 python tools/attn_bwd_a1024_micro.py >> gpurun_out/a1024.jsonl; done; done
