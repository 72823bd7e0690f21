#!/bin/bash
# End-of-session numbers, part 2: per-phase wall times (B=256 and config #5), decode benches
# (64 / 128 articles), CLI training throughput (multi-process loader), streaming latency,
# rocprof kernel stats of config #5.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUTD:-final2}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python tools/phase_micro.py > $OUT/phase.log 2>&1 || { tail -20 $OUT/phase.log; exit 1; }
tail -1 $OUT/phase.log
timeout -k 10 300 python tools/phase_micro.py --batch 1024 --hidden 512 --enc 800 --layers 2 --iters 2 > $OUT/phase5.log 2>&1 || { tail -20 $OUT/phase5.log; exit 1; }
tail -1 $OUT/phase5.log
timeout -k 10 300 python bench_decode.py > $OUT/dec64.log 2>&1 || { tail -20 $OUT/dec64.log; exit 1; }
tail -1 $OUT/dec64.log | cut -c1-200
timeout -k 10 300 python bench_decode.py --articles 128 > $OUT/dec128.log 2>&1 || { tail -20 $OUT/dec128.log; exit 1; }
tail -1 $OUT/dec128.log | cut -c1-200
timeout -k 10 300 python bench_decode.py --hidden 512 --layers 2 --enc 800 --batches 6 > $OUT/dec_c5.log 2>&1 || { tail -20 $OUT/dec_c5.log; exit 1; }
tail -1 $OUT/dec_c5.log | cut -c1-200
timeout -k 10 400 python tools/cli_throughput.py --root /tmp/tsamd_cli --examples 20000 --steps 300 --workers 8 > $OUT/cli.log 2>&1 || { tail -20 $OUT/cli.log; exit 1; }
tail -1 $OUT/cli.log
timeout -k 10 300 python tools/cli_throughput.py --root /tmp/tsamd_cli --examples 20000 --steps 600 --workers 14 --host-only > $OUT/cli_host.log 2>&1 || { tail -20 $OUT/cli_host.log; exit 1; }
tail -1 $OUT/cli_host.log
timeout -k 10 400 python tools/stream_latency.py --requests 60 --interval-ms 50 --waits 0,20 > $OUT/lat.log 2>&1 || { tail -20 $OUT/lat.log; exit 1; }
grep '^{' $OUT/lat.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof5 -o run --output-format csv -- python3 bench.py --hidden 512 --layers 2 --enc 800 --batch 512 --steps 2 --warmup 1 --decode-batches 0 > $OUT/prof5.log 2>&1 || { tail -20 $OUT/prof5.log; exit 1; }
python scripts/kstats.py $OUT/prof5/run_kernel_stats.csv 5 30 > $OUT/cfg5_kstats.txt
echo done
