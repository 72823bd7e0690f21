"""Per-kernel ms/step over the last N training steps of a rocprofv3 kernel_trace.csv (the
dispatches after the (N+1)-th last optimizer kernel up to the last one), so one-off work before
them (graph capture warm-up, blt_mm's candidate timing) is left out.
usage: kwin.py <kernel_trace.csv> <N> [top, default 40] [marker substring, default adagrad_kernel] [skip]
(skip: leave out the last `skip` steps, e.g. bench.py's phase-timed diagnostic steps)"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
n = int(sys.argv[2])
top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
mark = sys.argv[4] if len(sys.argv) > 4 else "adagrad_kernel"
idx = [i for i, r in enumerate(rows) if mark in r["Kernel_Name"]]
sk = int(sys.argv[5]) if len(sys.argv) > 5 else 0
win = rows[idx[-n - 1 - sk] + 1: idx[-1 - sk] + 1]
t0, t1 = int(win[0]["Start_Timestamp"]), int(win[-1]["End_Timestamp"])
agg = {}
for r in win:
    d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    a = agg.setdefault(r["Kernel_Name"], [0, 0])
    a[0] += 1
    a[1] += d
busy = sum(v[1] for v in agg.values())
print(f"last {n} steps: span {(t1 - t0) / 1e6 / n:.2f} ms/step, kernel busy {busy / 1e6 / n:.2f} ms/step "
      f"(kernels on concurrent streams overlap)")
for name, (c, d) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
    print(f"{d / 1e6 / n:8.3f} ms/step {c / n:7.1f} calls/step {d / c / 1e3:9.2f} us  {name[:90]}")
