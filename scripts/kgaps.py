"""Concurrency of the kernels in the last N training steps of a rocprofv3 kernel_trace.csv (same
window as kwin.py): time with 0 / 1 / 2 / 3 / 4+ kernels running, and per kernel name the time it
runs alone (nothing else on the GPU) and the time it shares the GPU, ms per step.
Idle intervals (no kernel running) are also grouped by (kernel that ended last -> kernel that
starts next): the bubbles of the step by where they sit.
usage: kgaps.py <kernel_trace.csv> <N> [top, default 25] [marker substring, default adagrad_kernel] [skip]
(skip: leave out the last `skip` steps, e.g. bench.py's phase-timed diagnostic steps)"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
n = int(sys.argv[2])
top = int(sys.argv[3]) if len(sys.argv) > 3 else 25
mark = sys.argv[4] if len(sys.argv) > 4 else "adagrad_kernel"
idx = [i for i, r in enumerate(rows) if mark in r["Kernel_Name"]]
sk = int(sys.argv[5]) if len(sys.argv) > 5 else 0
win = rows[idx[-n - 1 - sk] + 1: idx[-1 - sk] + 1]
ev = []
for k, r in enumerate(win):
    ev.append((int(r["Start_Timestamp"]), 1, k))
    ev.append((int(r["End_Timestamp"]), -1, k))
ev.sort()
active, last = set(), ev[0][0]
hist = [0] * 5
idle, last_end = {}, None  # (ended -> starts) -> [ms, count]
alone, shared = {}, {}
for t, kind, k in ev:
    dt = t - last
    if dt > 0:
        hist[min(len(active), 4)] += dt
        for a in active:
            nm = win[a]["Kernel_Name"][:80]
            (alone if len(active) == 1 else shared)[nm] = (alone if len(active) == 1 else shared).get(nm, 0) + dt
    if kind == 1:
        if not active and last_end is not None and t > last_end[0]:
            key = (win[last_end[1]]["Kernel_Name"][:40], win[k]["Kernel_Name"][:40])
            e = idle.setdefault(key, [0, 0])
            e[0] += t - last_end[0]
            e[1] += 1
        active.add(k)
    else:
        active.discard(k)
        if not active:
            last_end = (t, k)
    last = t
span = ev[-1][0] - ev[0][0]
print(f"span {span / 1e6 / n:.2f} ms/step; kernels running: " +
      ", ".join(f"{c}{'+' if c == 4 else ''}: {h / 1e6 / n:.2f}" for c, h in enumerate(hist)) + " ms/step")
names = sorted(set(alone) | set(shared), key=lambda x: -(alone.get(x, 0) + shared.get(x, 0)))
print("   alone   shared  (ms/step)")
for nm in names[:top]:
    print(f"{alone.get(nm, 0) / 1e6 / n:8.3f} {shared.get(nm, 0) / 1e6 / n:8.3f}  {nm}")
print("idle (ms/step, gaps/step, mean us): kernel that ended -> kernel that starts")
for (a, b), (d, c) in sorted(idle.items(), key=lambda kv: -kv[1][0])[:top]:
    print(f"{d / 1e6 / n:8.3f} {c / n:7.1f} {d / c / 1e3:8.2f}  {a} -> {b}")
