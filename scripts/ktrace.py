"""Ordered kernel sequence of the last training step in a rocprofv3 kernel_trace.csv (the
dispatches after the second-to-last optimizer kernel up to the last one); consecutive
dispatches of the same kernel are collapsed (count, mean us, total us).
usage: ktrace.py <kernel_trace.csv> [marker substring, default adagrad_kernel]"""
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
mark = sys.argv[2] if len(sys.argv) > 2 else "adagrad_kernel"
idx = [i for i, r in enumerate(rows) if mark in r["Kernel_Name"]]
last = rows[idx[-2] + 1: idx[-1] + 1] if len(idx) >= 2 else rows
t0, t1 = int(last[0]["Start_Timestamp"]), int(last[-1]["End_Timestamp"])
busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in last)
print(f"{len(last)} dispatches in the last step; span {(t1 - t0) / 1e3:.1f} us, kernel busy {busy / 1e3:.1f} us "
      f"({100 * busy / max(1, t1 - t0):.1f}%)")
groups = []
for r in last:
    n = r["Kernel_Name"][:90]
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    if groups and groups[-1][0] == n:
        groups[-1][1] += 1; groups[-1][2] += d
    else:
        groups.append([n, 1, d])
for n, c, d in groups:
    print(f"{c:5d} x {d / c:9.2f} us = {d:9.1f} us  {n}")
