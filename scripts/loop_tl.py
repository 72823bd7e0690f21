"""Per-kernel timeline of a window of decoder-loop steps in the last training step of a rocprofv3
kernel_trace.csv: for each dispatch its queue, start offset and duration (us), so the overlap of
the row-group streams and the launch gaps of the per-step chain can be read off.
usage: loop_tl.py <kernel_trace.csv> <kernel substring> [first occurrence, default 40] [count, 24]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "adagrad_kernel" in r["Kernel_Name"]]
last = rows[idx[-2] + 1: idx[-1] + 1] if len(idx) >= 2 else rows
key = sys.argv[2]
first = int(sys.argv[3]) if len(sys.argv) > 3 else 40
count = int(sys.argv[4]) if len(sys.argv) > 4 else 24
hits = [i for i, r in enumerate(last) if key in r["Kernel_Name"]]
if len(hits) <= first:
    sys.exit(f"only {len(hits)} dispatches of {key}")
a = hits[first]
win = last[a: a + count * 3]
t0 = int(win[0]["Start_Timestamp"])
qcol = "Queue_Id" if "Queue_Id" in win[0] else ("Stream_Id" if "Stream_Id" in win[0] else None)
prev_end = {}
for r in win:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    q = r.get(qcol, "?") if qcol else "?"
    gap = (s - prev_end[q]) / 1e3 if q in prev_end else float("nan")
    prev_end[q] = e
    print(f"q{q:>3} +{(s - t0) / 1e3:9.2f} us  {((e - s) / 1e3):7.2f} us  gap {gap:6.2f}  {r['Kernel_Name'][:70]}")
