"""Timeline summary of one training step from a rocprofv3 kernel trace (``--kernel-trace``
CSV): the step between the last two optimizer launches, its wall time, the time at least one
kernel was running (union of the kernel intervals), and per kernel name the union of its
own intervals plus the time it was the ONLY kernel running (what shortening it would save at
most; concurrent row groups overlap their kernels).

  python tools/timeline.py gpurun_out/tl/prof/run_kernel_trace.csv [top]
"""
import csv
import sys
from collections import defaultdict


def union(iv):
    iv = sorted(iv)
    tot, cur_s, cur_e = 0, None, None
    for s, e in iv:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def main():
    path, top = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 25
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    opt = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith(("adagrad", "clip_adagrad"))]
    if len(opt) < 2:
        sys.exit("need two optimizer launches in the trace")
    seg = rows[opt[-2] + 1:opt[-1] + 1]
    iv = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in seg]
    t0, t1 = iv[0][0], max(e for _, e, _ in iv)
    busy = union([(s, e) for s, e, _ in iv])
    print(f"step wall {(t1 - t0) / 1e6:.3f} ms, some kernel running {busy / 1e6:.3f} ms, idle {(t1 - t0 - busy) / 1e6:.3f} ms, "
          f"{len(iv)} launches")
    # exclusive time: sweep over interval boundaries
    ev = []
    for k, (s, e, n) in enumerate(iv):
        ev.append((s, 1, k))
        ev.append((e, -1, k))
    ev.sort()
    active, last, excl = set(), None, defaultdict(int)
    for t, d, k in ev:
        if last is not None and len(active) == 1:
            excl[iv[next(iter(active))][2]] += t - last
        if d == 1:
            active.add(k)
        else:
            active.discard(k)
        last = t
    by = defaultdict(list)
    for s, e, n in iv:
        by[n].append((s, e))
    stats = sorted(((union(v), len(v), excl[n], n) for n, v in by.items()), reverse=True)
    print(f"{'union ms':>9} {'alone ms':>9} {'calls':>6}  kernel")
    for u, c, x, n in stats[:top]:
        print(f"{u / 1e6:9.3f} {x / 1e6:9.3f} {c:6d}  {n[:100]}")


if __name__ == "__main__":
    main()
