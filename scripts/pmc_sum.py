"""Average rocprofv3 counter_collection.csv values per (kernel, counter)."""
import collections, csv, sys
acc = collections.defaultdict(lambda: [0.0, 0])
for path in sys.argv[1:]:
    for r in csv.DictReader(open(path)):
        k = (r["Kernel_Name"][:60], r["Counter_Name"])
        acc[k][0] += float(r["Counter_Value"]); acc[k][1] += 1
by_k = collections.defaultdict(dict)
for (k, c), (s, n) in acc.items():
    by_k[k][c] = s / n
for k, cs in sorted(by_k.items()):
    print(k, " ".join(f"{c}={v:.4g}" for c, v in sorted(cs.items())))
