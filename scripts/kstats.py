"""Summarise a rocprofv3 kernel_stats.csv: per-step ms by kernel."""
import csv, sys
path, steps = sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
rows = list(csv.DictReader(open(path)))
tot = sum(float(r['TotalDurationNs']) for r in rows)
print(f"total {tot/1e6:.2f} ms  ({tot/1e6/steps:.2f} ms/step over {steps:g} steps)")
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:int(sys.argv[3]) if len(sys.argv) > 3 else 25]:
    print(f"{float(r['TotalDurationNs'])/1e6/steps:8.3f} ms/step {int(r['Calls'])/steps:7.0f} calls/step {float(r['AverageNs'])/1e3:8.2f} us  {r['Name'][:90]}")
