"""Summarise a rocprofv3 --stats kernel_stats.csv: top kernels, per-step time."""
import csv
import sys

path, steps = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 13
rows = list(csv.DictReader(open(path)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:int(sys.argv[3]) if len(sys.argv) > 3 else 25]:
    print(f"{float(r['TotalDurationNs'])/1e6:8.2f} ms {float(r['Percentage']):5.1f}% n={r['Calls']:>5} "
          f"avg={float(r['AverageNs'])/1e3:8.1f}us {r['Name'][:100]}")
print(f"total {tot/1e6:.1f} ms, per step {tot/1e6/steps:.2f} ms")
