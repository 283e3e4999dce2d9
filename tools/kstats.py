"""Top kernels of a rocprofv3 kernel_stats.csv: python tools/kstats.py FILE [N] [FILTER]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 16
flt = sys.argv[3] if len(sys.argv) > 3 else ""
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:n]:
    if flt in r["Name"]:
        print(f'{float(r["TotalDurationNs"]) / 1e6:9.2f}ms {int(r["Calls"]):6d} '
              f'{float(r["AverageNs"]) / 1e3:8.1f}us  {r["Name"][:100]}')
print(f"total {tot / 1e6:.2f} ms")
