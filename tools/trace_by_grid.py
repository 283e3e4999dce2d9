"""Kernel-trace summary grouped by (kernel, grid): per-shape launch averages, so the bench's
HIP-event timing of one launch shape can be checked against rocprofv3 (the --stats summary
averages every shape of a kernel together, e.g. student and teacher batches).

    python tools/trace_by_grid.py <dir>/run_kernel_trace.csv [steps] [top]
"""
import collections
import csv
import sys

path = sys.argv[1]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 13
top = int(sys.argv[3]) if len(sys.argv) > 3 else 30
d = collections.defaultdict(list)
for r in csv.DictReader(open(path)):
    name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
    key = (name.split("(")[0][:90], r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"],
           r["Workgroup_Size_X"])
    d[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
tot = sum(sum(v) for v in d.values())
print(f"{'total_ms':>9} {'calls':>6} {'avg_us':>9}  kernel [grid x,y,z / wg]")
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1]))[:top]:
    print(f"{sum(v) / 1e3:9.2f} {len(v):6d} {sum(v) / len(v):9.1f}  {k[0]} [{k[1]},{k[2]},{k[3]} / {k[4]}]")
print(f"all kernels {tot / 1e3:.1f} ms = {tot / 1e3 / steps:.2f} ms/step over {steps} steps")
