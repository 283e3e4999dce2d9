"""Summarise rocprofv3 --pmc counter_collection.csv files per (kernel, grid): average counter
values per dispatch; wave-cycle breakdown when the SQ counters are present.

    python tools/pmc_kernels.py <dir> [<dir> ...]
"""
import collections
import csv
import glob
import os
import sys

acc = collections.defaultdict(lambda: collections.defaultdict(list))
for d in sys.argv[1:]:
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        per = {}
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:70]
            key = (name, r.get("Grid_Size", r.get("Grid_Size_X", "")))
            k2 = (int(r["Dispatch_Id"]), r["Counter_Name"])
            per.setdefault(k2, [key, 0.0])[1] += float(r["Counter_Value"])
        for (disp, cn), (key, v) in per.items():
            acc[key][cn].append(v)
names = sorted({c for k in acc for c in acc[k]})
print("kernel [grid] | " + " | ".join(names))
for key, cs in sorted(acc.items(), key=lambda kv: -sum(kv[1].get("SQ_WAVE_CYCLES", [0]))):
    vals = {c: sum(v) / len(v) for c, v in cs.items()}
    line = f"{key[0]} [{key[1]}] | " + " | ".join(f"{vals.get(c, float('nan')):.4g}" for c in names)
    wc = vals.get("SQ_WAVE_CYCLES")
    if wc:
        line += "  || wait %.0f%% issue-stall %.0f%% active %.0f%%" % (
            100 * vals.get("SQ_WAIT_ANY", 0) / wc, 100 * vals.get("SQ_WAIT_INST_ANY", 0) / wc,
            100 * vals.get("SQ_ACTIVE_INST_ANY", 0) / wc)
    print(line)
