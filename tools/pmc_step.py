"""Whole-step HBM traffic and per-kernel MFMA counters from tools/gpu_pmc_step.sh's passes.

    python tools/pmc_step.py gpurun_out TAG > profiles/..._pmc_step.txt

Traffic per step = (sum over all dispatches of the 4-step run - the 1-step run) / 3 for
FETCH_SIZE and WRITE_SIZE (KiB).  FETCH_SIZE is reported raw and doubled (MI355X_MICROARCH.md:
on gfx950 it counts half the bytes of 16-B-per-lane streaming reads, which is how this
library's kernels read; other widths are uncalibrated), WRITE_SIZE as is.  MFMA: per kernel
name, SQ_VALU_MFMA_BUSY_CYCLES / SQ_BUSY_CYCLES and the bf16 MOPS, summed over one step."""
import csv
import glob
import json
import os
import sys


def rows(d):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    out = []
    for f in files:
        out += list(csv.DictReader(open(f)))
    return out


def total(d, counter):
    return sum(float(r["Counter_Value"]) for r in rows(d) if r["Counter_Name"] == counter)


def main():
    root, tag = sys.argv[1], sys.argv[2]
    res = {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        a = total(os.path.join(root, f"pmc_{c}_4_{tag}"), c)
        b = total(os.path.join(root, f"pmc_{c}_1_{tag}"), c)
        res[c] = (a - b) / 3 * 1024.0
    B = 1024
    fetch2 = 2 * res["FETCH_SIZE"]
    step = fetch2 + res["WRITE_SIZE"]
    print(f"per step: FETCH_SIZE raw {res['FETCH_SIZE'] / 1e9:.3f} GB, doubled {fetch2 / 1e9:.3f} GB; "
          f"WRITE_SIZE {res['WRITE_SIZE'] / 1e9:.3f} GB")
    print(f"per step traffic (2 x FETCH + WRITE): {step / 1e9:.3f} GB = {step / B / 1e6:.2f} MB/pair "
          f"(algorithmic model: 17.37 MB/pair, 17.79 GB/step)")
    json.dump({"step:mse": {"traffic_bytes": step / B, "fetch_raw_bytes_per_step": res["FETCH_SIZE"],
                            "write_bytes_per_step": res["WRITE_SIZE"], "unit": "bytes per pair"}},
              open(os.path.join(root, f"traffic_step_{tag}.json"), "w"), indent=1)
    def short(name):
        return name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:72]

    per = {}
    for r in rows(os.path.join(root, f"pmc_sq_{tag}")):
        d = per.setdefault(short(r["Kernel_Name"]), {})
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    dur = {}
    for f in glob.glob(os.path.join(root, f"pmc_sq_{tag}", "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            dur[k] = dur.get(k, 0.0) + (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    peak = 2.5e15
    print("\nper kernel over one counter run (2 warm-up + 1 step, eager, serialised by the counter "
          "pass): bf16 MFMA FLOPs = SQ_INSTS_VALU_MFMA_MOPS_BF16 x 512, over the kernels' summed "
          "duration, as a fraction of the 2.5 PFLOP/s dense bf16 peak; MFMA-busy cycles raw")
    print(f"{'TFLOP/s':>9} {'of peak':>8} {'time ms':>8} {'MOPS bf16':>11} {'MFMA busy':>11}  kernel")
    for k, d in sorted(per.items(), key=lambda kv: -kv[1].get("SQ_INSTS_VALU_MFMA_MOPS_BF16", 0))[:30]:
        fl = d.get("SQ_INSTS_VALU_MFMA_MOPS_BF16", 0) * 512
        t = dur.get(k, 0.0)
        tf = fl / t / 1e12 if t else 0.0
        print(f"{tf:9.1f} {tf * 1e12 / peak:8.3f} {t * 1e3:8.3f} {d.get('SQ_INSTS_VALU_MFMA_MOPS_BF16', 0):11.4g} "
              f"{d.get('SQ_VALU_MFMA_BUSY_CYCLES', 0):11.4g}  {k}")


if __name__ == "__main__":
    main()
