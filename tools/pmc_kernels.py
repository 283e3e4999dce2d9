"""Per-kernel mean of every PMC counter in the rocprofv3 --pmc pass directories under DIR
(DIR/p*/…/run_counter_collection.csv).    python tools/pmc_kernels.py DIR [NAMELEN]
NAMELEN (default 60) = kernel-name prefix that keys the grouping; longer keys split template
instances."""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(root, nl=60):
    acc = defaultdict(lambda: defaultdict(list))
    files = sorted(glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True))
    # one pass written straight into DIR (rocprofv3 -d DIR -o run)
    files = files or sorted(glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True))
    for f in files:
        per = defaultdict(float)
        with open(f) as fh:
            for row in csv.DictReader(fh):
                per[(row["Kernel_Name"][:nl], row["Dispatch_Id"], row["Counter_Name"])] += float(row["Counter_Value"])
        for (k, _, c), v in per.items():
            acc[k][c].append(v)
    for k, cs in acc.items():
        print(k)
        for c, vs in sorted(cs.items()):
            print(f"   {c:28s} {sum(vs) / len(vs):16.4g}  (n={len(vs)})")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 60)
