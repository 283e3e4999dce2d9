"""Per-kernel VGPR / AGPR / spill / occupancy from hipcc -Rpass-analysis=kernel-resource-usage
output on stdin: python tools/resusage.py [FILTER] < remarks.txt"""
import re
import sys

flt = sys.argv[1] if len(sys.argv) > 1 else ""
cur, rows = None, []
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    for k in ("VGPRs", "AGPRs", "ScratchSize \\[bytes/lane\\]", "Occupancy \\[waves/SIMD\\]", "LDS Size \\[bytes/block\\]"):
        m = re.search(k + r": (\d+)", line)
        if m and cur is not None:
            cur[k.split()[0].split("\\")[0]] = int(m.group(1))
for r in rows:
    if flt in r["name"]:
        print(f'{r.get("VGPRs", "?"):>4} {r.get("AGPRs", "?"):>4} scratch {r.get("ScratchSize", "?"):>5} '
              f'occ {r.get("Occupancy", "?")} lds {r.get("LDS", "?"):>6}  {r["name"][:110]}')
