"""One step of a rocprofv3 kernel trace as a per-stream timeline: each launch's start offset,
duration and stream, plus busy time per stream and the time no stream is busy (gaps).

    python tools/timeline.py run_kernel_trace.csv [--step K] [--steps-total N]
Steps are delimited by the Adam launch (one per step)."""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--step", type=int, default=-2, help="which step (python index over steps)")
    ap.add_argument("--marker", default="adam_kernel")
    ap.add_argument("--top", type=int, default=0, help="print only the N longest launches")
    a = ap.parse_args()
    rows = []
    for r in csv.DictReader(open(a.trace)):
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
        name = name.split("(")[0][:90]
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Stream_Id"], r["Queue_Id"], name,
                     r["Grid_Size_X"]))
    rows.sort()
    marks = [i for i, r in enumerate(rows) if a.marker in r[4]]
    # a step = from the launch after the previous loss's step end to the next loss; use loss-to-loss
    i0, i1 = marks[a.step - 1], marks[a.step]
    seg = rows[i0:i1]
    t0 = seg[0][0]
    busy = {}
    for s, e, st, q, n, g in seg:
        busy.setdefault(st, 0)
        busy[st] += e - s
    # union of busy intervals
    iv = sorted((s, e) for s, e, *_ in seg)
    tot, cs, ce = 0, iv[0][0], iv[0][1]
    for s, e in iv[1:]:
        if s > ce:
            tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    tot += ce - cs
    span = seg[-1][1] - t0
    print(f"step span {span / 1e3:.1f} us, any-stream busy {tot / 1e3:.1f} us, idle {(span - tot) / 1e3:.1f} us")
    for st, b in busy.items():
        print(f"  stream {st}: busy {b / 1e3:.1f} us")
    lst = seg if not a.top else sorted(seg, key=lambda r: r[0] - r[1])[:a.top]
    for s, e, st, q, n, g in sorted(lst):
        print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  s{st} q{q}  {n} [{g}]")


if __name__ == "__main__":
    main()
