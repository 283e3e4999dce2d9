"""Phase timeline of the replayed (hipGraph) training step from in-graph marks (avd_mark): the
device real-time counter at each phase boundary on each stream, with no profiler attached.

    python tools/phase_marks.py [--mode mse] [--batch 1024] [--steps 8] [--no-graph]
Prints, for the last step, every mark (time since the step's first mark, stream, delta since the
previous mark on the same stream), then the step time from the marks."""
import argparse
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "multimodal-ssl-avmnist_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="mse")
    ap.add_argument("--batch", type=int, default=None)
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--workload", default="dino")
    ap.add_argument("--dtype", default="bf16")
    a = ap.parse_args()
    import bench
    from avdino import dist as avdist
    from avdino import ops
    dev = torch.device("cuda", 0)
    ns = argparse.Namespace(workload=a.workload, batch=a.batch, mode=a.mode, dtype=a.dtype, pipeline=False)
    eng, pool, B, workload, _ = bench.build_workload(ns, dev, torch.bfloat16, 1, 0, avdist)
    eng.use_graph = not a.no_graph
    ops.MARKS = ops.Marks(dev)
    times = []
    for i in range(a.steps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        eng.step(pool[i % len(pool)])
        e1.record()
        torch.cuda.synchronize()
        times.append(e0.elapsed_time(e1))
    marks = ops.MARKS.read()
    streams = {}
    for _n, s, _t in marks:
        streams.setdefault(s, len(streams))
    last = {}
    print(f"# {workload}; graph={eng.use_graph}; step ms (events) {[round(t, 3) for t in times]}")
    for n, s, t in sorted(marks, key=lambda m: m[2]):
        sid = streams[s]
        d = t - last.get(sid, 0.0)
        last[sid] = t
        print(f"{t:9.1f} us  s{sid}  +{d:8.1f}  {n}")
    print(f"# mark span {max(m[2] for m in marks):.1f} us over {len(marks)} marks")


if __name__ == "__main__":
    main()
