"""Per-launch timing of the bench step's kernels at bench shapes: runs one config-2 step to
populate every workspace, then replays each instrumented launch (same pointers/shapes) R times
between HIP events on the launching stream and prints avg us, achieved GB/s and TFLOP/s.

    python tools/opbench.py [--batch 1024] [--dtype bf16] [--reps 10] [--filter cl_conv]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "multimodal-ssl-avmnist_amd")):
    sys.path.insert(0, p)

import torch  # noqa: E402

from bench import synthetic_pool  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--filter", default="")
    a = ap.parse_args()
    from avdino import ops
    from avdino.engine import Hyper, MultiCentralEngine
    from avdino.params import ParamStore
    from avdino.spec import multimodal_dino_sd
    act = torch.bfloat16 if a.dtype == "bf16" else torch.float32
    store = ParamStore(multimodal_dino_sd("mse", 256, 256, 128), "cuda", seed=0)
    eng = MultiCentralEngine(store, "mse", 256, 256, 128, Hyper(), act_dtype=act)
    pool = synthetic_pool(1, a.batch, 2, 4, "cuda", 1)
    eng.step(pool[0])
    ops.TIMER = ops.KernelTimer()
    eng.step(pool[0])
    torch.cuda.synchronize()
    fns = ops.TIMER.fns
    calls = {k: v["calls"] for k, v in ops.TIMER.summary().items()}
    ops.TIMER = None
    rows = []
    for key, (fn, nb, fl) in fns.items():
        if a.filter and a.filter not in key:
            continue
        fn()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(a.reps):
            fn()
        e.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(e) * 1e3 / a.reps
        # roofline time of the launch: max(bytes / 8 TB/s, flops / 2.5 PF/s (bf16) or 157 TF/s)
        roof = max(nb / 8e6, fl / (2.5e9 if act == torch.bfloat16 else 157e6))
        rows.append((us * calls.get(key, 1), us, calls.get(key, 1), key, nb / us / 1e3, fl / us / 1e6,
                     roof))
    tot = sum(r[0] for r in rows)
    troof = sum(r[6] * r[2] for r in rows)
    print("  per-step    us/launch  calls   share    GB/s    TF/s   roof us  x-roof  key")
    for st, us, n, key, gbs, tfs, roof in sorted(rows, reverse=True):
        print(f"{st:9.1f} us {us:9.1f} {n:5d} {100 * st / tot:6.1f}%  {gbs:7.0f} {tfs:7.1f} "
              f"{roof:8.1f} {us / max(roof, 1e-3):7.2f}  {key}")
    print(f"serial step (sum over launches x calls): {tot / 1e3:.3f} ms; roofline sum {troof / 1e3:.3f} ms")


if __name__ == "__main__":
    main()
