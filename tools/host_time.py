"""Host-side enqueue time of the bench step (config 2): wall time of eng.step() calls that only
queue work, against the synchronized per-step time.

    python tools/host_time.py [--steps 3]
"""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "multimodal-ssl-avmnist_amd")):
    sys.path.insert(0, p)

import torch  # noqa: E402

from bench import synthetic_pool  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=3)
    a = ap.parse_args()
    from avdino import ops
    from avdino.engine import Hyper, MultiCentralEngine
    from avdino.params import ParamStore
    from avdino.spec import multimodal_dino_sd
    store = ParamStore(multimodal_dino_sd("mse", 256, 256, 128), "cuda", seed=0)
    eng = MultiCentralEngine(store, "mse", 256, 256, 128, Hyper(), act_dtype=torch.bfloat16)
    pool = synthetic_pool(2, 1024, 2, 4, "cuda", 1)
    for i in range(3):
        eng.step(pool[i % 2])
    torch.cuda.synchronize()
    n0 = ops.CALLS if hasattr(ops, "CALLS") else None
    t0 = time.perf_counter()
    for i in range(a.steps):
        eng.step(pool[i % 2])
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"host enqueue {1e3 * (t1 - t0) / a.steps:.2f} ms/step, wall {1e3 * (t2 - t0) / a.steps:.2f} ms/step")


if __name__ == "__main__":
    main()
