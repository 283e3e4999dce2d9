"""Time the device data path (avd_augment_views) on one config-2 batch: B=1024 pairs, 2 global +
4 local views of both modalities plus the originals, against its HBM roofline.

Algorithmic bytes per launch = outputs written (4 B x H x W per view) + each source row read
once (H x W bytes per sample; later views of a sample hit L2).  Timed with HIP events on the
current stream around `iters` repetitions of the same launches; parameter draws (host) are
made once, outside the timed region, and reported separately."""
import json
import sys
import time

import numpy as np
import torch

sys.path.insert(0, "multimodal-ssl-avmnist_amd")
sys.path.insert(0, ".")

from avdino import augment as A  # noqa: E402
from avdino import ops  # noqa: E402


def main(B=1024, N=55000, iters=20):
    dev = torch.device("cuda")
    rng = np.random.default_rng(0)
    src = {"image": torch.from_numpy(rng.integers(0, 256, (N, 784), dtype=np.uint8)).to(dev),
           "audio": torch.from_numpy(rng.integers(0, 256, (N, 12544), dtype=np.uint8)).to(dev)}
    lut = torch.arange(256, dtype=torch.float32, device=dev) / 255.0
    idx = rng.choice(N, B, replace=False)
    ch = A.default_chains()
    plan = []
    t0 = time.perf_counter()
    for mod, HW in (("image", 28), ("audio", 112)):
        aug = A.ViewAugmenter(src[mod], lut, HW, HW, seed=1)
        for grp, V in (("global", 2), ("local", 4)):
            rec, gm = aug.records(ch[grp][mod], B, V)
            plan.append((aug, rec, gm, V, HW))
        ident = np.zeros((B, A.REC), np.float32)
        ident[:, 22] = -1
        plan.append((aug, ident, None, 1, HW))
    host_ms = (time.perf_counter() - t0) * 1e3
    staged = []
    for aug, rec, gm, V, HW in plan:
        staged.append((aug.src, torch.from_numpy(idx).to(dev), torch.from_numpy(rec).to(dev),
                       None if gm is None else torch.from_numpy(gm.view(np.int32)).to(dev), V, HW,
                       torch.empty((B, V, HW, HW), device=dev)))
    nbytes = sum(B * V * HW * HW * 4 + B * HW * HW for *_, V, HW, _ in staged)

    def run():
        for s, i, r, g, V, HW, out in staged:
            ops.augment_views(s, i, lut, r, g, 4, 7, V, HW, HW, out, 0)

    run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        run()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / iters
    gbs = nbytes / (ms * 1e-3) / 1e9
    print(json.dumps({"what": "device augmentation, config-2 batch (B=1024, 2+4 views + originals, "
                      "both modalities, 6 launches)", "ms_per_batch": round(ms, 4),
                      "pairs_per_s": round(B / (ms * 1e-3), 1), "algorithmic_bytes": nbytes,
                      "achieved_GBps": round(gbs, 1), "peak_GBps": 8000.0,
                      "frac": round(gbs / 8000.0, 4), "host_param_draw_ms": round(host_ms, 2)}))


if __name__ == "__main__":
    main()
