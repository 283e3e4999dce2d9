"""Time the device data path on config-2 batches (B=1024 pairs, 2 global + 4 local views of both
modalities plus the originals) and the real-data training step it feeds.

  collated_f32  host numpy parameter draws + avd_augment_views (f32 collated views) +
                avd_stage_views (f32 -> bf16 staged input): the round-1 path
  staged_bf16   avd_augment_records (device draws) + avd_augment_views_dt writing bf16 straight
                into the engine's staged view-major input (MultiModalAugmentation.stage)
  step_*        MultiCentralEngine (mse, bf16, graph replay) steps fed by staged_bf16 batches of
                a synthetic AVMNIST-shaped uint8 dataset resident in HBM (serially before each
                step, or prefetched: the next batch's augmentation on the data stream under the
                current step, engine.prefetch), vs the same engine on pre-built synthetic views
                (bench.py's input)

Algorithmic bytes of the staged path per batch: the staged bf16 views written once
(2 B x H x W x views) + each source row read once per modality.  Times from HIP events on the
current stream; one JSON line per measurement."""
import json
import sys
import time

import numpy as np
import torch

sys.path.insert(0, "multimodal-ssl-avmnist_amd")
sys.path.insert(0, ".")

from avdino import augment as A  # noqa: E402
from avdino import ops  # noqa: E402


def timed(fn, iters):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters, (time.perf_counter() - t0) * 1e3 / iters


def main(B=1024, N=55000, G=2, L=4, iters=20):
    dev = torch.device("cuda")
    rng = np.random.default_rng(0)
    src = {"image": torch.from_numpy(rng.integers(0, 256, (N, 784), dtype=np.uint8)).to(dev),
           "audio": torch.from_numpy(rng.integers(0, 256, (N, 12544), dtype=np.uint8)).to(dev)}
    lut = torch.arange(256, dtype=torch.float32, device=dev) / 255.0
    idx = rng.choice(N, B, replace=False)
    nv = G + L + 1
    x_img = torch.empty(nv * B * 784, dtype=torch.bfloat16, device=dev)
    x_aud = torch.empty(nv * B * 12544, dtype=torch.bfloat16, device=dev)

    def make_aug(device_params):
        aug = A.MultiModalAugmentation(G, L)
        return aug.bind(A.ViewAugmenter(src["image"], lut, 28, 28, seed=1, device_params=device_params),
                        A.ViewAugmenter(src["audio"], lut, 112, 112, seed=2, device_params=device_params))

    host = make_aug(False)

    def collated():
        gi, ga, li, la = host(idx)
        img = host.image.identity(idx)
        aud = host.audio.identity(idx)
        ops.stage_views(gi, G, li, L, img, B, 784, x_img)
        ops.stage_views(ga, G, la, L, aud, B, 12544, x_aud)

    devp = make_aug(True)

    def staged():
        devp.stage(idx, x_img, x_aud, True)

    nbytes = nv * B * (784 + 12544) * 2 + B * (784 + 12544)
    for name, fn in (("collated_f32", collated), ("staged_bf16", staged)):
        gpu_ms, wall_ms = timed(fn, iters)
        print(json.dumps({"bench": "augment_batch", "path": name, "B": B, "views": nv,
                          "gpu_ms": round(gpu_ms, 3), "wall_ms": round(wall_ms, 3),
                          "pairs_per_s": round(B / (max(gpu_ms, wall_ms) / 1e3), 1),
                          "staged_GBps": round(nbytes / (gpu_ms / 1e3) / 1e9, 1)}), flush=True)

    # the training step fed by the device data path vs pre-built synthetic views
    from avdino.engine import Hyper, MultiCentralEngine
    from avdino.params import ParamStore
    from avdino.spec import multimodal_dino_sd
    E, D, P = 256, 256, 128
    store = ParamStore(multimodal_dino_sd("mse", E, D, P), dev, seed=0)
    eng = MultiCentralEngine(store, "mse", E, D, P, Hyper(), act_dtype=torch.bfloat16)
    eng.use_graph = True
    eng.graph.warmup = 2
    labels = torch.zeros(B, dtype=torch.int64, device=dev)
    batches = [{"aug": devp, "idx": rng.choice(N, B, replace=False), "label": labels}
               for _ in range(4)]
    px = lambda *s: torch.rand(*s, device=dev)  # noqa: E731
    synth = {"image": px(B, 1, 28, 28), "audio": px(B, 1, 112, 112), "label": labels,
             "g_img": px(B, G, 1, 28, 28), "g_aud": px(B, G, 1, 112, 112),
             "l_img": px(B, L, 1, 28, 28), "l_aud": px(B, L, 1, 112, 112)}
    for name, feed, nxt in (("step_synthetic_views", lambda i: synth, None),
                            ("step_device_augmented", lambda i: batches[i % len(batches)], None),
                            ("step_device_augmented_prefetched", lambda i: batches[i % len(batches)],
                             lambda i: batches[(i + 1) % len(batches)])):
        for i in range(6):
            eng.step(feed(i), next_batch=nxt(i) if nxt else None)
        torch.cuda.synchronize()
        k = [6]

        def one():
            eng.step(feed(k[0]), next_batch=nxt(k[0]) if nxt else None)
            k[0] += 1

        gpu_ms, wall_ms = timed(one, iters)
        print(json.dumps({"bench": "train_step", "path": name, "B": B, "mode": "mse", "dtype": "bf16",
                          "ms_per_step": round(max(gpu_ms, wall_ms), 3),
                          "pairs_per_s": round(B / (max(gpu_ms, wall_ms) / 1e3), 1)}), flush=True)


if __name__ == "__main__":
    main()
