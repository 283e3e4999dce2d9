"""Time the 3x3 conv kernels (fwd / dgrad / wgrad) of config 4 per shape with HIP events.
    python tools/c3bench.py   (AVDINO_LIB=... selects a library build)"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "multimodal-ssl-avmnist_amd")]
from avdino import ops  # noqa: E402

T = torch.bfloat16
SHAPES = [(32, 56, 64), (64, 28, 128), (128, 14, 256), (32, 14, 64), (64, 7, 128)]


def timeit(fn, n=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3


def main():
    N, B = 2048, 1024
    tag = os.path.basename(os.environ.get("AVDINO_LIB", "libavdino.so"))
    only = os.environ.get("C3B_ONLY")            # profiling: one op ("fwd"/"dgrad"/"wgrad")
    pick = os.environ.get("C3B_SHAPE")           # profiling: one shape index
    for si, (Ci, H, Co) in enumerate(SHAPES):
        if pick is not None and si != int(pick):
            continue
        x = torch.randn(N, H, H, Ci, device="cuda").to(T)
        w = torch.randn(Co, Ci, 3, 3, device="cuda") * 0.05
        wk = torch.empty(ops.cl_weight_elems(Co, Ci, 3, 0), device="cuda", dtype=T)
        wd = torch.empty(ops.cl_weight_elems(Co, Ci, 3, 1), device="cuda", dtype=T)
        ops.cl_weight_layout(w, wk, 0)
        ops.cl_weight_layout(w, wd, 1)
        bias = torch.zeros(Co, device="cuda")
        y = torch.empty(N, H, H, Co, device="cuda", dtype=T)
        R = ops.cl_stat_rows(H, H, B, 3, Ci, Co, T)
        st = torch.empty(Co * (N // B) * R * 2, device="cuda")
        dx = torch.empty_like(x)
        fl = 2.0 * N * H * H * Co * Ci * 9
        nch = ops.cl_wgrad_chunks(N, Co, Ci, 3)
        parts = torch.empty(nch * Co * Ci * 9, device="cuda")
        tf = td = tw = float("nan")
        if only in (None, "fwd"):
            tf = timeit(lambda: ops.cl_conv_fwd(x, wk, bias, y, st, N, B, Ci, H, H, Co, 3, 1))
        if only in (None, "dgrad"):
            td = timeit(lambda: ops.cl_conv_dgrad(y, wd, dx, N, Ci, H, H, Co, 3, 1))
        if only in (None, "wgrad"):
            tw = timeit(lambda: ops.cl_conv_wgrad(x, y, parts, N, Ci, H, H, Co, 3, 1), 3)
        print(f"{tag} {Ci:4d}->{Co:4d} @{H:3d}: fwd {tf:8.1f} us ({fl / tf / 1e6:6.1f} TF/s)  "
              f"dgrad {td:8.1f} us ({fl / td / 1e6:6.1f})  wgrad {tw:8.1f} us ({fl / tw / 1e6:6.1f})",
              flush=True)


if __name__ == "__main__":
    main()
