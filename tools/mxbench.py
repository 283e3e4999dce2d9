"""Standalone timing of the mid-layer conv kernels, bf16 (conv_ws) vs block-scaled fp8
(conv_ws8), forward and input gradient, at a given N (default: config 2's student N = 7168,
--n 28672: config 5's).  python tools/mxbench.py [--n N] [--reps R]"""
import argparse
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "multimodal-ssl-avmnist_amd"))
from avdino import ops  # noqa: E402

LAYERS = [(8, 16, 5, 2, 56), (16, 32, 5, 2, 28), (32, 64, 5, 2, 14), (32, 64, 5, 0, 14)]


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1000.0 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=7168)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    N, G = a.n, 7
    B = N // G
    for Cin, Cout, K, pad, H in LAYERS:
        Ho = H + 2 * pad - K + 1
        x = torch.randn(N, H, H, Cin, device="cuda").to(torch.bfloat16)
        w = torch.randn(Cout, Cin, K, K, device="cuda") * 0.05
        b = torch.zeros(Cout, device="cuda")
        y = torch.empty(N, Ho, Ho, Cout, dtype=torch.bfloat16, device="cuda")
        dy = torch.randn(N, Ho, Ho, Cout, device="cuda").to(torch.bfloat16)
        dx = torch.empty(N, H, H, Cin, dtype=torch.bfloat16, device="cuda")
        wk = torch.empty(ops.cl_weight_elems(Cout, Cin, K, 0), dtype=torch.bfloat16, device="cuda")
        wkd = torch.empty(ops.cl_weight_elems(Cout, Cin, K, 1), dtype=torch.bfloat16, device="cuda")
        ops.cl_weight_layout(w, wk, 0)
        ops.cl_weight_layout(w, wkd, 1)
        wq = torch.empty(ops.mx_weight_bytes(Cout, Cin, K, 0), dtype=torch.uint8, device="cuda")
        ws = torch.empty(ops.mx_scale_bytes(Cout, Cin, K, 0), dtype=torch.uint8, device="cuda")
        wqd = torch.empty(ops.mx_weight_bytes(Cout, Cin, K, 1), dtype=torch.uint8, device="cuda")
        wsd = torch.empty(ops.mx_scale_bytes(Cout, Cin, K, 1), dtype=torch.uint8, device="cuda")
        ops.mx_weight_layout(w, wq, ws, 0)
        ops.mx_weight_layout(w, wqd, wsd, 1)
        R = ops.cl_stat_rows(Ho, Ho, B, K, Cin, Cout, torch.bfloat16)
        R8 = ops.mx_stat_rows(H, B, K, Cin, Cout, pad)
        st = torch.empty(Cout * G * max(R, R8) * 2, device="cuda")
        fl = 2.0 * N * Ho * Ho * Cout * Cin * K * K
        tb = timeit(lambda: ops.cl_conv_fwd(x, wk, b, y, st, N, B, Cin, H, H, Cout, K, pad), a.reps)
        t8 = timeit(lambda: ops.mx_conv_fwd(x, wq, ws, b, y, st, N, B, Cin, H, H, Cout, K, pad), a.reps)
        db = timeit(lambda: ops.cl_conv_dgrad(dy, wkd, dx, N, Cin, H, H, Cout, K, pad), a.reps)
        d8 = timeit(lambda: ops.mx_conv_dgrad(dy, wqd, wsd, dx, N, Cin, H, H, Cout, K, pad), a.reps)
        nch = ops.cl_wgrad_chunks(N, Cout, Cin, K)
        nch8 = ops.mx_wgrad_chunks(N, Cin, H, Cout, K, pad)
        parts = torch.empty(max(nch, nch8) * Cout * Cin * K * K, device="cuda")
        wb = timeit(lambda: ops.cl_conv_wgrad(x, dy, parts, N, Cin, H, H, Cout, K, pad), a.reps)
        w8 = timeit(lambda: ops.mx_conv_wgrad(x, dy, parts, N, Cin, H, H, Cout, K, pad), a.reps)
        print(f"{Cin:>2}->{Cout:<2} @{H} p{pad} N={N}: fwd bf16 {tb:7.1f} us  mx {t8:7.1f} us ({tb / t8:4.2f}x, "
              f"{fl / t8 / 1e6:6.0f} TF/s)   dgrad bf16 {db:7.1f}  mx {d8:7.1f} ({db / d8:4.2f}x)   "
              f"wgrad bf16 {wb:7.1f}  mx {w8:7.1f} ({wb / w8:4.2f}x)", flush=True)


if __name__ == "__main__":
    main()
