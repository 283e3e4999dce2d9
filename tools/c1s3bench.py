"""Time config 4's 3x3 first-layer passes (1 -> 32 at 112^2 and 28^2, N = B = 2048) with HIP
events: statistics (pass 0), BN -> ReLU -> pool + codes, routed moments.
    python tools/c1s3bench.py"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "multimodal-ssl-avmnist_amd")]
from avdino import ops  # noqa: E402

T = torch.bfloat16


def timeit(fn, n=20):
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
    N = B = int(os.environ.get("C1S3_N", "2048"))
    C, K, pad = 32, 3, 1
    for H in (112, 28):
        Hp = H // 2
        x = torch.rand(N, H, H, 1, device="cuda").to(T)
        w = (torch.randn(C, 1, K, K, device="cuda") / 3).to(T).float()
        wk = torch.empty(ops.cl_weight_elems(C, 1, K, 0), device="cuda", dtype=T)
        ops.cl_weight_layout(w, wk, 0)
        bias = torch.randn(C, device="cuda") * 0.1
        R0 = ops.cl_c1_recompute_rows(ops.C1_STATS, T, N, B, 1, H, H, C, K, pad)
        st = torch.empty(C * R0 * 2, device="cuda")
        sc, sf = torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda") * 0.1
        z = torch.empty(N, Hp, Hp, C, device="cuda", dtype=T)
        codes = torch.empty(N * Hp * Hp * C // 4, device="cuda", dtype=torch.int16)
        gz = torch.randn(N, Hp, Hp, C, device="cuda").to(T)
        Rc, mc = ops.c1r3_codes_rows(N, B, H, H, C), ops.c1r3_codes_cols(C)
        parts = torch.empty(Rc * mc, device="cuda")
        t0 = timeit(lambda: ops.cl_c1_recompute(ops.C1_STATS, x, wk, bias, N, B, 1, H, H, C, K, pad, out=st))
        t1 = timeit(lambda: ops.c1r3_apply_codes(x, wk, bias, sc, sf, z, codes, N, B, H, H, C))
        t2 = timeit(lambda: ops.c1r3_moments_codes(x, wk, gz, codes, parts, N, B, H, H, C))
        xb, zb, cb = x.numel() * 2, z.numel() * 2, codes.numel() * 2
        print(f"N={N} {H}^2: stats {t0:7.1f} us ({xb / t0 / 1e3:6.0f} GB/s)  apply+codes {t1:7.1f} us "
              f"({(xb + zb + cb) / t1 / 1e3:6.0f} GB/s)  moments {t2:7.1f} us "
              f"({(xb + zb + cb) / t2 / 1e3:6.0f} GB/s)", flush=True)


if __name__ == "__main__":
    main()
