"""Time a Cin-1 first layer's passes standalone with HIP events (µs per launch): the stored-y
chain (conv + BN partials, BN -> ReLU -> pool, BN-backward reduce + apply + weight gradient)
against the stored-y-free recompute passes (statistics, apply, pass-4 moments) and, for the
audio conv1, the code-routed backward.

    python tools/c1bench.py [--shape audio|image|image3] [--n 7168]"""
import argparse
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "multimodal-ssl-avmnist_amd")]
from avdino import ops  # noqa: E402

T = torch.bfloat16
SHAPES = {"audio": (112, 8, 5, 2), "image": (28, 32, 5, 2), "image3": (28, 32, 3, 1),
          "audio3": (112, 32, 3, 1)}


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
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="image", choices=list(SHAPES))
    ap.add_argument("--n", type=int, default=7 * 1024)
    a = ap.parse_args()
    H, C, K, pad = SHAPES[a.shape]
    N, B = a.n, 1024
    G = N // B
    Hp = H // 2
    x = torch.rand(N, H, H, 1, device="cuda").to(T)
    w = (torch.rand(C, 1, K, K, device="cuda") - 0.5) / K
    bias = (torch.rand(C, device="cuda") - 0.5) / 5
    wk = torch.empty(ops.cl_weight_elems(C, 1, K, 0), device="cuda", dtype=T)
    ops.cl_weight_layout(w, wk, 0)
    y = torch.empty(N, H, H, C, device="cuda", dtype=T)
    R0 = ops.cl_stat_rows(H, H, B, K, 1, C, T)
    st0 = torch.empty(C * G * R0 * 2, device="cuda")
    gamma, beta = torch.ones(C, device="cuda"), torch.zeros(C, device="cuda")
    bn = torch.empty(4, G * C, device="cuda")
    gz = (torch.rand(N, Hp, Hp, C, device="cuda") - 0.5).to(T)
    z = torch.empty(N, Hp, Hp, C, device="cuda", dtype=T)
    dy = torch.empty_like(y)
    Rb = ops.cl_bn_bwd_rows(B, C, H, H, T)
    p0 = torch.empty(C * G * Rb * 2, device="cuda")
    coef = torch.empty(G * C * 3, device="cuda")
    dg, dbt = torch.empty(C, device="cuda"), torch.empty(C, device="cuda")
    ops.cl_conv_fwd(x, wk, bias, y, st0, N, B, 1, H, H, C, K, pad)
    ops.bn_finalize(st0, G, R0, C, B * H * H, gamma, beta, bn[0], bn[1], bn[2], bn[3])
    ops.cl_bn_bwd_reduce(y, gz, 0, bn[2], bn[3], bn[0], bn[1], p0, N, B, C, H, H)
    ops.bn_bwd_finalize(p0, G, Rb, C, B * H * H, gamma, bn[0], bn[1], coef, dg, dbt, None)
    res = {}
    res["fwd stored y"] = timeit(lambda: ops.cl_conv_fwd(x, wk, bias, y, st0, N, B, 1, H, H, C, K, pad))
    res["relu_pool"] = timeit(lambda: ops.cl_bn_relu_pool(y, bn[2], bn[3], z, 0, N, B, C, H, H))
    res["reduce pooled"] = timeit(lambda: ops.cl_bn_bwd_reduce_pooled(y, z, gz, 0, gamma, beta, bn[0], bn[1], p0,
                                                                      N, B, C, H, H))
    ns = ops.cl_apply_wgrad_slabs(T, N, 1, H, H, C, K, pad)
    if ns:
        f0 = torch.empty(ns * C * K * K, device="cuda")
        res["apply+wgrad fused"] = timeit(lambda: ops.cl_bn_bwd_apply_wgrad(y, gz, bn[2], bn[3], coef, x, f0, N, B, 1,
                                                                            H, H, C, K, pad))
    else:
        res["bwd apply"] = timeit(lambda: ops.cl_bn_bwd_apply(y, gz, 0, bn[2], bn[3], coef, dy, N, B, C, H, H))
        nch = ops.cl_wgrad_chunks(N, C, 1, K)
        wp = torch.empty(nch * C * K * K, device="cuda")
        res["wgrad"] = timeit(lambda: ops.cl_conv_wgrad(x, dy, wp, N, 1, H, H, C, K, pad))
    R1 = ops.cl_c1_recompute_rows(ops.C1_STATS, T, N, B, 1, H, H, C, K, pad)
    if R1:
        st1 = torch.empty(C * G * R1 * 2, device="cuda")
        R4 = ops.cl_c1_recompute_rows(ops.C1_REDUCE_MOMENTS, T, N, B, 1, H, H, C, K, pad)
        m4 = torch.empty(C * G * R4 * 2 + R4 * G * ops.c1_moment_cols(C, K), device="cuda")
        res["rc stats"] = timeit(lambda: ops.cl_c1_recompute(ops.C1_STATS, x, wk, bias, N, B, 1, H, H, C, K, pad,
                                                             out=st1))
        res["rc apply"] = timeit(lambda: ops.cl_c1_recompute(ops.C1_APPLY, x, wk, bias, N, B, 1, H, H, C, K, pad,
                                                             scale=bn[2], shift=bn[3], z=z))
        res["rc moments"] = timeit(lambda: ops.cl_c1_recompute(ops.C1_REDUCE_MOMENTS, x, wk, bias, N, B, 1, H, H, C,
                                                               K, pad, scale=bn[2], shift=bn[3], mean=bn[0],
                                                               invstd=bn[1], gz=gz, out=m4))
    if C == 8 and ops.c1_codes_rows(N, B, H, H):
        codes = torch.empty(N * Hp * Hp, device="cuda", dtype=torch.int32)
        Rc = ops.c1_codes_rows(N, B, H, H)
        mc = torch.empty(Rc * G * ops.c1_codes_cols(), device="cuda")
        res["apply+codes"] = timeit(lambda: ops.c1_apply_codes(x, wk, bias, bn[2], bn[3], z, codes, N, B, H, H))
        res["moments codes"] = timeit(lambda: ops.c1_moments_codes(x, gz, codes, mc, N, B, H, H))
    print(f"{a.shape} N={N}", " ".join(f"{k}={v:.1f}us" for k, v in res.items()), flush=True)


if __name__ == "__main__":
    main()
