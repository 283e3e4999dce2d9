"""Time the audio conv1 (1->8, 5x5, 112x112) kernels of the config-2 student step (N = 7168)
with HIP events: stored-y forward, recompute passes, the stored-y backward pair and the
moments pass.  AVDINO_LIB selects a library variant (tools/build_ws_variants.sh)."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "multimodal-ssl-avmnist_amd")]
from avdino import ops  # noqa: E402

T = torch.bfloat16


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
    N, B, H, C, K, pad = 7 * 1024, 1024, 112, 8, 5, 2
    G = N // B
    x = torch.rand(N, H, H, 1, device="cuda").to(T)
    w = (torch.rand(C, 1, K, K, device="cuda") - 0.5) / 3
    bias = (torch.rand(C, device="cuda") - 0.5) / 5
    wk = torch.empty(ops.cl_weight_elems(C, 1, K, 0), device="cuda", dtype=T)
    ops.cl_weight_layout(w, wk, 0)
    y = torch.empty(N, H, H, C, device="cuda", dtype=T)
    R0 = ops.cl_stat_rows(H, H, B, K, 1, C, T)
    st0 = torch.empty(C * G * R0 * 2, device="cuda")
    gamma, beta = torch.ones(C, device="cuda"), torch.zeros(C, device="cuda")
    bn = torch.empty(4, G * C, device="cuda")
    gz = (torch.rand(N, H // 2, H // 2, C, device="cuda") - 0.5).to(T)
    z = torch.empty(N, H // 2, H // 2, C, device="cuda", dtype=T)
    Rb = ops.cl_bn_bwd_rows(B, C, H, H, T)
    p0 = torch.empty(C * G * Rb * 2, device="cuda")
    coef = torch.empty(G * C * 3, device="cuda")
    dg, dbt = torch.empty(C, device="cuda"), torch.empty(C, device="cuda")
    ns = ops.cl_apply_wgrad_slabs(T, N, 1, H, H, C, K, pad)
    f0 = torch.empty(ns * C * K * K, device="cuda")
    R1 = ops.cl_c1_recompute_rows(ops.C1_STATS, T, N, B, 1, H, H, C, K, pad)
    st1 = torch.empty(C * G * R1 * 2, device="cuda")
    R4 = ops.cl_c1_recompute_rows(ops.C1_REDUCE_MOMENTS, T, N, B, 1, H, H, C, K, pad)
    mc = ops.c1_moment_cols(C, K)
    m4 = torch.empty(C * G * R4 * 2 + R4 * G * mc, device="cuda")

    def fwd():
        ops.cl_conv_fwd(x, wk, bias, y, st0, N, B, 1, H, H, C, K, pad)
    fwd()
    ops.bn_finalize(st0, G, R0, C, B * H * H, gamma, beta, bn[0], bn[1], bn[2], bn[3])
    ops.cl_bn_bwd_reduce(y, gz, 0, bn[2], bn[3], bn[0], bn[1], p0, N, B, C, H, H)
    ops.bn_bwd_finalize(p0, G, Rb, C, B * H * H, gamma, bn[0], bn[1], coef, dg, dbt, None)
    res = {
        "fwd stored y": timeit(fwd),
        "recompute stats": timeit(lambda: ops.cl_c1_recompute(ops.C1_STATS, x, wk, bias, N, B, 1, H, H, C, K, pad, out=st1)),
        "recompute apply": timeit(lambda: ops.cl_c1_recompute(ops.C1_APPLY, x, wk, bias, N, B, 1, H, H, C, K, pad,
                                                              scale=bn[2], shift=bn[3], z=z)),
        "reduce pooled": timeit(lambda: ops.cl_bn_bwd_reduce_pooled(y, z, gz, 0, gamma, beta, bn[0], bn[1], p0, N, B, C, H, H)),
        "bwd apply+wgrad": timeit(lambda: ops.cl_bn_bwd_apply_wgrad(y, gz, bn[2], bn[3], coef, x, f0, N, B, 1, H, H, C, K, pad)),
        "moments": timeit(lambda: ops.cl_c1_recompute(ops.C1_REDUCE_MOMENTS, x, wk, bias, N, B, 1, H, H, C, K, pad,
                                                      scale=bn[2], shift=bn[3], mean=bn[0], invstd=bn[1], gz=gz, out=m4)),
    }
    print(os.environ.get("AVDINO_LIB", "default"), " ".join(f"{k}={v:.1f}us" for k, v in res.items()), flush=True)


if __name__ == "__main__":
    main()
