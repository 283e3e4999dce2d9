"""The fused 56² layer backward alone at config-2 size, with the BN-backward apply in the kernel
(y + pooled gradient, AP = 1) and with a precomputed dY (AP = 0): how much of the launch is the
apply.    python tools/lbwd_ap.py"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "multimodal-ssl-avmnist_amd")]
import torch  # noqa: E402

from avdino import ops  # noqa: E402


def main():
    N, B, Cin, H, Cout, K, pad = 7168, 1024, 8, 56, 16, 5, 2
    g = torch.Generator(device="cuda").manual_seed(0)
    bf = torch.bfloat16

    def rnd(*s, dt=bf):
        return (torch.rand(*s, generator=g, device="cuda") * 2 - 1).to(dt)
    x = rnd(N * H * H * Cin)
    y = rnd(N * H * H * Cout)
    gout = rnd(N * (H // 2) * (H // 2) * Cout)
    dy = rnd(N * H * H * Cout)
    G = N // B
    scale = torch.rand(G * Cout, device="cuda") + 0.5
    shift = torch.rand(G * Cout, device="cuda") - 0.5
    coef = torch.rand(G * Cout * 3, device="cuda")
    w = torch.randn(Cout, Cin, K, K, device="cuda") * 0.1
    wk = torch.empty(ops.cl_weight_elems(Cout, Cin, K, 1), dtype=bf, device="cuda")
    ops.cl_weight_layout(w, wk, 1)
    slabs = ops.cl_layer_bwd_slabs(bf, N, Cin, H, H, Cout, K, pad)
    parts = torch.empty(slabs * Cout * Cin * K * K, device="cuda")
    dx = torch.empty_like(x)
    runs = {"apply (AP=1)": lambda: ops.cl_layer_bwd(y, gout, scale, shift, coef, None, x, wk, dx, parts, slabs,
                                                     N, B, Cin, H, H, Cout, K, pad),
            "dY given (AP=0)": lambda: ops.cl_layer_bwd(None, None, None, None, None, dy, x, wk, dx, parts, slabs,
                                                        N, B, Cin, H, H, Cout, K, pad)}
    for name, fn in runs.items():
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(20):
            fn()
        e.record()
        torch.cuda.synchronize()
        print(f"{name}: {s.elapsed_time(e) / 20 * 1e3:.1f} us per launch", flush=True)


if __name__ == "__main__":
    main()
