"""HIP-event times of the audio conv1 (1->8, 5x5 pad 2, 112x112) training passes at config 2's
student size (N = 7168, B = 1024): the Gram statistics pass + its float64 finalize, the
codes-writing BN -> ReLU -> pool pass, the routed window-moments pass and the combine.  AVDINO_LIB selects a library variant
(tools/build_variants.sh).  One line: us per pass and their sum."""
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
    N, B, H, C, K = 7 * 1024, 1024, 112, 8, 5
    G, Hp = N // B, H // 2
    x = torch.rand(N, H, H, 1, device="cuda").to(T)
    w = (torch.rand(C, 1, K, K, device="cuda") - 0.5) / 3
    bias = (torch.rand(C, device="cuda") - 0.5) / 5
    wk = torch.empty(ops.cl_weight_elems(C, 1, K, 0), device="cuda", dtype=T)
    ops.cl_weight_layout(w, wk, 0)
    gamma, beta = torch.ones(C, device="cuda"), torch.zeros(C, device="cuda")
    bn = torch.empty(4, G * C, device="cuda")
    R, gc, mc = ops.c1_codes_rows(N, B, H, H), ops.c1_gram_cols(), ops.c1_codes_cols()
    gparts = torch.empty(R * G * gc, device="cuda")
    gram = torch.empty(G * gc, device="cuda")
    z = torch.empty(N, Hp, Hp, C, device="cuda", dtype=T)
    codes = torch.empty(N * Hp * Hp, device="cuda", dtype=torch.int32)
    gz = (torch.rand(N, Hp, Hp, C, device="cuda") - 0.5).to(T)
    parts = torch.empty(R * G * mc, device="cuda")
    mom = torch.empty(G * mc, device="cuda")
    dw = torch.empty(C * 25, device="cuda")
    d3 = [torch.empty(C, device="cuda") for _ in range(3)]
    t = {}
    t["gram"] = timeit(lambda: ops.c1_gram(x, gparts, N, B, H, H))
    ops.sum_rows(gparts, R, G * gc, gram)
    t["gram_fin"] = timeit(lambda: ops.c1_gram_finalize(gram, wk, bias, gamma, beta, B * H * H, bn[0], bn[1],
                                                         bn[2], bn[3], None, None, G))
    t["apply"] = timeit(lambda: ops.c1_apply_codes(x, wk, bias, bn[2], bn[3], z, codes, N, B, H, H))
    t["moments"] = timeit(lambda: ops.c1_moments_codes_ng(x, gz, codes, parts, N, B, H, H))
    ops.sum_rows(parts, R, G * mc, mom)
    t["combine"] = timeit(lambda: ops.c1_codes_combine_gram(mom, gram, wk, bias, gamma, bn[0], bn[1], B * H * H,
                                                           dw, *d3, None, G))
    three = t["gram"] + t["apply"] + t["moments"]
    lib = os.path.basename(os.environ.get("AVDINO_LIB", "libavdino.so"))
    print(f"{lib}: " +
          "  ".join(f"{k} {v:.1f}" for k, v in t.items()) + f"  | three passes {three:.1f} us")


if __name__ == "__main__":
    main()
