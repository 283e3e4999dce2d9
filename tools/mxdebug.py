"""Debug helper: MX conv forward on exact integer data vs float64, mismatch pattern."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "multimodal-ssl-avmnist_amd"))
sys.path.insert(0, REPO)
from avdino import ops  # noqa: E402
from tests.test_gpu_mx import _ref_fwd, _weights, _bf, LAYERS  # noqa: E402

for li, (Cin, Cout, K, pad, H) in enumerate(LAYERS):
    Ho = H + 2 * pad - K + 1
    N = 2
    g = torch.Generator().manual_seed(1)
    for kind in ("xones", "wones", "rand"):
        x = torch.randint(-8, 9, (N, H, H, Cin), generator=g).float()
        w = torch.randint(-8, 9, (Cout, Cin, K, K), generator=g).float() * 2.0 ** -5
        if kind == "xones":
            x = torch.ones_like(x)
        if kind == "wones":
            w = torch.ones_like(w) * 2.0 ** -5
        x = _bf(x).cuda()
        w = w.cuda()
        b = torch.zeros(Cout, device="cuda")
        wq, wsc = _weights(w, 0)
        y = torch.empty(N, Ho, Ho, Cout, dtype=torch.bfloat16, device="cuda")
        ops.mx_conv_fwd(x, wq, wsc, b, y, None, N, N, Cin, H, H, Cout, K, pad)
        ref = _bf(_ref_fwd(x.float(), w, b, pad).float())
        bad = (y != ref)
        print(f"L{li} {kind}: {bad.sum().item()} / {bad.numel()} bad; by sample {bad.sum((1,2,3)).tolist()}; "
              f"by row {bad.sum((0,2,3)).tolist()[:16]}; by col {bad.sum((0,1,3)).tolist()[:16]}; "
              f"by ch {bad.sum((0,1,2)).tolist()}")
        if kind == "wones" and bad.any():
            i = bad.nonzero()[0].tolist()
            print("   first bad", i, y[tuple(i)].item(), ref[tuple(i)].item())
