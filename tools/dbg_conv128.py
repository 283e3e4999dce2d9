"""Debug: which dimension breaks the bf16 MFMA conv for (Cin=128, Cout=256, K=3)?"""
import sys, os
sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "multimodal-ssl-avmnist_amd")]
import numpy as np, torch
from avdino import ops
from oracle import numpy_oracle as O

def run(N, Cin, H, Cout, K, pad, stats=False):
    g = np.random.default_rng(0)
    x = torch.from_numpy(g.uniform(-1, 1, (N, Cin, H, H)).astype(np.float32)).to(torch.bfloat16)
    w = torch.from_numpy((g.uniform(-1, 1, (Cout, Cin, K, K)) / np.sqrt(Cin*K*K)).astype(np.float32)).to(torch.bfloat16).float()
    yref, _ = O.conv2d_fwd(x.float().numpy().astype(np.float64), w.numpy().astype(np.float64), np.zeros(Cout), pad)
    wk = torch.empty(ops.conv_weight_layout_elems(Cout, Cin, K, 2), device="cuda", dtype=torch.bfloat16)
    ops.conv_weight_layout(w.cuda(), wk, 2)
    y = torch.full((N, Cout, yref.shape[2], yref.shape[2]), 7.0, device="cuda", dtype=torch.bfloat16)
    T = ops.conv_stat_tiles(yref.shape[2], yref.shape[2])
    st = torch.zeros(Cout * N * T * 2, device="cuda") if stats else None
    ops.conv2d_fwd(x.cuda(), wk, torch.zeros(Cout, device="cuda") if stats else None, y, st, N, Cin, H, H, Cout, K, pad)
    torch.cuda.synchronize()
    yh = y.float().cpu().numpy()
    e = np.linalg.norm(yh - yref) / np.linalg.norm(yref)
    print(f"stats={stats} N={N} Cin={Cin} H={H} Cout={Cout} K={K}: rel={e:.3g} untouched={(yh == 7.0).mean():.3f} "
          f"wk_absmax={wk.float().abs().max().item():.3g}", flush=True)

for case in [(2, 64, 14, 64, 3, 1), (2, 128, 14, 64, 3, 1), (2, 64, 14, 256, 3, 1), (2, 128, 14, 256, 3, 1),
             (2, 128, 7, 64, 3, 1), (1, 128, 14, 128, 3, 1)]:
    run(*case, stats=True)
