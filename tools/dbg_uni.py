"""Layer-by-layer error of the unimodal engine's student conv stack vs the float64 oracle
(diagnostic, GPU).  usage: python tools/dbg_uni.py [case]"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "multimodal-ssl-avmnist_amd")]
from oracle import numpy_oracle as O  # noqa: E402
from oracle.params import make_multimodal_batch  # noqa: E402
from tests.test_gpu_uni import CASES, HP, build, dev_batch, host, rel  # noqa: E402

case = sys.argv[1] if len(sys.argv) > 1 else "uni_audio_g2l2_cos"
kind, D, P, B, G, L, pseed, bseed, alpha = CASES[case]
store, eng, state = build(kind, D, P, pseed, cos_alpha=alpha)
batch = make_multimodal_batch(B, G, L, bseed, with_originals=False)
eng.forward(dev_batch(batch))
V = G + L
Pm = {k: np.asarray(v, np.float64) for k, v in state.items()}
x = np.concatenate([O._views_to_rows(batch["g_aud"]), O._views_to_rows(batch["l_aud"])]).astype(np.float64)
st = eng.enc.branch.stack
ctxs = eng.ws.bufs
h = x
for i, (ci, co, k, pad) in enumerate(st.convs):
    y, _ = O.conv2d_fwd(h, Pm[st.conv_keys[i] + ".weight"], Pm[st.conv_keys[i] + ".bias"], pad)
    Ho = y.shape[2]
    ours_y = host(eng.ws.bufs[f"s.y{i}"][:V * B * Ho * Ho * co]).reshape(V * B, Ho, Ho, co).transpose(0, 3, 1, 2)
    z, _, _ = O.bn_train_fwd(y, Pm[st.bn_keys[i] + ".weight"], Pm[st.bn_keys[i] + ".bias"], V, (2, 3))
    p, _ = O.maxpool2_fwd(np.maximum(z, 0))
    print(f"layer {i}: conv out rel {rel(ours_y, y):.3g}")
    if i + 1 < len(st.convs):
        Hp = p.shape[2]
        ours_p = host(eng.ws.bufs[f"s.x{i + 1}"][:V * B * Hp * Hp * co]).reshape(V * B, Hp, Hp, co).transpose(0, 3, 1, 2)
        print(f"layer {i}: pooled rel {rel(ours_p, p):.3g}  (max abs {np.abs(ours_p - p).max():.3g})")
        h = ours_p   # continue from OUR input: isolates each layer's error
    else:
        f = p.mean(axis=(2, 3))
        ours_f = host(eng.ws.bufs["s.feat"][:V * B * co]).reshape(V * B, co)
        print(f"gap feat rel {rel(ours_f, f):.3g}")
