"""The CPU baseline (oracle/torch_port.py) computes the same step as the float64 oracle:
same state-dict keys as the reference, same loss on the same inputs (fp32 tolerance)."""
import numpy as np
import torch

from oracle import numpy_oracle as O
from oracle import spec as S
from oracle import torch_port as TP
from oracle.params import make_multimodal_batch, make_state

HP = dict(lr=1e-4, wd=1e-6, momentum=0.996, center_momentum=0.9, tau_s=0.1, tau_t=0.04)


def test_torch_port_matches_oracle():
    E, D, P, B, G, L = 32, 32, 16, 4, 2, 4
    model = TP.DinoMSE(E, D, P, dropout=0.0, fusion_dropout=0.0)
    spec = S.multimodal_dino_spec("mse", E, D, P)
    assert sorted(model.state_dict().keys()) == sorted(spec.keys())
    state = make_state(spec, 301)
    model.load_state_dict({k: torch.from_numpy(np.array(v)) for k, v in state.items()})
    model.train()
    batch = make_multimodal_batch(B, G, L, 3001)
    ref = O.multimodal_step(state, batch, "mse", HP)
    opt = TP.make_optimizer(model)
    loss = TP.train_step(model, opt, {k: torch.from_numpy(v) for k, v in batch.items()})
    assert abs(loss.item() - ref["loss"]) < 2e-5
    np.testing.assert_allclose(model.center.numpy(), ref["center_after"], rtol=1e-5, atol=1e-7)


def test_config1_pretrain_port_matches_reference_fixture():
    """The config-1 CPU baseline (torch_port.UniImageDINO + pretrain_step: the reference's
    training_structures.pretrain_dino loop) reproduces the reference's own step losses."""
    import numpy as np
    import torch
    from oracle import spec as OS
    from oracle import torch_port as TP
    from oracle.params import make_multimodal_batch, make_state
    from tests import golden_util as gu
    fx = gu.load("pretrain_image_simple")
    D, P, B, epochs, nb, pseed, bseed = [int(x) for x in fx["meta_dims"]]
    st = make_state(OS.unimodal_dino_spec("image", D, P), pseed)
    m = TP.UniImageDINO(D, P, dropout=0.0)
    m.load_state_dict({k: torch.from_numpy(np.array(v)) for k, v in st.items()}, strict=True)
    opt = torch.optim.AdamW(list(m.parameters()), lr=float(fx["meta_lr"]))
    bs = [make_multimodal_batch(B, 2, 0, bseed + i, with_originals=False) for i in range(nb)]
    ls = [TP.pretrain_step(m, opt, torch.from_numpy(b["g_img"])).item() for _ in range(epochs) for b in bs]
    np.testing.assert_allclose(ls, fx["step_losses"], atol=1e-6, rtol=0)
