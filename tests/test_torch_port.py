"""The CPU baseline (oracle/torch_port.py) computes the same step as the float64 oracle:
same state-dict keys as the reference, same loss on the same inputs (fp32 tolerance)."""
import numpy as np
import pytest
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


def _port_step_grads(dtype, fx, mode="mse"):
    E, D, P, B, G, L, pseed, bseed = [int(x) for x in fx["meta_dims"]]
    model = TP.DinoMSE(E, D, P, dropout=0.0, fusion_dropout=0.0, mode=mode)
    state = make_state(S.multimodal_dino_spec(mode, E, D, P), pseed)
    model.load_state_dict({k: torch.from_numpy(np.array(v)) for k, v in state.items()})
    model = model.to(dtype)
    model.train()
    b = {k: torch.from_numpy(v) for k, v in make_multimodal_batch(B, G, L, bseed).items()}
    b = {k: (v.to(dtype) if v.is_floating_point() else v) for k, v in b.items()}
    fi, fa, s, t = model(b["image"], b["audio"], b["g_img"], b["g_aud"], b["l_img"], b["l_aud"])
    aux = TP.supervised_loss(fi, fa, b["label"]) if mode == "semi_supervised" else TP.mse_loss(fi, fa)
    loss = TP.dino_loss(s, t) + aux
    model.update_teacher()
    model.zero_grad()
    loss.backward()
    return loss.item(), {k: p.grad.double().numpy() for k, p in model.named_parameters() if p.grad is not None}


@pytest.mark.parametrize("mode,name", [("mse", "mm_mse_small"), ("semi_supervised", "mm_semi_small")])
def test_torch_port_gradients_match_reference_fixture(mode, name):
    """the CPU baseline's gradients, not only its loss, against the reference's
    own step (fixture mm_mse_small): run in float64 it matches the reference's float64 run to
    1e-8 (same algorithm); in fp32 (how bench.py times it) it stays within the reference's own
    fp32-vs-float64 spread (2e-2 on the audio conv tensors, 1e-3 elsewhere)."""
    from tests import golden_util as gu
    f64, f32 = gu.load(name + "_f64"), gu.load(name)
    zero = gu.zero_grad_keys(f64)
    for dtype, fx, tol, lt in ((torch.float64, f64, 1e-8, 1e-9), (torch.float32, f32, None, 2e-5)):
        loss, grads = _port_step_grads(dtype, fx, mode)
        assert abs(loss - float(fx["loss"])) < lt, (loss, float(fx["loss"]))
        live = [str(k) for k in fx["live_keys"]]
        assert sorted(live) == sorted(grads)
        bad = []
        for k in live:
            if "grad/" + k in zero:
                continue
            rel = tol if tol is not None else (2e-2 if k.startswith("student.audio_encoder") else 1e-3)
            ok, msg = gu.compare(fx, "grad/" + k, grads[k], rel=rel)
            if not ok:
                bad.append(msg)
        assert not bad, bad[:10]
