"""Unimodal DINO training-step parity (BASELINE config 1): the HIP engine
(UniModalEngine, fp32 parity mode) vs the float64 oracle, from identical parameters and
inputs, on the exact dims/seeds of the committed golden cases (so the reference's own fp32
error on each tensor is known and bounds ours):

  uni_image_g2l0        ImageEncoder, 2 global views, no cosine term (config 1 shape, B=8)
  uni_image_g2l4_cos    ImageEncoder, 2 global + 4 local views, cosine_loss_alpha 0.3
  uni_audio_g2l2_cos    SpectrogramEncoder (3x3 CNN on 112x112), 2 + 2 views, alpha 0.3
  uni_speccentral_g2l2  SpectrogramEncoderCentral (CentralNet LeNet + dead fc1/fc2), 2 + 2 views

Tolerances: loss 3e-5 abs; student/teacher outputs, embeddings and centre 1e-5 rel-L2;
gradients max(1e-3, 3x the reference's fp32-vs-float64 error on that tensor), median 1e-4;
near-zero gradients (|g| < 1e-4: biases feeding a BatchNorm) 1e-4 abs; (3x: our rounding
noise and the reference's are independent draws of the same size); EMA'd teacher 1e-6;
BN running stats 1e-5; post-Adam parameters 1e-6 (Adam applied to our gradients)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

from oracle import numpy_oracle as O  # noqa: E402
from oracle import spec as OS  # noqa: E402
from oracle.params import make_multimodal_batch, make_state  # noqa: E402
from tests import golden_util as gu  # noqa: E402

HP = dict(lr=1e-4, wd=1e-6, momentum=0.996, center_momentum=0.9, tau_s=0.1, tau_t=0.04)
CASES = {  # name -> (encoder kind, D, P, B, G, L, pseed, bseed, cos_alpha)
    "uni_image_g2l0": ("image_simple", 256, 128, 8, 2, 0, 106, 1006, 0.0),
    "uni_image_g2l4_cos": ("image_simple", 64, 32, 6, 2, 4, 108, 1008, 0.3),
    "uni_audio_g2l2_cos": ("spectrogram_simple", 64, 32, 3, 2, 2, 109, 1009, 0.3),
    "uni_speccentral_g2l2": ("spectrogram_central", 32, 16, 3, 2, 2, 110, 1010, 0.0),
}


def rel(a, b):
    a = np.asarray(a, np.float64).ravel()
    b = np.asarray(b, np.float64).ravel()
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30)


def host(t):
    return t.detach().float().cpu().numpy().astype(np.float64)


def ref_fp32_err(case):
    """Per-gradient rel-L2 error of the reference's fp32 run vs its float64 run."""
    f32, f64 = gu.load(case), gu.load(case + "_f64")
    out = {}
    for k in f64:
        if k.startswith("grad/") and "@" not in k and np.linalg.norm(f64[k]) > 1e-9:
            out[k[5:]] = gu.rel_err(f32[k], f64[k])
        elif k.startswith("grad/") and k.endswith("@val"):
            out[k[5:-4]] = gu.rel_err(f32[k], f64[k])
    return out


def ref_fp32_out_err(case, key):
    f32, f64 = gu.load(case), gu.load(case + "_f64")
    if key in f64:
        return gu.rel_err(f32[key], f64[key])
    return gu.rel_err(f32[key + "@val"], f64[key + "@val"])


# Linear biases between the encoder and the projection head's BatchNorm1d: the DINO part of
# their gradient cancels exactly through the BN (column sums of its input gradient are 0), so
# they hold only the cosine term plus the rounding residue of large cancelling sums
CANCELLING = {"student.projection.0.bias", "student.encoder.14.bias", "student.encoder.18.bias",
              "student.encoder.1.bias"}


def build(kind, D, P, pseed, act=torch.float32, cos_alpha=0.0):
    from avdino.engine import Hyper, UniModalEngine
    from avdino.params import ParamStore
    from avdino.spec import unimodal_dino_sd
    sd = unimodal_dino_sd(kind, D, P)
    ospec = OS.unimodal_dino_spec(kind, D, P)
    assert list(sd.keys()) == list(ospec.keys())
    store = ParamStore(sd, "cuda")
    state = make_state(ospec, pseed)
    store.load_state_dict({k: torch.from_numpy(np.array(v)) for k, v in state.items()})
    hp = Hyper(lr=HP["lr"], weight_decay=HP["wd"], momentum=HP["momentum"],
               center_momentum=HP["center_momentum"], student_temperature=HP["tau_s"],
               teacher_temperature=HP["tau_t"], dropout=0.0, fusion_dropout=0.0)
    return store, UniModalEngine(store, kind, D, P, hp, act_dtype=act, cos_alpha=cos_alpha), state


def dev_batch(b):
    return {k: torch.from_numpy(v).cuda() for k, v in b.items()}


@pytest.mark.parametrize("case", list(CASES))
def test_unimodal_step_matches_oracle(case):
    from avdino.engine import adam_step, ema_step
    kind, D, P, B, G, L, pseed, bseed, alpha = CASES[case]
    store, eng, state = build(kind, D, P, pseed, cos_alpha=alpha)
    batch = make_multimodal_batch(B, G, L, bseed, with_originals=False)
    ref = O.unimodal_step(state, batch, HP, kind, alpha)
    # the oracle is pinned to the reference on exactly this case (tests/test_oracle_golden.py)
    assert abs(ref["loss"] - float(gu.load(case + "_f64")["loss"])) < 1e-8

    loss = eng.forward(dev_batch(batch))
    s_out, t_out, emb = eng.outputs()
    assert abs(loss.item() - ref["loss"]) < 3e-5, (loss.item(), ref["loss"])
    # outputs: 1e-5, or 3x the reference's own fp32 error on them (4-layer 256-channel audio CNN)
    obound = max(1e-5, 3 * ref_fp32_out_err(case, "s_out"), 3 * ref_fp32_out_err(case, "t_out"))
    assert rel(host(s_out), ref["s_out"]) < obound, (rel(host(s_out), ref["s_out"]), obound)
    assert rel(host(t_out), ref["t_out"]) < obound, (rel(host(t_out), ref["t_out"]), obound)
    assert rel(host(emb), ref["emb"]) < obound
    eng.update_center()
    assert rel(host(store["center"]), ref["center_after"]) < 1e-5
    ema_step(store, HP["momentum"])
    eng.backward()
    assert sorted(store.live_keys) == sorted(ref["grads"].keys())
    floor = ref_fp32_err(case)
    errs = {}
    for k in store.live_keys:
        g, r = host(store.grad_of(k)), ref["grads"][k]
        if np.linalg.norm(r) < 1e-4:
            assert np.linalg.norm(g - r) <= 1e-4, (k, np.linalg.norm(g - r))
            continue
        errs[k] = rel(g, r)
        bound = max(1e-3, 3 * floor.get(k, 0.0))
        assert errs[k] < bound, (k, errs[k], bound)
    print("worst grad errors:", sorted(errs.items(), key=lambda kv: -kv[1])[:4])
    assert np.median(list(errs.values())) < 1e-4
    new = ref["state"]
    for k in store.t_offs:
        assert rel(host(store[k]), new[k]) < 1e-6, k
    for k in store.buffers:
        if k.endswith("running_mean") or k.endswith("running_var"):
            assert rel(host(store.buffers[k]), new[k]) < 1e-5, k
        elif k.endswith("num_batches_tracked"):
            assert int(store.buffers[k].item()) == int(new[k]), k
    ours = {k: host(store.grad_of(k)) for k in store.live_keys}
    pre = {k: host(store[k]) for k in store.live_keys}
    adam_step(store, eng.hp)
    post = O.adam_update_state(pre, ours, {}, 1, HP)
    for k in store.live_keys:
        assert rel(host(store[k]), post[k]) < 1e-6, k


def test_unimodal_loss_curve_matches_oracle():
    """Config-1 shape over 3 steps: every step's loss equals the oracle's on the engine's own
    state, and the free-running curve stays within the fp32 band of the reference's curve."""
    kind, D, P, B, G, L, pseed, bseed, alpha = CASES["uni_image_g2l0"]
    store, eng, state = build(kind, D, P, pseed)
    st = {k: np.asarray(v, np.float64) if v.dtype != np.int64 else v for k, v in state.items()}
    opt, curve, ref_curve, from_ours = {}, [], [], []
    spec = OS.unimodal_dino_spec(kind, D, P)
    for step in range(3):
        b = make_multimodal_batch(B, G, L, bseed + step, with_originals=False)
        ours = {k: store[k].detach().double().cpu().numpy() for k in spec}
        from_ours.append(O.unimodal_step(ours, b, HP, kind, alpha)["loss"])
        r = O.unimodal_step(st, b, HP, kind, alpha)
        ref_curve.append(r["loss"])
        st = O.adam_update_state(r["state"], r["grads"], opt, step + 1, HP)
        curve.append(eng.step(dev_batch(b)).item())
    golden = gu.load("uni_image_g2l0_f64")["curve"]
    print("curve", curve, "oracle", ref_curve, "reference f64", golden)
    np.testing.assert_allclose(ref_curve, golden, atol=1e-7, rtol=0)
    np.testing.assert_allclose(curve, from_ours, atol=3e-5, rtol=0)
    np.testing.assert_allclose(curve, ref_curve, atol=1e-3, rtol=0)


@pytest.mark.parametrize("kind", ["image_simple", "spectrogram_simple"])
def test_unimodal_bf16_step_close_to_oracle(kind):
    D, P, B, G, L = 64, 32, 8, 2, 2
    store, eng, state = build(kind, D, P, 321, act=torch.bfloat16, cos_alpha=0.3)
    batch = make_multimodal_batch(B, G, L, 3210, with_originals=False)
    ref = O.unimodal_step(state, batch, HP, kind, 0.3)
    loss = eng.forward(dev_batch(batch))
    assert abs(loss.item() - ref["loss"]) < 2e-2 * abs(ref["loss"])
    eng.update_center()
    eng.backward()
    errs = sorted(((rel(host(store.grad_of(k)), ref["grads"][k]), k) for k in store.live_keys
                   if np.linalg.norm(ref["grads"][k]) > 1e-4 and k not in CANCELLING), reverse=True)
    med = np.median([e for e, _ in errs])
    assert med < 0.2 and errs[0][0] < 0.6, (med, errs[:6])


def test_lightning_api_unimodal():
    """UniModalDINOLightning surface: training_step -> zero_grad -> backward -> optimizer.step
    (Lightning's automatic optimisation), cosine loss API."""
    from avdino.models import UNIMODAL_MODEL_MAP, UniModalDINOLightning
    m = UniModalDINOLightning(encoder_class=UNIMODAL_MODEL_MAP["image_simple"], output_dim=64,
                              projection_dim=32, dropout=0.0, precision="32", device="cuda",
                              cosine_loss_alpha=0.3)
    b = make_multimodal_batch(4, 2, 2, 77, with_originals=False)
    views = tuple(torch.from_numpy(b[k]) for k in ("g_img", "g_aud", "l_img", "l_aud"))
    opt = m.configure_optimizers()["optimizer"]
    pre = m.model.store.student.clone()
    loss = m.training_step(views, 0)
    opt.zero_grad()
    loss.backward()
    opt.step()
    assert np.isfinite(loss.item())
    assert m.model.arena.grad is not None and not torch.equal(pre, m.model.store.student)
    e = torch.randn(4, 5, 16, device="cuda", requires_grad=True)
    c = m._cosine_consistency_loss(e)
    c.backward()
    ref, dref = O.cosine_consistency_loss(e.detach().double().cpu().numpy())
    assert abs(c.item() - ref) < 1e-5
    assert rel(host(e.grad), dref) < 1e-5
