"""Full training-step parity: the HIP engine (fp32) vs the float64 oracle (which is itself
pinned to the reference by tests/test_oracle_golden.py), from identical parameters and inputs.

Tolerances (fp32 kernels vs float64 truth):
  loss 3e-5 abs; outputs / centre rel-L2 1e-5; gradients rel-L2 1e-3, except the audio-encoder
  conv/BN tensors, whose bound is 1.5x the REFERENCE's own fp32-vs-float64 error on the same
  tensors (read from the committed golden fixtures at test time: the reference's fp32 run misses
  its float64 run by up to 5.7e-3 there -- max-pool argmax near-ties in the deeper audio layers
  relocate gradient, tests/golden/mm_mse_small*.npz); median gradient error 1e-4
  (mathematically-zero gradients -- biases feeding a BatchNorm -- |g| <= 1e-4); EMA'd teacher 1e-6; running stats
  1e-5; post-Adam parameters 1e-5 (zero-gradient biases excluded: their Adam step is the sign
  of rounding noise, in the reference too); free-running loss curve at E=32, B=4: 3e-5 on
  step 1, 1e-3 over 4 steps (Adam turns rounding noise on near-zero gradients into +-lr steps;
  the reference's own fp32 run drifts 1.8e-4 from its float64 run by step 4, 3e-4 by step 5);
  at the reference dims E=D=256, P=128 (fixture mm_mse_full, 5 steps, where the reference's own
  fp32 run stays within 3.6e-6 of its float64 run): north_star's 1e-4 on every step.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

from oracle import numpy_oracle as O  # noqa: E402
from oracle import spec as OS  # noqa: E402
from oracle.params import make_multimodal_batch, make_state  # noqa: E402

HP = dict(lr=1e-4, wd=1e-6, momentum=0.996, center_momentum=0.9, tau_s=0.1, tau_t=0.04)


def rel(a, b):
    a = np.asarray(a, np.float64).ravel()
    b = np.asarray(b, np.float64).ravel()
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30)


def host(t):
    return t.detach().float().cpu().numpy().astype(np.float64)


def build(mode, E, D, P, pseed, act=torch.float32, encoder="multi_central"):
    from avdino.engine import Hyper, MultiCentralEngine
    from avdino.params import ParamStore
    from avdino.spec import multimodal_dino_sd
    sd = multimodal_dino_sd(mode, E, D, P, encoder=encoder)
    ospec = OS.multimodal_dino_spec(mode, E, D, P, encoder=encoder)
    assert list(sd.keys()) == list(ospec.keys())
    store = ParamStore(sd, "cuda")
    state = make_state(ospec, pseed)
    store.load_state_dict({k: torch.from_numpy(np.array(v)) for k, v in state.items()})
    hp = Hyper(lr=HP["lr"], weight_decay=HP["wd"], momentum=HP["momentum"],
               center_momentum=HP["center_momentum"], student_temperature=HP["tau_s"],
               teacher_temperature=HP["tau_t"], dropout=0.0, fusion_dropout=0.0)
    return store, MultiCentralEngine(store, mode, E, D, P, hp, act_dtype=act, encoder=encoder), state


def dev_batch(b):
    return {k: torch.from_numpy(v).cuda() for k, v in b.items()}


def zero_grad_keys(grads):
    return {k for k, g in grads.items() if np.linalg.norm(g) < 1e-9}


def _golden(name):
    import os
    return np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", name + ".npz"))


def _ref_fp32_audio_err(case="mm_mse_small", prefix="grad/student.audio_encoder"):
    """Worst rel-L2 error of the reference's own fp32 run vs its float64 run over the
    audio-encoder gradients of the committed golden step (the fp32 chaos floor)."""
    f32, f64 = _golden(case), _golden(case + "_f64")
    worst = 0.0
    for k in f64.files:
        if k.startswith(prefix) and "@" not in k:
            b = f64[k].ravel()
            if np.linalg.norm(b) > 1e-9:
                worst = max(worst, rel(f32[k], b))
    return worst


AUDIO_TOL = max(1e-3, 1.5 * _ref_fp32_audio_err())


def check_grads(errs, audio_tol=None):
    """errs: {key: rel-L2}.  Audio-encoder tensors within the reference's fp32 floor, the rest
    within 1e-3, and the median tight."""
    audio_tol = AUDIO_TOL if audio_tol is None else audio_tol
    worst = sorted(errs.items(), key=lambda kv: -kv[1])[:5]
    print("worst grad rel errors:", worst, "audio bound", audio_tol)
    for k, e in errs.items():
        bound = audio_tol if k.startswith("student.audio_encoder") else 1e-3
        assert e < bound, (k, e, bound)
    assert np.median(list(errs.values())) < 1e-4, np.median(list(errs.values()))


@pytest.mark.parametrize("mode", ["mse", "default", "infonce", "semi_supervised"])
def test_step_matches_oracle(mode):
    from avdino.engine import adam_step, ema_step
    E, D, P, B, G, L = 32, 32, 16, 4, 2, 4
    store, eng, state = build(mode, E, D, P, 201)
    batch = make_multimodal_batch(B, G, L, 2001)
    ref = O.multimodal_step(state, batch, mode, HP)

    loss = eng.forward(dev_batch(batch))
    s_out, t_out = eng.outputs()
    assert abs(loss.item() - ref["loss"]) < 3e-5, (loss.item(), ref["loss"])
    assert rel(host(s_out), ref["s_out"]) < 1e-5
    assert rel(host(t_out), ref["t_out"]) < 1e-5
    eng.update_center()
    assert rel(host(store["center"]), ref["center_after"]) < 1e-5
    ema_step(store, HP["momentum"])
    eng.backward()
    zero = zero_grad_keys(ref["grads"])
    assert sorted(store.live_keys) == sorted(ref["grads"].keys())
    errs = {}
    for k in store.live_keys:
        g = host(store.grad_of(k))
        if k in zero:
            assert np.linalg.norm(g) <= 1e-4, (k, np.linalg.norm(g))
        else:
            errs[k] = rel(g, ref["grads"][k])
    check_grads(errs)
    new = ref["state"]
    for k in store.t_offs:
        assert rel(host(store[k]), new[k]) < 1e-6, k
    for k in store.buffers:
        if k.endswith("running_mean") or k.endswith("running_var"):
            assert rel(host(store.buffers[k]), new[k]) < 1e-5, k
        elif k.endswith("num_batches_tracked"):
            assert int(store.buffers[k].item()) == int(new[k]), k
    # Adam on the arena == torch.optim.Adam semantics applied to the same gradients (the
    # first Adam step is ~lr*sign(g), so comparing against the oracle's own gradients would
    # only measure sign flips of near-zero gradient entries)
    ours = {k: host(store.grad_of(k)) for k in store.live_keys}
    pre = {k: host(store[k]) for k in store.live_keys}
    adam_step(store, eng.hp)
    post = O.adam_update_state(pre, ours, {}, 1, HP)
    for k in store.live_keys:
        assert rel(host(store[k]), post[k]) < 1e-6, k


def test_loss_curve_matches_oracle():
    E, D, P, B, G, L = 32, 32, 16, 4, 2, 4
    store, eng, state = build("mse", E, D, P, 202)
    st = {k: np.asarray(v, np.float64) if v.dtype != np.int64 else v for k, v in state.items()}
    opt, ref_curve, curve, from_ours = {}, [], [], []
    for step in range(4):
        b = make_multimodal_batch(B, G, L, 3000 + step)
        # the oracle re-run from the engine's own current state: isolates the step's math
        ours = {k: store[k].detach().double().cpu().numpy() for k in OS.multimodal_dino_spec("mse", E, D, P)}
        from_ours.append(O.multimodal_step(ours, b, "mse", HP)["loss"])
        r = O.multimodal_step(st, b, "mse", HP)
        ref_curve.append(r["loss"])
        st = O.adam_update_state(r["state"], r["grads"], opt, step + 1, HP)
        curve.append(eng.step(dev_batch(b)).item())
    print("curve", curve, "ref", ref_curve, "oracle@ours", from_ours)
    # every step's loss equals the oracle's on the same state (fp32 rounding only) ...
    np.testing.assert_allclose(curve, from_ours, atol=3e-5, rtol=0)
    # ... and the free-running curves stay within the fp32 chaos band: Adam's first steps are
    # ~lr*sign(g), so entries whose gradient (or whose ReLU / max-pool decision) sits within
    # rounding of zero flip between fp32 and float64 -- the reference's own fp32 run drifts
    # from its float64 run the same way (tests/golden: 1.8e-4 by step 4, 3e-4 by step 5)
    np.testing.assert_allclose(curve[:1], ref_curve[:1], atol=3e-5, rtol=0)
    np.testing.assert_allclose(curve, ref_curve, atol=1e-3, rtol=0)


def test_full_dims_loss_curve_matches_reference():
    """north_star's loss-curve bar: the fp32 engine, free-running over 5 steps at the reference
    dims (E=D=256, P=128, B=2, 2 global + 4 local views), against the REFERENCE's own float64
    curve (fixture mm_mse_full_f64, made by running the reference; same parameters and
    batches), within 1e-4 on every step where the reference's own fp32 run is within 1e-5 of
    its float64 run (all 5 steps: it drifts at most 3.6e-6)."""
    f64, f32 = _golden("mm_mse_full_f64"), _golden("mm_mse_full")
    E, D, P, B, G, L, pseed, bseed = [int(x) for x in f64["meta_dims"]]
    ref, ref32 = np.asarray(f64["curve"]), np.asarray(f32["curve"])
    assert len(ref) == 5
    held = np.abs(ref32 - ref) < 1e-5
    assert held.all(), (ref32 - ref)
    store, eng, _ = build("mse", E, D, P, pseed)
    curve = [eng.step(dev_batch(make_multimodal_batch(B, G, L, bseed + s))).item() for s in range(len(ref))]
    print("engine", curve, "reference f64", ref.tolist(), "diff", (np.array(curve) - ref).tolist())
    np.testing.assert_allclose(np.array(curve)[held], ref[held], atol=1e-4, rtol=0)


@pytest.mark.parametrize("mode", ["mse", "default"])
def test_simple_encoder_step_matches_reference(mode):
    """--model multi_simple (SimpleMultiModalEncoder, dino.py:214-234: the 3x3 image_encoder /
    audio_encoder with global average pooling) against the reference's own float64 step
    (fixtures mm_simple_{mse,default}_small_f64): loss 3e-5, outputs 1e-5, gradients within
    the 3x3 audio tower's reference fp32 floor."""
    from tests import golden_util as gu
    name = f"mm_simple_{mode}_small"
    fx = gu.load(name + "_f64")
    E, D, P, B, G, L, pseed, bseed = [int(x) for x in fx["meta_dims"]]
    store, eng, _ = build(mode, E, D, P, pseed, encoder="multi_simple")
    loss = eng.forward(dev_batch(make_multimodal_batch(B, G, L, bseed)))
    s_out, t_out = eng.outputs()
    assert abs(loss.item() - float(fx["loss"])) < 3e-5, (loss.item(), float(fx["loss"]))
    for k, v in (("s_out", s_out), ("t_out", t_out)):
        ok, msg = gu.compare(fx, k, host(v), rel=1e-5)
        assert ok, msg
    eng.update_center()
    eng.backward()
    zero = gu.zero_grad_keys(fx)
    live = [str(k) for k in fx["live_keys"]]
    assert sorted(live) == sorted(store.live_keys)
    audio_tol = max(1e-3, 1.5 * _ref_fp32_audio_err(name))
    errs = {}
    for k in live:
        g = host(store.grad_of(k))
        if "grad/" + k in zero:
            assert np.linalg.norm(g) <= 1e-4, (k, np.linalg.norm(g))
            continue
        ok, msg = gu.compare(fx, "grad/" + k, g, rel=audio_tol)
        assert ok, msg
        if "grad/" + k in fx:
            errs[k] = rel(g, fx["grad/" + k])
    check_grads(errs, audio_tol)


def test_step_is_deterministic():
    """Fixed-order reductions everywhere: two runs from the same state are bitwise equal."""
    outs = []
    for _ in range(2):
        store, eng, _ = build("mse", 32, 32, 16, 203)
        b = dev_batch(make_multimodal_batch(4, 2, 4, 4000))
        eng.step(b)
        eng.step(b)
        outs.append((store.student.clone(), store.teacher.clone(), store.grad.clone()))
    for a, b in zip(*outs):
        assert torch.equal(a, b)


def test_full_dims_step_matches_oracle():
    """Reference dims (E=D=256, P=128) at a small batch."""
    E, D, P, B, G, L = 256, 256, 128, 2, 2, 4
    store, eng, state = build("mse", E, D, P, 204)
    batch = make_multimodal_batch(B, G, L, 5000)
    ref = O.multimodal_step(state, batch, "mse", HP)
    loss = eng.forward(dev_batch(batch))
    assert abs(loss.item() - ref["loss"]) < 3e-5
    eng.update_center()
    eng.backward()
    zero = zero_grad_keys(ref["grads"])
    check_grads({k: rel(host(store.grad_of(k)), ref["grads"][k]) for k in store.live_keys
                 if k not in zero})


def test_bf16_step_close_to_oracle():
    """bf16 activation storage (fp32 accumulate / statistics): statistical tolerance."""
    E, D, P, B, G, L = 32, 32, 16, 8, 2, 4
    store, eng, state = build("mse", E, D, P, 205, act=torch.bfloat16)
    batch = make_multimodal_batch(B, G, L, 6000)
    ref = O.multimodal_step(state, batch, "mse", HP)
    loss = eng.forward(dev_batch(batch))
    assert abs(loss.item() - ref["loss"]) < 2e-2 * abs(ref["loss"])
    eng.update_center()
    eng.backward()
    zero = zero_grad_keys(ref["grads"])
    errs = sorted(((rel(host(store.grad_of(k)), ref["grads"][k]), k) for k in store.live_keys
                   if k not in zero), reverse=True)
    med = np.median([e for e, _ in errs])
    # bf16 storage (8-bit mantissa) + bf16 MFMA operands: at B=8 the BatchNorm gradient sums
    # (large cancelling terms) amplify rounding; statistical agreement only
    assert med < 0.2 and errs[0][0] < 0.6, (med, errs[:6])
