"""The first-layer training routes of the bf16 step against each other.

* The image conv1's pixel-major passes (avd_cl_c1r5_stats / avd_cl_c1r5_apply_codes) and its
  routed moments pass (avd_cl_c1r5_moments_codes) with the grid_cap option forcing a handful of
  blocks, so every block walks many samples across BN-group boundaries: the pooled map and the
  codes are bit-identical to the uncapped launch, the statistics and moments are fp32 sums in
  another order (rel 1e-6).
* The engine's first-layer backward routes -- routed by the forward pooling pass's codes, and
  the recomputing moments pass (ConvBranch.CODES = False) -- and its two audio conv1 statistics routes
  (patch Gram, ConvBranch.GRAM; recomputing statistics pass) each against float64 autograd of
  the layer on the same input, weights and pooled gradient (tests/first_layer_truth.py): the
  routed backward within 1e-4, the recomputing one (sum dz * y at the bf16-rounded y) within
  5e-3, the Gram statistics within 1e-5; every gradient outside the first layers is bitwise equal
  between the backward routes.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

T = torch.bfloat16
F64 = torch.float64


@pytest.fixture(scope="module")
def ops():
    from avdino import ops as _ops
    return _ops


def grel(a, b):
    a, b = a.to(F64).reshape(-1), b.to(F64).reshape(-1)
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


@pytest.mark.parametrize("cap", [3, 7])
def test_image_conv1_passes_capped_grid(ops, avd_opts, cap):
    N, B, H, C = 96, 32, 28, 32
    G, Hp = N // B, H // 2
    g = torch.Generator(device="cuda").manual_seed(23)
    x = (torch.randint(0, 256, (N, H, H, 1), generator=g, device="cuda").float() / 255).to(T)
    w = ((torch.rand(C, 1, 5, 5, generator=g, device="cuda") - 0.5) / 2.5).to(T).float()
    bias = (torch.rand(C, generator=g, device="cuda") - 0.5) / 5
    wk = torch.empty(ops.cl_weight_elems(C, 1, 5, False), device="cuda", dtype=T)
    ops.cl_weight_layout(w.contiguous(), wk, False)
    gamma = 0.8 + 0.4 * torch.rand(C, generator=g, device="cuda")
    beta = (torch.rand(C, generator=g, device="cuda") - 0.5) / 2.5
    gz = ((torch.rand(N, Hp, Hp, C, generator=g, device="cuda") - 0.5) * 2).to(T)

    def stats():
        R = ops.c1r5_stats_rows(N, B, H, H)
        sp = torch.empty(C * G * R * 2, device="cuda")
        ops.c1r5_stats(x, wk, bias, sp, N, B, H, H)
        bn = torch.empty(4, G * C, device="cuda")
        ops.bn_finalize(sp, G, R, C, B * H * H, gamma, beta, bn[0], bn[1], bn[2], bn[3])
        return bn

    def apply(bn):
        z = torch.full((N, Hp, Hp, C), float("nan"), device="cuda", dtype=T)
        codes = torch.full((N * Hp * Hp * 8,), -1, device="cuda", dtype=torch.int16)
        ops.c1r5_apply_codes(x, wk, bias, bn[2], bn[3], z, codes, N, B, H, H)
        return z, codes

    def moments(codes):
        Rc, mc = ops.c1r5_codes_rows(N, B, H, H), ops.c1r5_codes_cols()
        parts = torch.empty(Rc * G * mc, device="cuda")
        ops.c1r5_moments_codes(x, gz, codes, parts, N, B, H, H)
        mom = torch.empty(G * mc, device="cuda")
        ops.sum_rows(parts, Rc, G * mc, mom)
        return mom

    bn0 = stats()
    z0, c0 = apply(bn0)
    m0 = moments(c0)
    avd_opts(grid_cap=cap)
    bn1 = stats()
    z1, c1 = apply(bn0)                   # the uncapped coefficients: a block-independent map
    m1 = moments(c0)
    avd_opts(grid_cap=0)
    assert grel(bn1, bn0) < 1e-6
    assert torch.equal(z1, z0) and torch.equal(c1, c0)
    assert grel(m1, m0) < 1e-6


def _engine_step(monkeypatch, codes=True, gram=True, label=""):
    """One MultiCentral (mse) forward + backward at B = 64 with the first-layer flags set; returns
    the loss, every gradient, the running statistics and the first layers' errors against the
    float64 truth (tests/first_layer_truth.py)."""
    from avdino.engine import ConvBranch, Hyper, MultiCentralEngine
    from avdino.params import ParamStore
    from avdino.spec import multimodal_dino_sd
    from oracle.params import make_state
    from oracle import spec as OS
    from tests.first_layer_truth import compare, record
    E = D = 64
    P, B, G, L = 32, 64, 2, 4
    state = make_state(OS.multimodal_dino_spec("mse", E, D, P), 411)
    gen = torch.Generator(device="cuda").manual_seed(412)

    def px(*s):
        return torch.randint(0, 256, s, generator=gen, device="cuda", dtype=torch.int32).float() / 255

    batch = dict(g_img=px(B, G, 1, 28, 28), g_aud=px(B, G, 1, 112, 112), l_img=px(B, L, 1, 28, 28),
                 l_aud=px(B, L, 1, 112, 112), image=px(B, 1, 28, 28), audio=px(B, 1, 112, 112))
    with monkeypatch.context() as mp:
        mp.setattr(ConvBranch, "CODES", codes)
        mp.setattr(ConvBranch, "GRAM", gram)
        calls = record(mp)
        store = ParamStore(multimodal_dino_sd("mse", E, D, P), "cuda")
        store.load_state_dict({k: torch.from_numpy(np.array(v)) for k, v in state.items()})
        eng = MultiCentralEngine(store, "mse", E, D, P, Hyper(dropout=0.0, fusion_dropout=0.0),
                                 act_dtype=torch.bfloat16)
        loss = eng.forward(batch).item()
        eng.backward()
        torch.cuda.synchronize()
        assert len(calls) == 2, len(calls)          # the student's image and audio conv1
        errs = compare(calls, store, label)
        return loss, {k: store.grad_of(k).detach().clone() for k in store.live_keys}, \
            {k: store[k].detach().clone() for k in store.buffers if "running_" in k}, errs


FIRST = ("student.audio_encoder.0.conv1.", "student.audio_encoder.0.bn1.",
         "student.image_encoder.0.conv1.", "student.image_encoder.0.bn1.")


def test_engine_first_layer_routes_against_float64(monkeypatch):
    """Both first-layer backward routes of the bf16 step against float64 autograd of the layer
    (same input, weights, pooled gradient): the routed one (codes) forms its moments from the
    exact conv output in fp32 and is within 1e-4 (dW, dgamma, dbeta; measured 4e-7 audio, 2.4e-5
    image); the recomputing one forms sum dz*y at the bf16-rounded y and is within 1e-2 (measured
    7.5e-3 on dgamma).  Batch statistics within 5e-5 of float64.  The forward is one launch sequence for
    both (bitwise equal loss) and every gradient outside the two first layers is bitwise equal."""
    l1, g1, _, e1 = _engine_step(monkeypatch, codes=True, label="routed")
    l0, g0, _, e0 = _engine_step(monkeypatch, codes=False, label="recompute")
    assert l1 == l0
    for n, e in e1.items():
        if n.endswith(("|mean", "|invstd")):
            assert e < 5e-5, (n, e)     # fp32 statistics passes (the audio Gram's: 1e-6 below)
        elif n.endswith("|abs"):
            assert e < 1e-3 and e0[n] < 1e-3, (n, e, e0[n])
        else:
            assert e < 1e-4, (n, e)
            assert e0[n] < 1e-2, (n, e0[n])
    for k in g0:
        if not k.startswith(FIRST):
            assert torch.equal(g1[k], g0[k]), k


def test_engine_gram_stats_against_float64(monkeypatch):
    """Audio conv1 BN statistics from the patch Gram (ConvBranch.GRAM = True, avd_cl_c1_gram) and from
    the recomputing statistics pass (False), each against float64 of the same layer: the Gram route's
    batch mean / invstd within 1e-6 (measured 3e-7; the fp32 statistics pass 1.2e-5) and its
    routed gradients within 1e-4; the loss of the two
    routes agrees to 1e-3 and the running statistics to 1e-4."""
    l1, g1, r1, e1 = _engine_step(monkeypatch, gram=True, label="gram")
    l0, g0, r0, e0 = _engine_step(monkeypatch, gram=False, label="stats pass")
    print("loss", l1, l0, "rel", abs(l1 - l0) / abs(l0))
    for n, e in e1.items():
        if n.endswith(("|mean", "|invstd")):
            assert e < (1e-6 if "audio" in n else 5e-5), (n, e)
        elif n.endswith("|abs"):
            assert e < 1e-3, (n, e)
        else:
            assert e < 1e-4, (n, e)
    assert abs(l1 - l0) <= 1e-3 * abs(l0)
    for k in r0:
        if "audio_encoder.0.bn1" in k:
            assert grel(r1[k], r0[k]) < 1e-4, (k, grel(r1[k], r0[k]))
