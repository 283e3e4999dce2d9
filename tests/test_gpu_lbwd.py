"""The fused audio-conv2 layer backward (avd_cl_layer_bwd, csrc/lbwd.hip)
against the three launches it replaces -- avd_cl_bn_bwd_apply (y + pooled gradient -> dY),
avd_cl_conv_dgrad (dX) and avd_cl_conv_wgrad (dW slabs) -- on the same bf16 operands:

* dX: the kernel computes two output rows per MFMA tile (row pairs: 15 k-steps over the 6 x 5
  dY window instead of 2 x 13), so the even rows keep conv_ws's DgrA2 k order (bit-identical)
  and the odd rows sum the same products in other k-step groups: equal to the separate input
  gradient up to one bf16 rounding step (|d| <= 2^-7 |dX| + 1e-5 max|dX|, >= 97 % of the values
  bit-identical), and within 1e-5 rel-L2 of float64 -- both when the kernel forms dY itself from
  y and the pooled gradient (bit-identical to bwd_apply) and when dY is given;
* dW (f32 slabs summed in float64 by avd_sum_rows, another slab partition) within 1e-6 of the
  separate weight gradient, and within 1e-5 of float64 of the same dY at small N;
* at config-2 size (N = 7168, B = 1024, 7 BN groups: every persistent block walks ~98 tiles),
  and at small N with a capped grid (many tiles per block, tiles of one sample split between
  blocks);
* in the engine: a bf16 step with the fused backward equals the three-launch step -- loss and
  every gradient tensor upstream of the layer bit for bit, the audio conv2 weight gradient
  within 1e-6, the audio conv1 / bn1 gradients (fed by dX) within 1e-3."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

T = torch.bfloat16
F64 = torch.float64
CIN, COUT, K, PAD, H = 8, 16, 5, 2, 56


def _operands(N, B, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    G = N // B

    def r(*s, lo=-1.0, hi=1.0):
        return torch.rand(*s, generator=g, device="cuda") * (hi - lo) + lo
    y = r(N, H, H, COUT, lo=-2, hi=2).to(T)
    gout = (r(N, H // 2, H // 2, COUT) * 1e-3).to(T)
    x = r(N, H, H, CIN, lo=0, hi=2).to(T)
    scale, shift = r(G * COUT, lo=0.5, hi=1.5), r(G * COUT, lo=-0.5, hi=0.5)
    coef = torch.stack([r(G * COUT, lo=0.5, hi=1.5), r(G * COUT) * 1e-3, r(G * COUT) * 1e-4], 1).contiguous()
    w = r(COUT, CIN, K, K) * 0.1
    return y, gout, x, scale, shift, coef.view(-1), w


def _reference(ops, y, gout, x, scale, shift, coef, wk_d, N, B):
    dy = torch.empty_like(y)
    ops.cl_bn_bwd_apply(y, gout, 0, scale, shift, coef, dy, N, B, COUT, H, H)
    dx = torch.empty(N, H, H, CIN, dtype=T, device="cuda")
    ops.cl_conv_dgrad(dy, wk_d, dx, N, CIN, H, H, COUT, K, PAD)
    nch = ops.cl_wgrad_chunks(N, COUT, CIN, K)
    parts = torch.empty(nch * COUT * CIN * K * K, device="cuda")
    ops.cl_conv_wgrad(x, dy, parts, N, CIN, H, H, COUT, K, PAD)
    dw = torch.empty(COUT * CIN * K * K, device="cuda")
    ops.sum_rows(parts, nch, COUT * CIN * K * K, dw)
    return dy, dx, dw


def _fused(ops, y, gout, x, scale, shift, coef, dy, wk_d, N, B):
    slabs = ops.cl_layer_bwd_slabs(T, N, CIN, H, H, COUT, K, PAD)
    assert slabs > 0
    parts = torch.full((slabs * COUT * CIN * K * K,), float("nan"), device="cuda")
    dx = torch.full((N, H, H, CIN), float("nan"), device="cuda").to(T)
    ops.cl_layer_bwd(y, gout, scale, shift, coef, dy, x, wk_d, dx, parts, slabs, N, B, CIN, H, H, COUT, K, PAD)
    dw = torch.empty(COUT * CIN * K * K, device="cuda")
    ops.sum_rows(parts, slabs, COUT * CIN * K * K, dw)
    return dx, dw


def _wgrad64(x, dy):
    xp = torch.nn.functional.pad(x.to(F64), (0, 0, PAD, PAD, PAD, PAD))
    d = dy.to(F64).reshape(-1, COUT)
    dw = torch.zeros(COUT, CIN, K, K, dtype=F64, device="cuda")
    for i in range(K):
        for j in range(K):
            dw[:, :, i, j] = d.T @ xp[:, i:i + H, j:j + H, :].reshape(-1, CIN)
    return dw.reshape(-1)


def _rel(a, b):
    return ((a.double() - b.double()).norm() / b.double().norm()).item()


@pytest.mark.parametrize("N,B,cap", [(7168, 1024, None), (12, 4, 5), (10, 5, None)],
                         ids=["config2", "capped", "small"])
def test_layer_bwd_equals_apply_dgrad_wgrad(N, B, cap, avd_opts, capsys):
    from avdino import ops
    if cap:
        avd_opts(grid_cap=cap)
    y, gout, x, scale, shift, coef, w = _operands(N, B, 60 + N)
    wk_d = torch.empty(ops.cl_weight_elems(COUT, CIN, K, 1), dtype=T, device="cuda")
    ops.cl_weight_layout(w, wk_d, 1)
    dy, dx0, dw0 = _reference(ops, y, gout, x, scale, shift, coef, wk_d, N, B)
    dx1, dw1 = _fused(ops, y, gout, x, scale, shift, coef, None, wk_d, N, B)       # forms dY itself
    dx2, dw2 = _fused(ops, None, None, x, None, None, None, dy, wk_d, N, B)        # given dY
    torch.cuda.synchronize()
    e1, e2 = _rel(dw1, dw0), _rel(dw2, dw0)
    with capsys.disabled():
        print(f"\nlayer bwd N={N}: dW rel {e1:.1e} / {e2:.1e}")
    assert torch.equal(dx1, dx2) and torch.equal(dw1, dw2)
    d, r = (dx1.float() - dx0.float()).abs(), dx0.float().abs()
    same = (dx1 == dx0).float().mean().item()
    with capsys.disabled():
        print(f"  dX vs the separate dgrad: {same:.4f} bit-identical, max |d|/|dX| "
              f"{(d / r.clamp_min(1e-30)).max().item():.2e}")
    assert bool((d <= r * 2.0 ** -7 + 1e-5 * r.max()).all()) and same >= 0.97
    if N <= 12:
        w2 = w.flip(2, 3).transpose(0, 1).contiguous().double()
        ref = torch.nn.functional.conv2d(dy.double().permute(0, 3, 1, 2), w2, padding=K - 1 - PAD)
        assert _rel(dx1.permute(0, 3, 1, 2), ref) < 5e-3
    assert e1 < 1e-6, e1
    if N <= 12:
        assert _rel(dw1, _wgrad64(x, dy)) < 1e-5


def test_engine_step_with_fused_layer_bwd_equals_three_launches():
    from avdino import engine as EN
    from avdino.params import ParamStore
    from avdino.spec import multimodal_dino_sd
    from oracle import spec as OS
    from oracle.params import make_multimodal_batch, make_state
    E, D, P, B, G, L = 64, 64, 32, 32, 2, 2
    state = {k: torch.from_numpy(np.array(v)) for k, v in
             make_state(OS.multimodal_dino_spec("mse", E, D, P), 71).items()}
    batch = {k: torch.from_numpy(v).cuda() for k, v in make_multimodal_batch(B, G, L, 72).items()}
    out = {}
    for on in (False, True):
        EN.ConvBranch.LAYER_BWD = on
        try:
            store = ParamStore(multimodal_dino_sd("mse", E, D, P), "cuda")
            store.load_state_dict(state)
            eng = EN.MultiCentralEngine(store, "mse", E, D, P, EN.Hyper(dropout=0.0, fusion_dropout=0.0),
                                        act_dtype=T)
            loss = eng.forward(batch).item()
            eng.backward()
            torch.cuda.synchronize()
            out[on] = (loss, {k: store.grad_of(k).detach().clone() for k in store.live_keys})
        finally:
            EN.ConvBranch.LAYER_BWD = True
    (l0, g0), (l1, g1) = out[False], out[True]
    assert l0 == l1
    wkey = "student.audio_encoder.0.conv2.weight"
    for k in g0:
        if k == wkey:
            assert _rel(g1[k], g0[k]) < 1e-6, k
        elif k.startswith(("student.audio_encoder.0.conv1.", "student.audio_encoder.0.bn1.")):
            assert _rel(g1[k], g0[k]) < 1e-3, (k, _rel(g1[k], g0[k]))
        else:
            assert torch.equal(g1[k], g0[k]), k
