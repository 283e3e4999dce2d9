"""The 3x3 first layer (Conv2d(1, 32, 3, padding=1) -> BN2d -> ReLU -> MaxPool2d of the SimCLR /
unimodal encoders' image_encoder / audio_encoder, dino.py:18-73) with its training backward routed
by the forward's codes (avd_cl_c1r3_apply_codes + avd_cl_c1r3_moments_codes +
avd_cl_c1r3_codes_combine), at config 4's size (N = 2048 per tower call) and small N:

* the codes-writing BN -> ReLU -> pool pass's pooled map is bit-identical to c1r3 pass 1 (the
  recomputing apply the engine used before) and to the stored-y chain;
* the moments (M = sum dz x9, Gram, S, sum dz) within 1e-5 of float64 from the same routing
  (first max of relu(bn(y)) of the stored bf16 y, only a positive max routes);
* dW, dgamma, dbeta and the BN-backward coefficients within 1e-5 / 1e-6 of the float64 formulas,
  and dW within 3e-3 of the recomputing moments pass (c1r3 pass 4, whose BN sums are f32);
* in the engine, a SimCLR audio/audio step: each route's first-layer gradients against float64
  autograd of the layer on the same input and pooled gradient (routed 1e-4, recomputing 1e-2),
  loss and every other gradient bit for bit between the routes."""
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
F = pytest.importorskip("torch.nn.functional")

from tests.test_gpu_benchsize import F64, T, _chunks, grel, layout, rnd  # noqa: E402


@pytest.fixture(scope="module")
def ops():
    from avdino import ops as _ops
    return _ops


@pytest.mark.parametrize("H,N,B", [(28, 24, 8), (112, 16, 8), (28, 2048, 2048), (112, 2048, 2048)])
def test_conv1_3x3_routed_backward(ops, H, N, B):
    C, K, pad = 32, 3, 1
    G, Hp, KK = N // B, H // 2, 9
    g = torch.Generator(device="cuda").manual_seed(23 + H)
    x = rnd(g, (N, H, H, 1), 0, 1, T)
    w = rnd(g, (C, 1, K, K)).to(T).float() / 3
    bias = rnd(g, (C,), -0.1, 0.1)
    wk = layout(ops, w, 0)
    y = torch.empty(N, H, H, C, device="cuda", dtype=T)
    R0 = ops.cl_stat_rows(H, H, B, K, 1, C, T)
    st0 = torch.empty(C * G * R0 * 2, device="cuda")
    ops.cl_conv_fwd(x, wk, bias, y, st0, N, B, 1, H, H, C, K, pad)
    gamma, beta = rnd(g, (C,), 0.8, 1.2), rnd(g, (C,), -0.2, 0.2)
    bn = torch.empty(4, G * C, device="cuda")
    ops.bn_finalize(st0, G, R0, C, B * H * H, gamma, beta, bn[0], bn[1], bn[2], bn[3])
    z0 = torch.empty(N, Hp, Hp, C, device="cuda", dtype=T)
    ops.cl_bn_relu_pool(y, bn[2], bn[3], z0, 0, N, B, C, H, H)
    z1 = torch.full_like(z0, float("nan"))
    ops.cl_c1_recompute(ops.C1_APPLY, x, wk, bias, N, B, 1, H, H, C, K, pad, scale=bn[2], shift=bn[3], z=z1)
    z2 = torch.full_like(z0, float("nan"))
    codes = torch.full((N * Hp * Hp * C // 4,), -1, device="cuda", dtype=torch.int16)
    ops.c1r3_apply_codes(x, wk, bias, bn[2], bn[3], z2, codes, N, B, H, H, C)
    assert torch.equal(z1, z2) and torch.equal(z0, z2)
    gz = rnd(g, (N, Hp, Hp, C), dtype=T)
    Rc, mc = ops.c1r3_codes_rows(N, B, H, H, C), ops.c1r3_codes_cols(C)
    assert Rc > 0 and mc == C * KK + KK * KK + KK + C
    parts = torch.full((Rc * G * mc,), float("nan"), device="cuda")
    ops.c1r3_moments_codes(x, wk, gz, codes, parts, N, B, H, H, C)
    mom = torch.empty(G * mc, device="cuda")
    ops.sum_rows(parts, Rc, G * mc, mom)
    dw = torch.empty(C * KK, device="cuda")
    dg, db, dbi = (torch.empty(C, device="cuda") for _ in range(3))
    coef = torch.empty(G * C * 3, device="cuda")
    ops.c1r3_codes_combine(mom, wk, bias, gamma, bn[0], bn[1], B * H * H, dw, dg, db, dbi, coef, G, C)
    # float64 from the same routing
    gram = torch.zeros(G, KK, KK, device="cuda", dtype=F64)
    sx = torch.zeros(G, KK, device="cuda", dtype=F64)
    mz = torch.zeros(G, C, KK, device="cuda", dtype=F64)
    s1 = torch.zeros(G, C, device="cuda", dtype=F64)
    sc, sf = bn[2].view(G, C).to(F64), bn[3].view(G, C).to(F64)
    for a, b in _chunks(N, H * H * KK * 2 * 8):
        u = F.unfold(x[a:b].permute(0, 3, 1, 2).to(F64), K, padding=pad)     # [n, 9, H*H]
        for gi in range(a // B, (b - 1) // B + 1):
            lo, hi = max(a, gi * B) - a, min(b, (gi + 1) * B) - a
            n = hi - lo
            gram[gi] += torch.einsum("nip,njp->ij", u[lo:hi], u[lo:hi])
            sx[gi] += u[lo:hi].sum((0, 2))
            zz = torch.relu(y[a + lo:a + hi].to(F64) * sc[gi] + sf[gi])
            zw = zz.view(n, Hp, 2, Hp, 2, C).permute(0, 1, 3, 5, 2, 4).reshape(n, Hp, Hp, C, 4)
            best, am = zw.max(-1)
            gzw = gz[a + lo:a + hi].to(F64)
            dzw = torch.where((torch.arange(4, device="cuda") == am[..., None]) & (best[..., None] > 0),
                              gzw[..., None], torch.zeros((), device="cuda", dtype=F64))
            dz = dzw.view(n, Hp, Hp, C, 2, 2).permute(0, 1, 4, 2, 5, 3).reshape(n, H * H, C)
            mz[gi] += torch.einsum("npc,ntp->ct", dz, u[lo:hi])
            s1[gi] += dz.sum((0, 1))
    mh = mom.view(G, mc).to(F64)
    assert grel(mh[:, :C * KK].view(G, C, KK), mz) < 1e-5
    assert grel(mh[:, C * KK:C * KK + KK * KK].view(G, KK, KK), gram) < 1e-5
    assert grel(mh[:, C * KK + KK * KK:C * KK + KK * KK + KK], sx) < 1e-5
    assert grel(mh[:, C * KK + KK * KK + KK:], s1) < 1e-5
    w64 = w.view(C, KK).to(T).to(F64)
    b64 = bias.to(F64)
    n = float(B * H * H)
    sy = torch.einsum("ct,gct->gc", w64, mz) + b64[None] * s1
    mu, iv, ga = bn[0].view(G, C).to(F64), bn[1].view(G, C).to(F64), gamma.to(F64)[None]
    s2 = (sy - mu * s1) * iv
    k1, kx, k0 = ga * iv, -ga * iv * iv * s2 / n, -ga * iv * s1 / n + ga * iv * iv * mu * s2 / n
    syg = torch.einsum("ct,gts->gcs", w64, gram) + b64[None, :, None] * sx[:, None, :]
    dw64 = (k1[..., None] * mz + kx[..., None] * syg + k0[..., None] * sx[:, None, :]).sum(0)
    k3 = coef.view(G, C, 3).to(F64)
    assert grel(k3, torch.stack([k1, kx, k0], -1)) < 1e-6
    assert grel(dg, s2.sum(0)) < 1e-5 and grel(db, s1.sum(0)) < 1e-5
    assert grel(dw, dw64) < 1e-5, grel(dw, dw64)
    # the recomputing moments pass (c1r3 pass 4) on the same state
    R4 = ops.cl_c1_recompute_rows(ops.C1_REDUCE_MOMENTS, T, N, B, 1, H, H, C, K, pad)
    mc4 = ops.c1_moment_cols(C, K)
    m4 = torch.empty(C * G * R4 * 2 + R4 * G * mc4, device="cuda")
    ops.cl_c1_recompute(ops.C1_REDUCE_MOMENTS, x, wk, bias, N, B, 1, H, H, C, K, pad, scale=bn[2],
                        shift=bn[3], mean=bn[0], invstd=bn[1], gz=gz, out=m4)
    cf4 = torch.empty(G * C * 3, device="cuda")
    dg4, db4 = torch.empty(C, device="cuda"), torch.empty(C, device="cuda")
    ops.bn_bwd_finalize(m4, G, R4, C, B * H * H, gamma, bn[0], bn[1], cf4, dg4, db4, None)
    mom4 = torch.empty(G * mc4, device="cuda")
    ops.sum_rows(m4, R4, G * mc4, mom4, off=C * G * R4 * 2)
    d4 = torch.empty(C * KK, device="cuda")
    ops.cl_c1_recompute_combine(mom4, cf4, wk, bias, d4, G, C, K)
    assert grel(dw, d4) < 3e-3 and grel(db, db4) < 1e-5, (grel(dw, d4), grel(db, db4))


def _simclr_step(monkeypatch, codes, label):
    from avdino.engine import ConvBranch, Hyper, SimCLREngine
    from avdino.params import ParamStore
    from avdino.spec import simclr_sd
    from oracle.params import make_simclr_batch
    from tests.first_layer_truth import compare, record
    with monkeypatch.context() as mp:
        mp.setattr(ConvBranch, "CODES3", codes)
        calls = record(mp)
        store = ParamStore(simclr_sd(64, 32), "cuda", seed=3, has_teacher=False,
                           groups=list(SimCLREngine.GROUPS))
        eng = SimCLREngine(store, 64, 32, Hyper(lr=1e-3), act_dtype=torch.bfloat16)
        b = {k: torch.from_numpy(v).cuda() for k, v in make_simclr_batch(64, 6300).items()}
        loss = eng.forward(b, 1)          # audio / audio: both towers' first layer is the 112^2 one
        eng.backward()
        torch.cuda.synchronize()
        assert calls
        return loss.item(), store, compare(calls, store, label)


def test_simclr_step_first_layer_routes_against_float64(monkeypatch):
    """SimCLR audio/audio step: the routed 3x3 first-layer backward and the recomputing one each
    against float64 autograd of the layer (tests/first_layer_truth.py): routed within 1e-4
    (measured 1.4e-5), recomputing within 1e-2 (8.4e-3 on dgamma), statistics within 5e-5; loss and every other gradient bitwise equal between the routes."""
    l0, s0, e0 = _simclr_step(monkeypatch, False, "recompute")
    l1, s1, e1 = _simclr_step(monkeypatch, True, "routed")
    assert l0 == l1
    for n, e in e1.items():
        if n.endswith(("|mean", "|invstd")):
            assert e < 5e-5, (n, e)
        elif n.endswith("|abs"):
            assert e < 1e-3 and e0[n] < 1e-3, (n, e, e0[n])
        else:
            assert e < 1e-4, (n, e)
            assert e0[n] < 1e-2, (n, e0[n])
    first = [k for k in s0.live_keys if ".encoder.0." in k or ".encoder.1." in k]   # conv1 / bn1
    assert first, s0.live_keys[:8]
    for k in s0.live_keys:
        if k not in first:
            assert torch.equal(s0.grad_of(k), s1.grad_of(k)), k
