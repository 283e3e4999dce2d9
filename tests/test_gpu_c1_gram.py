"""Audio conv1 BN statistics from the patch Gram (include/avdino.h avd_cl_c1_gram*), VERDICT r3
item 3.  The audio conv1 (1->8, 5x5 pad 2 on 112x112; reference dino.py:441-452
CentralUnimodalAudio conv1 -> BatchNorm2d(8) -> ReLU -> MaxPool) has a 25-wide patch, so its
per-channel sum y and sum y^2 follow from the 25x25 patch Gram G and patch sums S of the INPUT:
    sum y = w.S + n b,  sum y^2 = w^T G w + 2 b w.S + n b^2
and the routed backward needs the same G and S.  One forward pass (avd_cl_c1_gram) replaces the
recompute stats pass, and the backward's moments pass drops its Gram half
(avd_cl_c1_moments_codes_ng + avd_cl_c1_codes_combine_gram).

Checked here against float64 of the exact conv output w . x25 + b (w rounded to bf16 as the
kernels use it): mean / invstd / scale / shift / running stats within 1e-5 (2e-4 for the variance
of a strongly off-centre channel, where E[y^2] - mean^2 cancels), the Gram rows within 1e-6 of
the Gram half of the full routed moments pass (fp32 sums of the same products, rows split
differently), and dW / dgamma / dbeta / coefficients from the split path within 1e-5 of the full
routed combine."""
import pytest

torch = pytest.importorskip("torch")
F = pytest.importorskip("torch.nn.functional")

pytestmark = pytest.mark.gpu

T = torch.bfloat16
F64 = torch.float64
H, C, K, PAD = 112, 8, 5, 2


@pytest.fixture(scope="module")
def ops():
    from avdino import ops as _ops
    return _ops


def grel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def layout(ops, w):
    wk = torch.empty(ops.cl_weight_elems(C, 1, K, 0), device="cuda", dtype=T)
    ops.cl_weight_layout(w.float().contiguous(), wk, 0)
    return wk


def truth(x, w, bias, B):
    """float64 per-group mean and biased variance of y = conv(x, w) + b, plus G and S."""
    N = x.shape[0]
    G = N // B
    w64 = w.view(C, 25).to(F64)
    s1 = torch.zeros(G, C, device="cuda", dtype=F64)
    s2 = torch.zeros(G, C, device="cuda", dtype=F64)
    gram = torch.zeros(G, 25, 25, device="cuda", dtype=F64)
    sx = torch.zeros(G, 25, device="cuda", dtype=F64)
    step = 64
    for a in range(0, N, step):
        b = min(N, a + step)
        u = F.unfold(x[a:b].permute(0, 3, 1, 2).to(F64), K, padding=PAD)        # [n, 25, H*H]
        y = torch.einsum("ct,ntp->ncp", w64, u) + bias.to(F64)[None, :, None]
        for gi in range(a // B, (b - 1) // B + 1):
            lo, hi = max(a, gi * B) - a, min(b, (gi + 1) * B) - a
            s1[gi] += y[lo:hi].sum((0, 2))
            s2[gi] += (y[lo:hi] ** 2).sum((0, 2))
            gram[gi] += torch.einsum("nip,njp->ij", u[lo:hi], u[lo:hi])
            sx[gi] += u[lo:hi].sum((0, 2))
    n = float(B * H * H)
    mean = s1 / n
    var = s2 / n - mean * mean
    return mean, var, gram, sx


@pytest.mark.parametrize("N,B,off", [(24, 8, 0.0), (320, 32, 0.0), (320, 32, 3.0), (7168, 1024, 0.0)])
def test_gram_stats(ops, N, B, off):
    G = N // B
    g = torch.Generator(device="cuda").manual_seed(23 + N)
    x = torch.rand((N, H, H, 1), generator=g, device="cuda").to(T)
    w = ((torch.rand((C, 1, K, K), generator=g, device="cuda") * 2 - 1) / 5).to(T).float()
    bias = (torch.rand((C,), generator=g, device="cuda") * 0.2 - 0.1) + off
    if off:
        w[::2] = w[::2].abs()          # half the channels strongly off-centre (mean >> std)
    gamma = torch.rand((C,), generator=g, device="cuda") * 0.4 + 0.8
    beta = torch.rand((C,), generator=g, device="cuda") * 0.4 - 0.2
    wk = layout(ops, w)
    R, gc = ops.c1_codes_rows(N, B, H, H), ops.c1_gram_cols()
    assert R > 0 and gc == 650
    parts = torch.full((R * G * gc,), float("nan"), device="cuda")
    ops.c1_gram(x, parts, N, B, H, H)
    gram = torch.empty(G * gc, device="cuda")
    ops.sum_rows(parts, R, G * gc, gram)
    bn = torch.empty(4, G * C, device="cuda")
    rm0 = torch.rand((C,), generator=g, device="cuda")
    rv0 = torch.rand((C,), generator=g, device="cuda") + 0.5
    rm, rv = rm0.clone(), rv0.clone()
    n = B * H * H
    ops.c1_gram_finalize(gram, wk, bias, gamma, beta, n, bn[0], bn[1], bn[2], bn[3], rm, rv, G)
    mean, var, gram64, sx64 = truth(x, w, bias, B)
    gh = gram.view(G, gc).double()
    assert grel(gh[:, :625].view(G, 25, 25), gram64) < 1e-6
    assert grel(gh[:, 625:], sx64) < 1e-6
    iv = 1 / torch.sqrt(var + 1e-5)
    sc = gamma.double()[None] * iv
    sf = beta.double()[None] - mean * sc
    tol = 2e-4 if off else 1e-5
    print(f"N={N} off={off}: mean {grel(bn[0].view(G, C), mean):.2e} invstd {grel(bn[1].view(G, C), iv):.2e}"
          f" shift {grel(bn[3].view(G, C), sf):.2e} |mean|/std {(mean.abs() * iv).max().item():.1f}")
    assert grel(bn[0].view(G, C), mean) < 1e-5
    assert grel(bn[1].view(G, C), iv) < tol
    assert grel(bn[2].view(G, C), sc) < tol
    assert grel(bn[3].view(G, C), sf) < tol
    erm, erv = rm0.double(), rv0.double()
    for gi in range(G):
        erm = 0.9 * erm + 0.1 * mean[gi]
        erv = 0.9 * erv + 0.1 * var[gi] * n / (n - 1)
    assert grel(rm, erm) < 1e-5 and grel(rv, erv) < tol


@pytest.mark.parametrize("N,B", [(24, 8), (7168, 1024)])
def test_split_backward_matches_full(ops, N, B):
    """avd_cl_c1_moments_codes_ng + avd_cl_c1_codes_combine_gram (Gram from the forward's
    avd_cl_c1_gram) against the full routed pass avd_cl_c1_moments_codes + avd_cl_c1_codes_combine
    on the same codes: dW / dgamma / dbeta / coefficients within 1e-5 (the dbias, analytically 0,
    within 1e-6 of the largest)."""
    G = N // B
    Hp = H // 2
    g = torch.Generator(device="cuda").manual_seed(29 + N)
    x = torch.rand((N, H, H, 1), generator=g, device="cuda").to(T)
    w = ((torch.rand((C, 1, K, K), generator=g, device="cuda") * 2 - 1) / 5).to(T).float()
    bias = torch.rand((C,), generator=g, device="cuda") * 0.2 - 0.1
    gamma = torch.rand((C,), generator=g, device="cuda") * 0.4 + 0.8
    beta = torch.rand((C,), generator=g, device="cuda") * 0.4 - 0.2
    wk = layout(ops, w)
    R, gc, mc = ops.c1_codes_rows(N, B, H, H), ops.c1_gram_cols(), ops.c1_codes_cols()
    parts = torch.empty(R * G * max(gc, mc), device="cuda")
    ops.c1_gram(x, parts, N, B, H, H)
    gram = torch.empty(G * gc, device="cuda")
    ops.sum_rows(parts, R, G * gc, gram)
    bn = torch.empty(4, G * C, device="cuda")
    ops.c1_gram_finalize(gram, wk, bias, gamma, beta, B * H * H, bn[0], bn[1], bn[2], bn[3], None, None, G)
    z = torch.empty(N, Hp, Hp, C, device="cuda", dtype=T)
    codes = torch.empty((N * Hp * Hp,), device="cuda", dtype=torch.int32)
    ops.c1_apply_codes(x, wk, bias, bn[2], bn[3], z, codes, N, B, H, H)
    gz = ((torch.rand((N, Hp, Hp, C), generator=g, device="cuda") * 2 - 1)).to(T)
    outs = []
    for split in (False, True):
        parts.fill_(float("nan"))
        (ops.c1_moments_codes_ng if split else ops.c1_moments_codes)(x, gz, codes, parts, N, B, H, H)
        mom = torch.empty(G * mc, device="cuda")
        ops.sum_rows(parts, R, G * mc, mom)
        r = [torch.empty(C * 25, device="cuda")] + [torch.empty(C, device="cuda") for _ in range(3)]
        coef = torch.empty(G * C * 3, device="cuda")
        if split:
            ops.c1_codes_combine_gram(mom, gram, wk, bias, gamma, bn[0], bn[1], B * H * H, *r, coef, G)
        else:
            mh = mom.view(G, mc)
            print("Gram half vs the Gram pass", grel(mh[:, C * 25:C * 25 + 650], gram.view(G, gc)))
            assert grel(mh[:, C * 25:C * 25 + 650], gram.view(G, gc)) < 1e-6
            ops.c1_codes_combine(mom, wk, bias, gamma, bn[0], bn[1], B * H * H, *r, coef, G)
        outs.append(r + [coef])
    for a, b in zip(*outs):
        print("split vs full", grel(b, a))
        assert grel(b, a) < 1e-5 or (a - b).abs().max() < 1e-6 * a.abs().max().clamp_min(1.0), grel(a, b)
