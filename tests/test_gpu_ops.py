"""Per-kernel parity: every libavdino entry point vs the float64 numpy oracle (oracle/),
on seeded inputs.  fp32 kernels: rel-L2 <= 2e-5 unless stated (reductions over up to
~10^5 terms); bf16 storage: rel-L2 <= 1e-2."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from oracle import numpy_oracle as O  # noqa: E402


def dev(a, dtype=None):
    t = torch.from_numpy(np.ascontiguousarray(a)).cuda()
    return t.to(dtype) if dtype is not None else t


def host(t):
    return t.detach().float().cpu().numpy().astype(np.float64)


def rel(a, b):
    a = np.asarray(a, np.float64).ravel()
    b = np.asarray(b, np.float64).ravel()
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30)


def _bf16_round(a):
    return torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(torch.bfloat16).float().numpy()


@pytest.fixture(scope="module")
def ops():
    from avdino import ops as _ops
    return _ops


@pytest.mark.parametrize("H", [28, 10, 7])
def test_bn_finalize_block_stats(ops, H):
    """BN2d(train, per group) statistics and the reference's sequential running-stat update
    from per-sample partial sums (the layout the channels-last conv epilogue writes)."""
    G, B, C = 3, 4, 16
    N = G * B
    g = np.random.default_rng(H)
    y = g.normal(0.3, 1.5, (N, C, H, H)).astype(np.float32)
    gamma = (1 + g.uniform(-0.2, 0.2, C)).astype(np.float32)
    beta = g.uniform(-0.2, 0.2, C).astype(np.float32)
    _, _, stats = O.bn_train_fwd(y.astype(np.float64), gamma.astype(np.float64), beta.astype(np.float64), G, (2, 3))
    rm_ref, rv_ref = O.bn_running_update(np.zeros(C), np.ones(C), stats)
    parts = np.stack([y.reshape(G, B, C, -1).transpose(2, 0, 1, 3).sum(-1),
                      (y.astype(np.float64) ** 2).reshape(G, B, C, -1).transpose(2, 0, 1, 3).sum(-1)], -1)
    st = torch.empty(4, G * C, device="cuda")
    rm = torch.zeros(C, device="cuda")
    rv = torch.ones(C, device="cuda")
    ops.bn_finalize(dev(parts.astype(np.float32)), G, B, C, B * H * H, dev(gamma), dev(beta),
                    st[0], st[1], st[2], st[3], rm, rv)
    np.testing.assert_allclose(host(st[0]).reshape(G, C), stats[0], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(host(rm), rm_ref, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(host(rv), rv_ref, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("R", [1, 2, 3, 4097, 50177])
def test_bn_finalize_chunked(ops, R):
    """Chunked two-pass statistics (in-place f64 chunk sums) incl. ragged last chunks and the
    sequential per-group running-stat updates."""
    G, C = 3, 5
    g = np.random.default_rng(R)
    parts = np.stack([g.normal(2.0, 1.0, (C, G, R)), g.uniform(5.0, 9.0, (C, G, R))], -1)
    count = R * 7
    gamma = 1 + g.uniform(-0.2, 0.2, C)
    beta = g.uniform(-0.2, 0.2, C)
    p32 = parts.astype(np.float32)
    s = p32.astype(np.float64).sum(2)
    mean = s[..., 0] / count
    var = s[..., 1] / count - mean ** 2
    rm, rv = np.zeros(C), np.ones(C)
    for k in range(G):
        rm = 0.9 * rm + 0.1 * mean[:, k]
        rv = 0.9 * rv + 0.1 * var[:, k] * count / (count - 1)
    st = torch.empty(4, G * C, device="cuda")
    trm, trv = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
    ops.bn_finalize(dev(p32), G, R, C, count, dev(gamma.astype(np.float32)),
                    dev(beta.astype(np.float32)), st[0], st[1], st[2], st[3], trm, trv)
    np.testing.assert_allclose(host(st[0]).reshape(G, C), mean.T, rtol=1e-6)
    np.testing.assert_allclose(host(st[1]).reshape(G, C), 1 / np.sqrt(var.T + 1e-5), rtol=1e-6)
    np.testing.assert_allclose(host(trm), rm, rtol=1e-6)
    np.testing.assert_allclose(host(trv), rv, rtol=1e-6)


@pytest.mark.parametrize("mode", [0, 1, 2])
@pytest.mark.parametrize("shape", [(70, 130, 45), (256, 3136, 300), (130, 64, 1000),
                                   (256, 512, 7168), (1000, 200, 3000), (2048, 1920, 72),
                                   (7168, 256, 1600)])
def test_gemm_modes_and_strides(ops, mode, shape):
    """f32 VALU (0), f32 MFMA (1), bf16 MFMA (2; operands rounded to bf16 on both sides).
    Shapes cover the 64x64 / 128x64 / 128x128 tiles, ragged M/N/K and deep-K split-K
    (the weight-gradient products, K = batch rows)."""
    g = np.random.default_rng(1)
    M, N, K = shape
    A = g.normal(size=(M, K)).astype(np.float32)
    Bm = g.normal(size=(K, N)).astype(np.float32)
    if mode == 2:
        A, Bm = _bf16_round(A), _bf16_round(Bm)
    bias = g.normal(size=N).astype(np.float32)
    # f32 accumulation error grows ~sqrt(K)
    tol = (1e-6 if mode < 2 else 1e-5) * max(1.0, np.sqrt(K / 1000))
    ref = A.astype(np.float64) @ Bm + bias
    C = torch.empty(M, N, device="cuda")
    ops.gemm(M, N, K, dev(A), K, 1, dev(Bm), N, 1, C, N, bias=dev(bias), mode=mode)
    assert rel(host(C), ref) < tol
    # A^T and B^T storage (scalar / transposed staging paths), alpha / beta
    At, Bt = dev(A.T.copy()), dev(Bm.T.copy())
    C2 = dev(np.ones((M, N), np.float32))
    ops.gemm(M, N, K, At, 1, M, Bt, 1, K, C2, N, alpha=0.5, beta=2.0, mode=mode)
    assert rel(host(C2), 0.5 * (A.astype(np.float64) @ Bm) + 2.0) < tol
    # column sums with a leading dimension and offset (Linear bias gradient)
    cs = torch.empty(N - 3, device="cuda")
    ops.sum_rows(dev(Bm), K, N - 3, cs, ld=N, off=3)
    assert rel(host(cs), Bm[:, 3:].astype(np.float64).sum(0)) < 1e-6


def test_linear_fwd_bwd_with_offsets(ops):
    g = np.random.default_rng(2)
    rows, In, O_ = 33, 40, 24
    x_big = g.normal(size=(rows, 2 * In)).astype(np.float32)   # x = cols [In, 2In) of a wider buffer
    w = g.normal(size=(O_, In)).astype(np.float32)
    b = g.normal(size=O_).astype(np.float32)
    x = x_big[:, In:].astype(np.float64)
    tx = dev(x_big)
    out = torch.empty(rows, 3 * O_, device="cuda")
    ops.linear_fwd(tx, dev(w), dev(b), out, rows, x_ld=2 * In, x_off=In, out_ld=3 * O_, out_off=O_)
    assert rel(host(out)[:, O_:2 * O_], x @ w.T + b) < 1e-6
    dout = g.normal(size=(rows, O_)).astype(np.float32)
    dw, db = torch.empty(O_, In, device="cuda"), torch.empty(O_, device="cuda")
    dx = torch.zeros(rows, 2 * In, device="cuda")
    ops.linear_bwd(dev(dout), tx, dev(w), dw, db, dx, rows, x_ld=2 * In, x_off=In, dx_ld=2 * In, dx_off=In)
    dxr, dwr, dbr = O.linear_bwd(dout.astype(np.float64), x, w.astype(np.float64))
    assert rel(host(dw), dwr) < 1e-6 and rel(host(db), dbr) < 1e-6
    assert rel(host(dx)[:, In:], dxr) < 1e-6 and np.abs(host(dx)[:, :In]).max() == 0


def test_projection_head_pieces(ops):
    """BN1d(train) + GELU + dropout(0) forward/backward."""
    g = np.random.default_rng(3)
    rows, C = 96, 512
    h = g.normal(0.2, 1.3, (rows, C)).astype(np.float32)
    gamma = (1 + g.uniform(-.2, .2, C)).astype(np.float32)
    beta = g.uniform(-.2, .2, C).astype(np.float32)
    z, bnc, _ = O.bn_train_fwd(h.astype(np.float64), gamma.astype(np.float64), beta.astype(np.float64), 1, ())
    a_ref = O.gelu_fwd(z)
    da = g.normal(size=(rows, C))
    dz_ref = O.gelu_bwd(da, z)
    dh_ref, dg_ref, db_ref = O.bn_train_bwd(dz_ref, bnc)
    th = dev(h)
    R = ops.colstats_parts(rows)
    parts = torch.empty(C * R * 2, device="cuda")
    piv = torch.empty(C, device="cuda")
    ops.colstats(th, rows, 1, C, parts, piv)
    st = torch.empty(4, C, device="cuda")
    ops.bn_finalize(parts, 1, R, C, rows, dev(gamma), dev(beta), st[0], st[1], st[2], st[3], pivot=piv)
    a = torch.empty_like(th)
    ops.act_fwd(th, a, 1, st[2], st[3], rows, 1, C, 0.0, 0)
    assert rel(host(a), a_ref) < 1e-5
    dz = torch.empty_like(th)
    ops.act_bwd(th, dev(da.astype(np.float32)), dz, 1, st[2], st[3], rows, 1, C, 0.0, 0)
    assert rel(host(dz), dz_ref) < 1e-5
    bp = torch.empty(C * R * 2, device="cuda")
    ops.bn1d_bwd_reduce(th, dz, st[0], st[1], rows, 1, C, bp)
    coef = torch.empty(C * 3, device="cuda")
    dg, db = torch.empty(C, device="cuda"), torch.empty(C, device="cuda")
    ops.bn_bwd_finalize(bp, 1, R, C, rows, dev(gamma), st[0], st[1], coef, dg, db, None)
    dh = torch.empty_like(th)
    ops.bn1d_bwd_apply(th, dz, coef, dh, rows, 1, C)
    assert rel(host(dg), dg_ref) < 1e-5 and rel(host(db), db_ref) < 1e-5
    assert rel(host(dh), dh_ref) < 1e-4


@pytest.mark.parametrize("G", [1, 3])
def test_bn1d_stats_offset_columns(ops, G):
    """BatchNorm1d statistics of columns whose mean is 100x their std (ReLU'd, pooled encoder
    features): the pivot-shifted sums keep the variance exact to f32 rounding."""
    g = np.random.default_rng(12)
    rpg, C = 40, 300
    h = (g.normal(0, 1, (G * rpg, C)) * 0.05 + g.uniform(2, 8, C)).astype(np.float32)
    R = ops.colstats_parts(rpg)
    parts = torch.empty(C * G * R * 2, device="cuda")
    piv = torch.empty(G * C, device="cuda")
    ops.colstats(dev(h), G * rpg, G, C, parts, piv)
    st = torch.empty(4, G * C, device="cuda")
    one, zero = torch.ones(C, device="cuda"), torch.zeros(C, device="cuda")
    ops.bn_finalize(parts, G, R, C, rpg, one, zero, st[0], st[1], st[2], st[3], pivot=piv)
    hs = h.astype(np.float64).reshape(G, rpg, C)
    assert rel(host(st[0]), hs.mean(1).ravel()) < 1e-7
    assert rel(host(st[1]), 1 / np.sqrt(hs.var(1) + 1e-5).ravel()) < 2e-6


def test_dropout_mask_statistics_and_consistency(ops):
    rows, C, p = 512, 256, 0.3
    x = torch.rand(rows, C, device="cuda") + 0.5
    out = torch.empty_like(x)
    ops.act_fwd(x, out, 0, None, None, rows, 1, C, p, 1234)
    keep = (out != 0).float().mean().item()
    assert abs(keep - (1 - p)) < 0.01
    kept = out[out != 0] / x[out != 0]
    assert torch.allclose(kept, torch.full_like(kept, 1 / (1 - p)), rtol=1e-6)
    dx = torch.empty_like(x)
    ops.act_bwd(x, torch.ones_like(x), dx, 0, None, None, rows, 1, C, p, 1234)
    assert torch.equal(dx != 0, out != 0)


@pytest.mark.parametrize("center_teacher", [False, True])
def test_dino_loss(ops, center_teacher):
    g = np.random.default_rng(4)
    V, T, B, P = 6, 2, 8, 128
    s = g.normal(size=(V, B, P)).astype(np.float32)
    t_raw = g.normal(size=(T, B, P)).astype(np.float32)
    center = g.normal(scale=0.1, size=P).astype(np.float32)
    loss_ref, ds_ref = O.dino_loss(s.astype(np.float64), (t_raw - center).astype(np.float64), 0.1, 0.04,
                                   center_teacher=center_teacher)
    parts = torch.empty(V * B, device="cuda")
    ds = torch.empty(V * B * P, device="cuda")
    cn = torch.empty(P, device="cuda")
    work = torch.empty((B + T * B) * P, device="cuda")
    ops.dino_loss(dev(s), dev(t_raw), dev(center), V, T, B, P, 0.1, 0.04, 0.9, center_teacher, parts,
                  ds, cn, work)
    assert abs(host(parts).sum() - loss_ref) < 1e-5
    assert rel(host(ds), ds_ref) < 1e-5
    cref = 0.9 * center + 0.1 * t_raw.reshape(-1, P).astype(np.float64).mean(0)
    assert rel(host(cn), cref) < 1e-6


def test_mse_l2norm_xent_ntxent(ops):
    g = np.random.default_rng(6)
    B, P = 16, 128
    a = g.normal(size=(B, P)).astype(np.float32)
    b = g.normal(size=(B, P)).astype(np.float32)
    lref, daref, dbref = O.mse_loss(a.astype(np.float64), b.astype(np.float64))
    parts, da, db = torch.empty(B, device="cuda"), torch.empty(B * P, device="cuda"), torch.empty(B * P, device="cuda")
    ops.mse_loss(dev(a), dev(b), B, P, parts, da, db)
    assert abs(host(parts).sum() - lref) < 1e-6
    assert rel(host(da), daref) < 1e-5 and rel(host(db), dbref) < 1e-5
    # InfoNCE pieces: l2norm + S + symmetric CE
    ta, tb = dev(a), dev(b)
    na, nb = torch.empty_like(ta), torch.empty_like(tb)
    nra, nrb = torch.empty(B, device="cuda"), torch.empty(B, device="cuda")
    ops.l2norm_fwd(ta, na, nra, B, P)
    ops.l2norm_fwd(tb, nb, nrb, B, P)
    S = torch.empty(B, B, device="cuda")
    ops.gemm(B, B, P, na, P, 1, nb, 1, P, S, B, alpha=1 / 0.07)
    dS = torch.empty(B, B, device="cuda")
    lp = torch.empty(2 * B, device="cuda")
    ops.softmax_xent(S, B, B, B, None, 1, False, False, 0.5 / B, lp[:B], dS, B, False)
    ops.softmax_xent(S, B, B, B, None, 1, True, False, 0.5 / B, lp[B:], dS, B, True)
    lref, diref, daref = O.infonce_loss(a.astype(np.float64), b.astype(np.float64))
    assert abs(host(lp).sum() / (2 * B) - lref) < 1e-5
    dni = torch.empty(B, P, device="cuda")
    ops.gemm(B, P, B, dS, B, 1, nb, P, 1, dni, P, alpha=1 / 0.07)
    dI = torch.empty(B, P, device="cuda")
    ops.l2norm_bwd(na, nra, dni, dI, B, P)
    assert rel(host(dI), diref) < 1e-5
    # NT-Xent: diagonal masked, targets (i+B) mod 2B
    reps = np.concatenate([a, b])
    lref, dref = O.nt_xent_loss(reps.astype(np.float64))
    tr = dev(reps)
    nr, nn_ = torch.empty_like(tr), torch.empty(2 * B, device="cuda")
    ops.l2norm_fwd(tr, nr, nn_, 2 * B, P)
    S2 = torch.empty(2 * B, 2 * B, device="cuda")
    ops.gemm(2 * B, 2 * B, P, nr, P, 1, nr, 1, P, S2, 2 * B, alpha=1 / 0.07)
    d2 = torch.empty_like(S2)
    lp2 = torch.empty(2 * B, device="cuda")
    ops.softmax_xent(S2, 2 * B, 2 * B, 2 * B, None, 2, False, True, 1 / (2 * B), lp2, d2, 2 * B, False)
    assert abs(host(lp2).mean() - lref) < 1e-5
    # CE with integer targets
    lab = g.integers(0, 10, B)
    logits = g.normal(size=(B, 10)).astype(np.float32)
    lref, dref = O.cross_entropy(logits.astype(np.float64), lab)
    lp3, d3 = torch.empty(B, device="cuda"), torch.empty(B, 10, device="cuda")
    ops.softmax_xent(dev(logits), 10, B, 10, dev(lab.astype(np.int64)), 0, False, False, 1 / B, lp3, d3, 10, False)
    assert abs(host(lp3).mean() - lref) < 1e-6 and rel(host(d3), dref) < 1e-6


def test_ema_adam(ops):
    g = np.random.default_rng(7)
    n = 1000 * 4 + 3
    p = g.normal(size=n).astype(np.float32)
    gr = g.normal(size=n).astype(np.float32)
    t = g.normal(size=n).astype(np.float32)
    tp, tg, tt = dev(p), dev(gr), dev(t)
    m, v = torch.zeros_like(tp), torch.zeros_like(tp)
    ops.ema(tt, tp, n, 0.996)
    assert rel(host(tt), O.ema(t.astype(np.float64), p.astype(np.float64), 0.996)) < 1e-7
    pr, mr, vr = p.astype(np.float64), np.zeros(n), np.zeros(n)
    for step in (1, 2, 3):
        ops.adam(tp, tg, m, v, n, 1e-3, 0.9, 0.999, 1e-8, 1e-2, 1 - 0.9 ** step, 1 - 0.999 ** step)
        pr, mr, vr = O.adam_step(pr, gr.astype(np.float64), mr, vr, step, 1e-3, 1e-2)
    assert rel(host(tp), pr) < 1e-7


def test_adamw(ops):
    g = np.random.default_rng(9)
    n = 257 * 4
    p = g.normal(size=n).astype(np.float32)
    gr = g.normal(size=n).astype(np.float32)
    tp, tg = dev(p), dev(gr)
    m, v = torch.zeros_like(tp), torch.zeros_like(tp)
    pr, mr, vr = p.astype(np.float64), np.zeros(n), np.zeros(n)
    for step in (1, 2, 3):
        ops.adamw(tp, tg, m, v, n, 1e-3, 0.9, 0.999, 1e-8, 1e-2, 1 - 0.9 ** step, 1 - 0.999 ** step)
        pr, mr, vr = O.adamw_step(pr, gr.astype(np.float64), mr, vr, step, 1e-3, 1e-2)
    assert rel(host(tp), pr) < 1e-7


def test_xent_offsets_global_rows(ops):
    """Shard view of a global-batch CE: rows r0..r0+R of S [R, C] with target / masked column
    at r + offset equal the corresponding rows of the full-batch loss (NT-Xent / InfoNCE with
    all-gathered negatives)."""
    g = np.random.default_rng(10)
    C, R, r0 = 24, 6, 12
    S = g.normal(size=(C, C)).astype(np.float32)
    # full NT-Xent style rows: mask diagonal, targets (i + C/2) % C
    full = S.astype(np.float64).copy()
    np.fill_diagonal(full, -np.inf)
    lab = (np.arange(C) + C // 2) % C
    lref, dref = O.cross_entropy(full, lab)
    rows = dev(S[r0:r0 + R])
    lp, d = torch.empty(R, device="cuda"), torch.empty(R, C, device="cuda")
    tgt = dev(lab[r0:r0 + R].astype(np.int64))
    ops.softmax_xent(rows, C, R, C, tgt, 0, False, True, 1.0 / C, lp, d, C, False, mask_off=r0)
    per_row = -O.log_softmax(full)[np.arange(C), lab]
    assert np.abs(host(lp) - per_row[r0:r0 + R]).max() < 1e-5
    dfull = dref.copy()
    np.fill_diagonal(dfull, 0.0)
    assert rel(host(d), dfull[r0:r0 + R]) < 1e-5
    # InfoNCE diagonal target with offset, no mask
    lp2 = torch.empty(R, device="cuda")
    ops.softmax_xent(rows, C, R, C, None, 1, False, False, 1.0, lp2, None, C, False, tgt_off=r0)
    ls = O.log_softmax(S.astype(np.float64))
    assert np.abs(host(lp2) + ls[np.arange(r0, r0 + R), np.arange(r0, r0 + R)]).max() < 1e-5


def test_stage_views(ops):
    g = np.random.default_rng(8)
    B, G, L = 3, 2, 4
    gv = g.random((B, G, 1, 28, 28)).astype(np.float32)
    lv = g.random((B, L, 1, 28, 28)).astype(np.float32)
    orig = g.random((B, 1, 28, 28)).astype(np.float32)
    out = torch.empty((G + L + 1) * B, 784, device="cuda")
    ops.stage_views(dev(gv), G, dev(lv), L, dev(orig), B, 784, out)
    ref = np.concatenate([gv.transpose(1, 0, 2, 3, 4).reshape(-1, 784), lv.transpose(1, 0, 2, 3, 4).reshape(-1, 784),
                          orig.reshape(-1, 784)])
    assert np.array_equal(host(out), ref)


@pytest.mark.parametrize("rows,cols,ld,off", [(7168, 256, 512, 256), (512, 3200, 3200, 0), (64, 320, 320, 0),
                                              (256, 51200, 51200, 0), (7, 5, 9, 3), (6144, 512, 512, 0)])
def test_sum_rows_split_matches_f64(ops, rows, cols, ld, off):
    """avd_sum_rows_split (row chunks in parallel, chunk partials summed in fixed order) against
    the float64 column sums, with and without accumulation; bitwise equal across runs."""
    from avdino._lib import lib
    g = np.random.default_rng(rows + cols)
    x = g.standard_normal(off + (rows - 1) * ld + cols).astype(np.float32)
    base = g.standard_normal(cols).astype(np.float32)
    xm = np.pad(x[off:], (0, rows * ld - (x.size - off))).reshape(rows, ld)[:, :cols]
    want = xm.astype(np.float64).sum(0)
    tx = dev(x)
    out = torch.empty(cols, device="cuda")
    ops.sum_rows(tx, rows, cols, out, ld=ld, off=off)
    assert rel(host(out), want) < 1e-6
    out2 = torch.empty(cols, device="cuda")
    ops.sum_rows(tx, rows, cols, out2, ld=ld, off=off)
    assert torch.equal(out, out2)
    acc = dev(base.copy())
    ops.sum_rows(tx, rows, cols, acc, accumulate=1, ld=ld, off=off)
    assert rel(host(acc), want + base) < 1e-6
    assert lib.avd_sum_rows_chunks(rows, cols) >= 1


@pytest.mark.parametrize("mode", [1, 2])
@pytest.mark.parametrize("rows,O_,In", [(1024, 128, 512), (1024, 512, 256), (6144, 256, 512),
                                        (2048, 256, 1600)])
def test_linear_bwd_pair_launch_equals_two_gemms(ops, monkeypatch, mode, rows, O_, In):
    """avd_linear_bwd (dW and dX tile grids in one launch, split-K where the plans split) gives
    bitwise the dW / dX of the two separate avd_gemm launches; dX lands in a column slice of a
    wider buffer as the heads' backward writes it (dcat).  Its bias gradient (row-chunk
    partials folded in the reduce launch) is within 1e-6 of float64 and of avd_sum_rows, and
    bitwise repeatable."""
    g = np.random.default_rng(rows + O_ + In + mode)
    dout = dev(g.normal(size=(rows, O_)).astype(np.float32))
    x = dev(g.normal(size=(rows, In)).astype(np.float32))
    w = dev(g.normal(size=(O_, In)).astype(np.float32))
    res = []
    for pair in (False, True):
        monkeypatch.setattr(ops, "PAIR_BWD", pair)
        dw, db = torch.empty(O_, In, device="cuda"), torch.empty(O_, device="cuda")
        dx = torch.zeros(rows, 2 * In, device="cuda")
        ops.linear_bwd(dout, x, w, dw, db, dx, rows, dx_ld=2 * In, dx_off=In, mode=mode)
        res.append((dw, db, dx))
    (a, b, c), (a2, b2, c2) = res
    assert torch.equal(a, a2) and torch.equal(c, c2)
    db64 = host(dout).astype(np.float64).sum(0)
    assert rel(host(b2), db64) < 1e-6 and rel(host(b), db64) < 1e-6
    db3 = torch.empty(O_, device="cuda")
    ops.linear_bwd(dout, x, w, torch.empty_like(dw), db3, torch.zeros_like(dx), rows, dx_ld=2 * In,
                   dx_off=In, mode=mode)
    assert torch.equal(db3, b2)
    assert c2[:, :In].abs().max().item() == 0
    ref = host(dout).astype(np.float64).T @ host(x).astype(np.float64)
    assert rel(host(a2), ref) < (1e-6 if mode == 1 else 1e-2)


@pytest.mark.parametrize("rows,cols,off,acc", [(256, 51200, 0, 0), (256, 3200, 0, 1), (7168, 256, 0, 0),
                                               (37, 1001, 0, 0), (96, 600, 3, 1), (1, 4, 0, 0)])
def test_sum_rows_vs_float64(ops, rows, cols, off, acc):
    """avd_sum_rows_split, the weight-gradient slab / bias-gradient reduction: the 16-byte path
    (cols % 4 == 0, aligned), the scalar path (odd columns, an unaligned offset), one-pass and
    row-chunked shapes, accumulate; float64 accumulation inside, so within 1 ulp of the float64
    column sums; bitwise repeatable."""
    g = torch.Generator(device="cuda").manual_seed(rows + cols)
    x = torch.randn(off + rows * cols, generator=g, device="cuda")
    base = torch.randn(cols, generator=g, device="cuda")
    ref = x[off:].view(rows, cols).double().sum(0) + (base.double() if acc else 0.0)
    outs = []
    for _ in range(2):
        out = base.clone()
        ops.sum_rows(x, rows, cols, out, accumulate=acc, off=off)
        outs.append(out)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])
    err = (outs[0].double() - ref).abs().max().item()
    assert err <= 2e-7 * max(ref.abs().max().item(), 1.0), err


@pytest.mark.parametrize("rows,O,C,HW", [(7168, 256, 64, 49), (7168, 256, 64, 25), (300, 256, 64, 49)])
def test_linear_hwc_kernels_vs_float64(ops, rows, O, C, HW):
    """The encoder Linear over NHWC bf16 features (avd_linear_*_hwc, the bf16 step's image /
    audio Linear at config-2 size and a ragged row count): the weight copy equals torch's
    permute + bf16 cast bit for bit; forward, dW (scattered back to the reference's (c, h, w)
    columns), db and dX (bf16, NHWC) against float64 of the same bf16-rounded operands -- the
    forward / dW / db differ only by fp32 accumulation order (rel-L2 1e-5), dX by its bf16
    storage (4e-3)."""
    g = torch.Generator(device="cuda").manual_seed(rows + HW)
    In = C * HW
    W = torch.randn(O, In, generator=g, device="cuda") / In ** 0.5
    b = torch.randn(O, generator=g, device="cuda")
    feat = torch.rand(rows, HW, C, generator=g, device="cuda").to(torch.bfloat16)     # NHWC
    wp = torch.empty(O * In, device="cuda", dtype=torch.bfloat16)
    ops.linear_weight_hwc([(W, wp, C, HW)])
    ref_wp = W.view(O, C, HW).permute(0, 2, 1).reshape(O, In).to(torch.bfloat16)
    torch.cuda.synchronize()
    assert torch.equal(wp.view(O, In), ref_wp)
    # the (c, h, w)-ordered features the reference's x.view(N, -1) sees
    f_chw = feat.double().permute(0, 2, 1).reshape(rows, In)
    Wd = W.to(torch.bfloat16).double()
    out = torch.zeros(rows, 2 * O, device="cuda")
    ops.linear_fwd_hwc(feat, wp, b, out, rows, O, C, HW, out_ld=2 * O, out_off=O)
    ref = f_chw @ Wd.T + b.double()
    assert out[:, :O].abs().max().item() == 0.0
    assert rel(host(out[:, O:]), ref.cpu().numpy()) < 1e-5
    dout_full = torch.randn(rows, 2 * O, generator=g, device="cuda")
    dout = dout_full[:, O:]
    dw = torch.empty(O, In, device="cuda")
    db = torch.empty(O, device="cuda")
    dx = torch.empty(rows, HW, C, device="cuda", dtype=torch.bfloat16)
    ops.linear_bwd_hwc(dout_full, feat, wp, dw, db, dx, rows, O, C, HW, dout_ld=2 * O, dout_off=O)
    dd = dout.to(torch.bfloat16).double()
    assert rel(host(dw), (dd.T @ f_chw).cpu().numpy()) < 1e-5
    assert rel(host(db), dout.double().sum(0).cpu().numpy()) < 1e-6
    dx_ref = (dd @ Wd).view(rows, C, HW).permute(0, 2, 1)
    assert rel(host(dx), dx_ref.cpu().numpy()) < 4e-3


@pytest.mark.parametrize("rows,G,C,drop,dev_seed", [(6144, 1, 512, 0.3, False), (6144, 6, 256, 0.3, True),
                                                   (1000, 2, 128, 0.0, False)])
def test_bn1d_act_bwd_reduce_equals_two_launches(ops, rows, G, C, drop, dev_seed):
    """The fused GELU/dropout backward + BatchNorm1d partials (ProjectionHead backward,
    dino.py:1240-1254) is bit-identical to avd_act_bwd + avd_bn1d_bwd_reduce."""
    g = torch.Generator(device="cuda").manual_seed(7)
    h = torch.randn(rows, C, device="cuda", generator=g)
    da = torch.randn(rows, C, device="cuda", generator=g)
    mean = torch.randn(G * C, device="cuda", generator=g) * 0.1
    invstd = torch.rand(G * C, device="cuda", generator=g) + 0.5
    scale = torch.rand(G * C, device="cuda", generator=g) + 0.5
    shift = torch.randn(G * C, device="cuda", generator=g) * 0.2
    seed_off = torch.tensor([12345], dtype=torch.int64, device="cuda") if dev_seed else None
    R = ops.colstats_parts(rows // G)
    dz1, dz2 = torch.empty_like(h), torch.empty_like(h)
    p1 = torch.empty(C * G * R * 2, device="cuda")
    p2 = torch.empty_like(p1)
    ops.act_bwd(h, da, dz1, 1, scale, shift, rows, G, C, drop, 99, seed_off)
    ops.bn1d_bwd_reduce(h, dz1, mean, invstd, rows, G, C, p1)
    ops.bn1d_act_bwd_reduce(h, da, dz2, scale, shift, mean, invstd, rows, G, C, drop, 99, p2, seed_off)
    torch.cuda.synchronize()
    assert torch.equal(dz1, dz2)
    assert torch.equal(p1, p2)
