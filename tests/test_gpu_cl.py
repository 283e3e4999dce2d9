"""Per-kernel parity of the channels-last (NHWC) conv-block path (include/avdino.h avd_cl_*)
against the float64 numpy oracle, in both storage types:
  f32  (v_mfma_f32_16x16x4f32, exact f32 products): rel-L2 <= 2e-6 on maps, 1e-5 on reductions
  bf16 (v_mfma_f32_16x16x32_bf16 on bf16-rounded operands, fp32 accumulate, bf16 stores):
       rel-L2 <= 5e-3 on stored maps (one bf16 rounding), 1e-5 on f32 reductions of them.
Shapes cover every conv of the CentralNet image/audio encoders and the 3x3 CNNs, ragged
tilings, whole-map packing of small maps (NS > 1), and two BN groups."""
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


def bf(a):
    return torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(torch.bfloat16).float().numpy()


def nhwc(a):
    return np.ascontiguousarray(np.asarray(a).transpose(0, 2, 3, 1))


def nchw(a):
    return np.ascontiguousarray(np.asarray(a).transpose(0, 3, 1, 2))


@pytest.fixture(scope="module")
def ops():
    from avdino import ops as _ops
    return _ops


DT = {"f32": torch.float32, "bf16": torch.bfloat16}
TOL = {"f32": 2e-6, "bf16": 5e-3}

CASES = [  # N, Cin, H, Cout, K, pad
    (3, 1, 28, 32, 5, 2), (2, 1, 112, 8, 5, 2), (2, 8, 56, 16, 5, 2), (2, 16, 28, 32, 5, 2),
    (4, 32, 14, 64, 5, 2), (8, 32, 14, 64, 5, 0), (2, 1, 28, 32, 3, 1), (4, 32, 14, 64, 3, 1),
    (8, 64, 7, 128, 3, 1), (2, 128, 14, 256, 3, 1), (2, 8, 20, 8, 5, 2), (4, 1, 48, 8, 5, 2),
    (6, 1, 112, 8, 5, 2),
]


def _inputs(case, dt, seed):
    N, Cin, H, Cout, K, pad = case
    g = np.random.default_rng(seed)
    x = g.uniform(-1, 1, (N, Cin, H, H))
    w = g.uniform(-1, 1, (Cout, Cin, K, K)) / np.sqrt(Cin * K * K)
    b = g.uniform(-0.1, 0.1, Cout).astype(np.float32)
    if dt == "bf16":
        x, w = bf(x), bf(w)
    return x.astype(np.float32), w.astype(np.float32), b


@pytest.mark.parametrize("dt", ["f32", "bf16"])
@pytest.mark.parametrize("case", CASES)
def test_cl_conv_fwd_stats(ops, case, dt):
    N, Cin, H, Cout, K, pad = case
    B = N // 2 if N % 2 == 0 else N
    G = N // B
    x, w, b = _inputs(case, dt, hash(case) % 2**32)
    y_ref, _ = O.conv2d_fwd(x.astype(np.float64), w.astype(np.float64), b.astype(np.float64), pad)
    Ho = y_ref.shape[2]
    T = DT[dt]
    wk = torch.empty(ops.cl_weight_elems(Cout, Cin, K, 0), device="cuda", dtype=T)
    ops.cl_weight_layout(dev(w), wk, 0)
    y = torch.empty(N, Ho, Ho, Cout, device="cuda", dtype=T)
    R = ops.cl_stat_rows(Ho, Ho, B, K, Cin, Cout, T)
    stats = torch.full((Cout * G * R * 2,), float("nan"), device="cuda")
    ops.cl_conv_fwd(dev(nhwc(x), T), wk, dev(b), y, stats, N, B, Cin, H, H, Cout, K, pad)
    yh = nchw(host(y))
    assert rel(yh, y_ref) < TOL[dt], rel(yh, y_ref)
    st = host(stats).reshape(Cout, G, R, 2).sum(2)               # per (channel, group)
    ys = yh.reshape(G, B, Cout, Ho, Ho)                          # statistics of the stored values
    assert rel(st[..., 0], ys.sum((1, 3, 4)).T) < 1e-5
    assert rel(st[..., 1], (ys ** 2).sum((1, 3, 4)).T) < 1e-5


@pytest.mark.parametrize("dt", ["f32", "bf16"])
@pytest.mark.parametrize("case", [c for c in CASES if c[1] > 1])
def test_cl_conv_dgrad(ops, case, dt):
    N, Cin, H, Cout, K, pad = case
    x, w, _ = _inputs(case, dt, hash(case) % 2**32 + 1)
    y_ref, win = O.conv2d_fwd(x.astype(np.float64), w.astype(np.float64), np.zeros(Cout), pad)
    g = np.random.default_rng(5)
    dy = g.uniform(-1, 1, y_ref.shape).astype(np.float32)
    if dt == "bf16":
        dy = bf(dy)
    dx_ref, _, _ = O.conv2d_bwd(dy.astype(np.float64), win, w.astype(np.float64), x.shape, pad)
    T = DT[dt]
    wd = torch.empty(ops.cl_weight_elems(Cout, Cin, K, 1), device="cuda", dtype=T)
    ops.cl_weight_layout(dev(w), wd, 1)
    dx = torch.empty(N, H, H, Cin, device="cuda", dtype=T)
    ops.cl_conv_dgrad(dev(nhwc(dy), T), wd, dx, N, Cin, H, H, Cout, K, pad)
    assert rel(nchw(host(dx)), dx_ref) < TOL[dt]


@pytest.mark.parametrize("dt", ["f32", "bf16"])
@pytest.mark.parametrize("case", CASES + [(5, 8, 112, 16, 5, 2), (3, 32, 10, 64, 5, 0)])
def test_cl_conv_wgrad(ops, case, dt):
    N, Cin, H, Cout, K, pad = case
    x, _, _ = _inputs(case, dt, hash(case) % 2**32 + 2)
    Ho = H + 2 * pad - K + 1
    g = np.random.default_rng(6)
    dy = g.uniform(-1, 1, (N, Cout, Ho, Ho)).astype(np.float32)
    if dt == "bf16":
        dy = bf(dy)
    wz = np.zeros((Cout, Cin, K, K))
    _, win = O.conv2d_fwd(x.astype(np.float64), wz, np.zeros(Cout), pad)
    _, dw_ref, _ = O.conv2d_bwd(dy.astype(np.float64), win, wz, x.shape, pad)
    T = DT[dt]
    nch = ops.cl_wgrad_chunks(N, Cout, Cin, K)
    parts = torch.full((nch * Cout * Cin * K * K,), float("nan"), device="cuda")
    ops.cl_conv_wgrad(dev(nhwc(x), T), dev(nhwc(dy), T), parts, N, Cin, H, H, Cout, K, pad)
    dw = torch.empty(Cout, Cin, K, K, device="cuda")
    ops.sum_rows(parts, nch, Cout * Cin * K * K, dw)
    # operands are exact in both types; only the fp32 accumulation order differs
    assert rel(host(dw), dw_ref) < 1e-5


POOL_CASES = [(112, 8), (56, 16), (28, 32), (14, 64), (10, 64), (7, 128), (28, 8)]


@pytest.mark.parametrize("dt", ["f32", "bf16"])
@pytest.mark.parametrize("mode", [0, 1, 2])
@pytest.mark.parametrize("HC", POOL_CASES)
def test_cl_bn_block_fwd_bwd(ops, HC, mode, dt):
    """BN(train, per group) -> ReLU -> maxpool2 [-> GAP | -> (c,h,w) flatten] forward and the
    full backward (reduce -> avd_bn_bwd_finalize -> apply), NHWC, incl. odd maps (7x7)."""
    H, C = HC
    G, B = 2, 3
    N = G * B
    T = DT[dt]
    g = np.random.default_rng(H * 1000 + C + 7 * mode)
    y = g.normal(0.3, 1.5, (N, C, H, H))
    if dt == "bf16":
        y = bf(y)
    y = y.astype(np.float32)
    gamma = (1 + g.uniform(-0.2, 0.2, C)).astype(np.float32)
    beta = g.uniform(-0.2, 0.2, C).astype(np.float32)
    z, bnc, stats = O.bn_train_fwd(y.astype(np.float64), gamma.astype(np.float64),
                                   beta.astype(np.float64), G, (2, 3))
    r = np.maximum(z, 0)
    pmap, pc = O.maxpool2_fwd(r)
    Hp = H // 2
    out_ref = {0: pmap, 1: pmap.mean((2, 3)), 2: pmap.reshape(N, -1)}[mode]
    gout = g.uniform(-1, 1, out_ref.shape).astype(np.float32)
    if mode == 0 and dt == "bf16":
        gout = bf(gout)
    if mode == 0:
        dp = gout.astype(np.float64)
    elif mode == 1:
        dp = np.broadcast_to(gout[:, :, None, None] / (Hp * Hp), pmap.shape)
    else:
        dp = gout.reshape(pmap.shape).astype(np.float64)
    dz = O.maxpool2_bwd(dp, pc) * (z > 0)
    dy_ref, dg_ref, db_ref = O.bn_train_bwd(dz, bnc)

    # stats from the oracle's partials (conv epilogue tested above), finalize on device
    parts = np.stack([y.astype(np.float64).reshape(G, B, C, -1).transpose(2, 0, 1, 3).sum(-1),
                      (y.astype(np.float64) ** 2).reshape(G, B, C, -1).transpose(2, 0, 1, 3).sum(-1)], -1)
    st = torch.empty(4, G * C, device="cuda")
    ops.bn_finalize(dev(parts.astype(np.float32)), G, B, C, B * H * H, dev(gamma), dev(beta),
                    st[0], st[1], st[2], st[3])
    ty = dev(nhwc(y), T)
    if mode == 0:
        out = torch.empty(N, Hp, Hp, C, device="cuda", dtype=T)
    else:
        out = torch.empty(out_ref.shape, device="cuda")
    ops.cl_bn_relu_pool(ty, st[2], st[3], out, mode, N, B, C, H, H)
    oh = nchw(host(out)) if mode == 0 else host(out)
    assert rel(oh, out_ref) < (4e-3 if (dt == "bf16" and mode == 0) else 1e-5)

    tg = dev(nhwc(gout), T) if mode == 0 else dev(gout)
    R = ops.cl_bn_bwd_rows(B, C, H, H, T)
    bparts = torch.full((C * G * R * 2,), float("nan"), device="cuda")
    ops.cl_bn_bwd_reduce(ty, tg, mode, st[2], st[3], st[0], st[1], bparts, N, B, C, H, H)
    coef = torch.empty(G * C * 3, device="cuda")
    dgam, dbet = torch.empty(C, device="cuda"), torch.empty(C, device="cuda")
    ops.bn_bwd_finalize(bparts, G, R, C, B * H * H, dev(gamma), st[0], st[1], coef, dgam, dbet, None)
    assert rel(host(dgam), dg_ref) < 1e-5
    assert rel(host(dbet), db_ref) < 1e-5
    dy = torch.empty_like(ty)
    ops.cl_bn_bwd_apply(ty, tg, mode, st[2], st[3], coef, dy, N, B, C, H, H)
    assert rel(nchw(host(dy)), dy_ref) < (5e-3 if dt == "bf16" else 1e-5)


@pytest.mark.parametrize("HN", [(112, 4, 8, 5, 2), (48, 6, 8, 5, 2), (112, 4, 32, 3, 1),
                                (28, 24, 32, 3, 1), (56, 6, 16, 3, 1)])
def test_cl_bn_bwd_apply_wgrad_fused_first_layer(ops, HN):
    """Fused BN-backward apply + weight gradient of a first layer -- the CentralNet audio conv1
    (1->8 5x5 p2, c1p8) and the 3x3 encoders' conv1 (1->16/32 3x3 p1, c1w3), bf16 ==
    avd_cl_bn_bwd_apply followed by avd_cl_conv_wgrad: dy is rounded to bf16 the same way in
    both, so only the fp32 accumulation order differs (rel 1e-5); and the float64 truth from
    the same bf16 operands within 1e-5."""
    H, N, C, K, pad = HN
    B = N // 2
    G = N // B
    g = np.random.default_rng(H)
    T = torch.bfloat16
    x = bf(g.uniform(0, 1, (N, H, H, 1)))
    y = bf(g.normal(0.2, 1.0, (N, H, H, C)))
    gout = bf(g.uniform(-1, 1, (N, H // 2, H // 2, C)))
    scale = g.uniform(0.5, 1.5, G * C).astype(np.float32)
    shift = g.uniform(-0.3, 0.3, G * C).astype(np.float32)
    coef = g.uniform(-0.5, 0.5, G * C * 3).astype(np.float32)
    ty, tg, tx = dev(y, T), dev(gout, T), dev(x, T)
    dy = torch.empty_like(ty)
    ops.cl_bn_bwd_apply(ty, tg, 0, dev(scale), dev(shift), dev(coef), dy, N, B, C, H, H)
    nch = ops.cl_wgrad_chunks(N, C, 1, K)
    parts = torch.empty(nch * C * K * K, device="cuda")
    ops.cl_conv_wgrad(tx, dy, parts, N, 1, H, H, C, K, pad)
    dw_ref = torch.empty(C, 1, K, K, device="cuda")
    ops.sum_rows(parts, nch, C * K * K, dw_ref)
    ns = ops.cl_apply_wgrad_slabs(T, N, 1, H, H, C, K, pad)
    assert ns > 0
    fparts = torch.full((ns * C * K * K,), float("nan"), device="cuda")
    ops.cl_bn_bwd_apply_wgrad(ty, tg, dev(scale), dev(shift), dev(coef), tx, fparts, N, B, 1, H, H,
                              C, K, pad)
    dw = torch.empty(C, 1, K, K, device="cuda")
    ops.sum_rows(fparts, ns, C * K * K, dw)
    assert rel(host(dw), host(dw_ref)) < 1e-5, rel(host(dw), host(dw_ref))
    # float64 truth on the same bf16 dy
    win = np.lib.stride_tricks.sliding_window_view(np.pad(nchw(x).astype(np.float64),
                                                          ((0, 0), (0, 0), (pad, pad), (pad, pad))), (K, K), (2, 3))
    dw64 = np.einsum("nohw,nchwij->ocij", nchw(host(dy)), win, optimize=True)
    assert rel(host(dw), dw64) < 1e-5


@pytest.mark.parametrize("HN", [(112, 4, 8, 5, 2), (48, 6, 8, 5, 2),
                                # the 3x3 encoders' first layer (c1r3_kernel, c1w3.hip)
                                (112, 4, 32, 3, 1), (112, 6, 16, 3, 1), (56, 4, 64, 3, 1),
                                (48, 6, 32, 3, 1), (8, 4, 16, 3, 1),
                                # widths 4 mod 8 (virtual columns) and the 5x5 CentralNet image
                                # conv1 (1->32 at 28^2, unimodal.py:127-141)
                                (28, 6, 32, 3, 1), (28, 8, 32, 3, 1), (28, 6, 32, 5, 2), (20, 6, 32, 5, 2),
                                (48, 4, 32, 5, 2)])
def test_cl_c1_recompute_passes_match_stored_y_path(ops, HN, avd_opts):
    """avd_cl_c1_recompute (the audio conv1 without a stored conv output) against the stored-y
    kernels on the same bf16 operands: identical pooled output (bit-exact: same rounded y), and
    the statistics / BN-backward partials / weight gradient to fp32 summation order."""
    H, N, C, K, pad = HN
    B, Cin = N // 2, 1
    G = N // B
    T = torch.bfloat16
    g = np.random.default_rng(H + C + K)
    x = bf(g.uniform(0, 1, (N, H, H, 1)))
    w = bf(g.uniform(-1, 1, (C, 1, K, K)) / K)
    b = g.uniform(-0.1, 0.1, C).astype(np.float32)
    tx, tb = dev(x, T), dev(b)
    wk = torch.empty(ops.cl_weight_elems(C, 1, K, 0), device="cuda", dtype=T)
    ops.cl_weight_layout(dev(w), wk, 0)
    # stored-y path
    y = torch.empty(N, H, H, C, device="cuda", dtype=T)
    R0 = ops.cl_stat_rows(H, H, B, K, 1, C, T)
    st0 = torch.empty(C * G * R0 * 2, device="cuda")
    ops.cl_conv_fwd(tx, wk, tb, y, st0, N, B, 1, H, H, C, K, pad)
    R1 = ops.cl_c1_recompute_rows(ops.C1_STATS, T, N, B, 1, H, H, C, K, pad)
    assert R1 > 0
    st1 = torch.empty(C * G * R1 * 2, device="cuda")
    ops.cl_c1_recompute(ops.C1_STATS, tx, wk, tb, N, B, 1, H, H, C, K, pad, out=st1)
    s0 = host(st0).reshape(C, G, R0, 2).sum(2)
    s1 = host(st1).reshape(C, G, R1, 2).sum(2)
    if K == 3 and C == 32 and H in (28, 112):
        # the 3x3 1 -> 32 statistics pass (c1s3.hip) sums the EXACT conv output from the block's
        # patch Gram (as the audio conv1's, avd_cl_c1_gram): float64 of the exact conv
        y64 = torch.nn.functional.conv2d(torch.from_numpy(x).double().permute(0, 3, 1, 2),
                                         torch.from_numpy(w).double(), torch.from_numpy(b).double(),
                                         padding=pad).view(G, B, C, H * H)
        ref = torch.stack([y64.sum((1, 3)), (y64 ** 2).sum((1, 3))], -1).transpose(0, 1).numpy()
        assert rel(s1, ref) < 1e-6, rel(s1, ref)
        assert rel(s1, s0) < 1e-4              # the stored-y sums are of the bf16-rounded y
    else:
        assert rel(s1, s0) < 1e-6
    gamma = (1 + g.uniform(-.2, .2, C)).astype(np.float32)
    beta = g.uniform(-.2, .2, C).astype(np.float32)
    bn = torch.empty(4, G * C, device="cuda")
    ops.bn_finalize(st0, G, R0, C, B * H * H, dev(gamma), dev(beta), bn[0], bn[1], bn[2], bn[3])
    z0 = torch.empty(N, H // 2, H // 2, C, device="cuda", dtype=T)
    ops.cl_bn_relu_pool(y, bn[2], bn[3], z0, 0, N, B, C, H, H)
    z1 = torch.empty_like(z0)
    ops.cl_c1_recompute(ops.C1_APPLY, tx, wk, tb, N, B, 1, H, H, C, K, pad, scale=bn[2],
                        shift=bn[3], z=z1)
    assert torch.equal(z0, z1)
    gz = dev(bf(g.uniform(-1, 1, (N, H // 2, H // 2, C))), T)
    Rb = ops.cl_bn_bwd_rows(B, C, H, H, T)
    p0 = torch.empty(C * G * Rb * 2, device="cuda")
    ops.cl_bn_bwd_reduce(y, gz, 0, bn[2], bn[3], bn[0], bn[1], p0, N, B, C, H, H)
    Rr = ops.cl_c1_recompute_rows(ops.C1_REDUCE, T, N, B, 1, H, H, C, K, pad)
    p1 = torch.empty(C * G * Rr * 2, device="cuda")
    ops.cl_c1_recompute(ops.C1_REDUCE, tx, wk, tb, N, B, 1, H, H, C, K, pad, scale=bn[2],
                        shift=bn[3], mean=bn[0], invstd=bn[1], gz=gz, out=p1)
    r0 = host(p0).reshape(C, G, Rb, 2).sum(2)
    r1 = host(p1).reshape(C, G, Rr, 2).sum(2)
    assert rel(r1, r0) < 1e-5, rel(r1, r0)
    coef = torch.empty(G * C * 3, device="cuda")
    dg, dbt = torch.empty(C, device="cuda"), torch.empty(C, device="cuda")
    ops.bn_bwd_finalize(p0, G, Rb, C, B * H * H, dev(gamma), bn[0], bn[1], coef, dg, dbt, None)
    ns = ops.cl_apply_wgrad_slabs(T, N, 1, H, H, C, K, pad)
    if ns:   # the stored-y fused apply + wgrad (c1p8 / c1w3)
        f0 = torch.empty(ns * C * K * K, device="cuda")
        ops.cl_bn_bwd_apply_wgrad(y, gz, bn[2], bn[3], coef, tx, f0, N, B, 1, H, H, C, K, pad)
    else:    # (5x5 Cout 32: no fused stored-y kernel) the unfused apply, then the weight gradient
        dyk = torch.empty_like(y)
        ops.cl_bn_bwd_apply(y, gz, 0, bn[2], bn[3], coef, dyk, N, B, C, H, H)
        ns = ops.cl_wgrad_chunks(N, C, 1, K)
        f0 = torch.empty(ns * C * K * K, device="cuda")
        ops.cl_conv_wgrad(tx, dyk, f0, N, 1, H, H, C, K, pad)
    nw = ops.cl_c1_recompute_rows(ops.C1_WGRAD, T, N, B, 1, H, H, C, K, pad)
    f1 = torch.empty(nw * C * K * K, device="cuda")
    ops.cl_c1_recompute(ops.C1_WGRAD, tx, wk, tb, N, B, 1, H, H, C, K, pad, scale=bn[2],
                        shift=bn[3], coef=coef, gz=gz, out=f1)
    d0, d1 = torch.empty(C * K * K, device="cuda"), torch.empty(C * K * K, device="cuda")
    ops.sum_rows(f0, ns, C * K * K, d0)
    ops.sum_rows(f1, nw, C * K * K, d1)
    assert rel(host(d1), host(d0)) < 1e-6
    R4 = ops.cl_c1_recompute_rows(ops.C1_REDUCE_MOMENTS, T, N, B, 1, H, H, C, K, pad)
    assert R4 > 0
    # pass 4: the reduce rows of pass 2 plus the moments; dW = combine(moments, coef)
    # (3x3: [C*9 | Gram rows 9 x 10 with the ones tap]; 5x5 audio conv1: [C*25 | 25 x 25 | 25])
    KK = K * K
    mc = ops.c1_moment_cols(C, K)
    m4 = torch.full((C * G * R4 * 2 + R4 * G * mc,), float("nan"), device="cuda")
    ops.cl_c1_recompute(ops.C1_REDUCE_MOMENTS, tx, wk, tb, N, B, 1, H, H, C, K, pad, scale=bn[2],
                        shift=bn[3], mean=bn[0], invstd=bn[1], gz=gz, out=m4)
    r4 = host(m4[:C * G * R4 * 2]).reshape(C, G, R4, 2).sum(2)
    assert rel(r4, r0) < 1e-5, rel(r4, r0)
    mom = torch.empty(G * mc, device="cuda")
    ops.sum_rows(m4, R4, G * mc, mom, off=C * G * R4 * 2)
    mh = host(mom).reshape(G, mc)
    # the Gram block against float64 (exact products, f32 sums): sum xk_t xk_t' and sum xk_t
    win = np.lib.stride_tricks.sliding_window_view(
        np.pad(nchw(x).astype(np.float64), ((0, 0), (0, 0), (pad, pad), (pad, pad))), (K, K), (2, 3))
    xk = win.reshape(G, B, H, H, KK)
    gram = np.einsum("gbhwi,gbhwj->gij", xk, xk)
    if C != 8:   # c1r3 layout: Gram rows with the ones tap [KK][KK + 1]
        gk = mh[:, C * KK:].reshape(G, KK, KK + 1)[:, :, :KK]
        sk = mh[:, C * KK:].reshape(G, KK, KK + 1)[:, :, KK]
    else:
        gk, sk = mh[:, C * KK:C * KK + KK * KK].reshape(G, KK, KK), mh[:, C * KK + KK * KK:]
    assert rel(gk, gram) < 1e-5, rel(gk, gram)
    assert rel(sk, xk.sum((1, 2, 3))) < 1e-5
    dk = torch.empty(C * KK, device="cuda")
    ops.cl_c1_recompute_combine(mom, coef, wk, tb, dk, G, C, K)
    # dW from the unrounded dy = k1 dz + kx y + k0 (y = w . xk + b unrounded in the kx term):
    # against float64 of exactly that, and within the bf16 rounding of dy of the stored-y path
    # (dy is centred, so its rounding shows in dW amplified by the cancellation: ~0.5 %)
    yb = host(y).astype(np.float64).reshape(G, B, H, H, C)
    zr = np.maximum(yb * host(bn[2]).reshape(G, 1, 1, 1, C) + host(bn[3]).reshape(G, 1, 1, 1, C), 0)
    zw = zr.reshape(G, B, H // 2, 2, H // 2, 2, C).transpose(0, 1, 2, 4, 6, 3, 5).reshape(
        G, B, H // 2, H // 2, C, 4)
    am, best = zw.argmax(-1), zw.max(-1)
    gzh = host(gz).astype(np.float64).reshape(G, B, H // 2, H // 2, C)
    dzw = np.where((np.arange(4) == am[..., None]) & (best[..., None] > 0), gzh[..., None], 0.0)
    dz = dzw.reshape(G, B, H // 2, H // 2, C, 2, 2).transpose(0, 1, 2, 5, 3, 6, 4).reshape(G, B, H, H, C)
    assert rel(mh[:, :C * KK].reshape(G, C, KK), np.einsum("gbhwc,gbhwt->gct", dz, xk)) < 1e-5
    yex = np.einsum("gbhwt,ct->gbhwc", xk, w.reshape(C, KK).astype(np.float64)) + b.astype(np.float64)
    k3 = host(coef).astype(np.float64).reshape(G, 1, 1, 1, C, 3)
    dy64 = k3[..., 0] * dz + k3[..., 1] * yex + k3[..., 2]
    dw64 = np.einsum("gbhwc,gbhwt->ct", dy64, xk)
    e64 = rel(host(dk), dw64.reshape(-1))
    err = rel(host(dk), host(d0))
    print("pass-4 dW rel: vs float64", e64, "vs stored-y path", err)
    assert e64 < 1e-4, e64
    assert err < 1e-2, err


# The bench's mid-layer convs are served by the weights-stationary kernel (conv_ws.hip) in bf16;
# avd_options.generic_conv = 1 routes them to conv_cl_kernel.  The 56x56 and 28x28 layers keep the
# legacy K order and accumulation order: bit-identical maps.  The 14x14 layers split K over two
# waves (summed in fixed order), so there the two differ by bf16 rounding only; both paths are
# also checked against float64.
WS_SHAPES = [  # N, B, Cin, H, Cout, K, pad
    (48, 24, 8, 56, 16, 5, 2), (48, 24, 16, 28, 32, 5, 2), (48, 24, 32, 14, 64, 5, 2),
    (48, 24, 32, 14, 64, 5, 0)]


def _both_paths(avd_opts, fn):
    avd_opts(generic_conv=0)
    a = fn()
    avd_opts(generic_conv=1)
    b = fn()
    avd_opts(generic_conv=0)
    return a, b


@pytest.mark.parametrize("shape", WS_SHAPES)
def test_ws_conv_fwd_matches_legacy(ops, shape, avd_opts):
    N, B, Cin, H, Cout, K, pad = shape
    G = N // B
    x, w, b = _inputs((N, Cin, H, Cout, K, pad), "bf16", 11)
    Ho = H + 2 * pad - K + 1
    T = torch.bfloat16
    wk = torch.empty(ops.cl_weight_elems(Cout, Cin, K, 0), device="cuda", dtype=T)
    ops.cl_weight_layout(dev(w), wk, 0)
    xd, bd = dev(nhwc(x), T), dev(b)

    def run():
        y = torch.empty(N, Ho, Ho, Cout, device="cuda", dtype=T)
        R = ops.cl_stat_rows(Ho, Ho, B, K, Cin, Cout, T)
        st = torch.full((Cout * G * R * 2,), float("nan"), device="cuda")
        ops.cl_conv_fwd(xd, wk, bd, y, st, N, B, Cin, H, H, Cout, K, pad)
        torch.cuda.synchronize()
        return host(y), host(st).reshape(Cout, G, R, 2).sum(2)

    (y1, s1), (y0, s0) = _both_paths(avd_opts, run)
    if H > 14:
        assert np.array_equal(y1, y0)
        assert rel(s1, s0) < 1e-6
    else:   # statistics of two differently rounded maps
        assert rel(y1, y0) < 4e-3
        assert rel(s1, s0) < 1e-3
    y_ref, _ = O.conv2d_fwd(x.astype(np.float64), w.astype(np.float64), b.astype(np.float64), pad)
    assert rel(nchw(y1), y_ref) < TOL["bf16"]


@pytest.mark.parametrize("shape", WS_SHAPES)
def test_ws_conv_dgrad_matches_legacy(ops, shape, avd_opts):
    N, _, Cin, H, Cout, K, pad = shape
    x, w, _ = _inputs((N, Cin, H, Cout, K, pad), "bf16", 12)
    y_ref, win = O.conv2d_fwd(x.astype(np.float64), w.astype(np.float64), np.zeros(Cout), pad)
    dy = bf(np.random.default_rng(13).uniform(-1, 1, y_ref.shape))
    T = torch.bfloat16
    wd = torch.empty(ops.cl_weight_elems(Cout, Cin, K, 1), device="cuda", dtype=T)
    ops.cl_weight_layout(dev(w), wd, 1)
    dyd = dev(nhwc(dy), T)

    def run():
        dx = torch.empty(N, H, H, Cin, device="cuda", dtype=T)
        ops.cl_conv_dgrad(dyd, wd, dx, N, Cin, H, H, Cout, K, pad)
        torch.cuda.synchronize()
        return host(dx)

    d1, d0 = _both_paths(avd_opts, run)
    if H > 14:
        assert np.array_equal(d1, d0)
    else:
        assert rel(d1, d0) < 4e-3
    dx_ref, _, _ = O.conv2d_bwd(dy.astype(np.float64), win, w.astype(np.float64), x.shape, pad)
    assert rel(nchw(d1), dx_ref) < TOL["bf16"]


@pytest.mark.parametrize("shape", WS_SHAPES)
def test_ws_conv_wgrad_matches_legacy(ops, shape, avd_opts):
    """wgrad_ws.hip (one block = all weight columns of its sample chunk) vs the legacy kernel
    and float64: exact bf16 products, fp32 sums in another order."""
    N, _, Cin, H, Cout, K, pad = shape
    x, _, _ = _inputs((N, Cin, H, Cout, K, pad), "bf16", 14)
    Ho = H + 2 * pad - K + 1
    dy = bf(np.random.default_rng(15).uniform(-1, 1, (N, Cout, Ho, Ho)))
    T = torch.bfloat16
    xd, dyd = dev(nhwc(x), T), dev(nhwc(dy), T)

    def run():
        nch = ops.cl_wgrad_chunks(N, Cout, Cin, K)
        parts = torch.full((nch * Cout * Cin * K * K,), float("nan"), device="cuda")
        ops.cl_conv_wgrad(xd, dyd, parts, N, Cin, H, H, Cout, K, pad)
        dw = torch.empty(Cout, Cin, K, K, device="cuda")
        ops.sum_rows(parts, nch, Cout * Cin * K * K, dw)
        torch.cuda.synchronize()
        return host(dw)

    w1, w0 = _both_paths(avd_opts, run)
    wz = np.zeros((Cout, Cin, K, K))
    _, win = O.conv2d_fwd(x.astype(np.float64), wz, np.zeros(Cout), pad)
    _, dw_ref, _ = O.conv2d_bwd(dy.astype(np.float64), win, wz, x.shape, pad)
    assert rel(w1, dw_ref) < 1e-5
    assert rel(w0, dw_ref) < 1e-5


@pytest.mark.parametrize("dt", ["f32", "bf16"])
@pytest.mark.parametrize("HC", [(112, 8), (56, 16), (28, 32), (14, 64), (10, 64)])
@pytest.mark.parametrize("mode", [0, 2])
def test_bn_bwd_reduce_pooled_matches_y_path(ops, HC, mode, dt):
    """avd_cl_bn_bwd_reduce_pooled (xhat from the pooled output) vs avd_cl_bn_bwd_reduce (xhat
    from y at the argmax): same sums up to the rounding of the stored pooled value, incl. a
    gamma == 0 channel (whose xhat the pooled kernel takes from y)."""
    H, C = HC
    N, B = 6, 3
    G = N // B
    T = DT[dt]
    g = torch.Generator(device="cuda").manual_seed(31)
    y = torch.randn(N, H, H, C, generator=g, device="cuda").to(T)
    gamma = torch.rand(C, generator=g, device="cuda") + 0.5
    gamma[1] = 0.0
    beta = torch.randn(C, generator=g, device="cuda") * 0.1
    yf = y.float().view(G, B * H * H, C)
    mean = yf.mean(1).reshape(-1).contiguous()
    invstd = (yf.var(1, unbiased=False) + 1e-5).rsqrt().reshape(-1).contiguous()
    scale = (gamma.view(1, C) * invstd.view(G, C)).reshape(-1).contiguous()
    shift = (beta.view(1, C) - mean.view(G, C) * scale.view(G, C)).reshape(-1).contiguous()
    Hp = H // 2
    if mode == 0:
        pooled = torch.empty(N, Hp, Hp, C, device="cuda", dtype=T)
        gout = torch.randn(N, Hp, Hp, C, generator=g, device="cuda").to(T)
    else:
        pooled = torch.empty(N * C * Hp * Hp, device="cuda")
        gout = torch.randn(N * C * Hp * Hp, generator=g, device="cuda")
    ops.cl_bn_relu_pool(y, scale, shift, pooled, mode, N, B, C, H, H)
    R = ops.cl_bn_bwd_rows(B, C, H, H, T)
    p0 = torch.zeros(C * G * R * 2, device="cuda")
    p1 = torch.zeros(C * G * R * 2, device="cuda")
    ops.cl_bn_bwd_reduce(y, gout, mode, scale, shift, mean, invstd, p0, N, B, C, H, H)
    ops.cl_bn_bwd_reduce_pooled(y, pooled, gout, mode, gamma, beta, mean, invstd, p1, N, B, C, H, H)
    s0 = host(p0).reshape(C, G, R, 2).sum(2)
    s1 = host(p1).reshape(C, G, R, 2).sum(2)
    assert np.allclose(s1[..., 0], s0[..., 0], rtol=1e-5, atol=1e-4)     # sum dz: identical routing
    tol = 2e-6 if dt == "f32" else 4e-3                                  # bf16: rounding of p
    assert rel(s1[..., 1], s0[..., 1]) < tol


@pytest.mark.parametrize("dt", ["f32", "bf16"])
@pytest.mark.parametrize("mode", [0, 2])
def test_bn_bwd_reduce_pooled_small_gamma(ops, mode, dt):
    """channels whose |beta / gamma| would amplify the stored pooled value's rounding
    (gamma 1e-2, beta 1 here) take xhat from y; the sums then match the y-path kernel."""
    H, C, N, B = 28, 32, 6, 3
    G = N // B
    T = DT[dt]
    g = torch.Generator(device="cuda").manual_seed(37)
    y = torch.randn(N, H, H, C, generator=g, device="cuda").to(T)
    gamma = torch.rand(C, generator=g, device="cuda") + 0.5
    beta = torch.randn(C, generator=g, device="cuda") * 0.1
    gamma[:8] = 1e-2
    beta[:8] = 1.0
    gamma[8] = -2e-3
    beta[8] = -0.5
    yf = y.float().view(G, B * H * H, C)
    mean = yf.mean(1).reshape(-1).contiguous()
    invstd = (yf.var(1, unbiased=False) + 1e-5).rsqrt().reshape(-1).contiguous()
    scale = (gamma.view(1, C) * invstd.view(G, C)).reshape(-1).contiguous()
    shift = (beta.view(1, C) - mean.view(G, C) * scale.view(G, C)).reshape(-1).contiguous()
    Hp = H // 2
    if mode == 0:
        pooled = torch.empty(N, Hp, Hp, C, device="cuda", dtype=T)
        gout = torch.randn(N, Hp, Hp, C, generator=g, device="cuda").to(T)
    else:
        pooled = torch.empty(N * C * Hp * Hp, device="cuda")
        gout = torch.randn(N * C * Hp * Hp, generator=g, device="cuda")
    ops.cl_bn_relu_pool(y, scale, shift, pooled, mode, N, B, C, H, H)
    R = ops.cl_bn_bwd_rows(B, C, H, H, T)
    p0 = torch.zeros(C * G * R * 2, device="cuda")
    p1 = torch.zeros(C * G * R * 2, device="cuda")
    ops.cl_bn_bwd_reduce(y, gout, mode, scale, shift, mean, invstd, p0, N, B, C, H, H)
    ops.cl_bn_bwd_reduce_pooled(y, pooled, gout, mode, gamma, beta, mean, invstd, p1, N, B, C, H, H)
    s0 = host(p0).reshape(C, G, R, 2).sum(2)
    s1 = host(p1).reshape(C, G, R, 2).sum(2)
    for c in range(9):       # the small-gamma channels: xhat from y, as the y-path kernel
        assert rel(s1[c, :, 1], s0[c, :, 1]) < 5e-5, c
    assert rel(s1[9:, :, 1], s0[9:, :, 1]) < (2e-6 if dt == "f32" else 4e-3)
