"""The production bf16 conv kernels at the shapes the bench runs (VERDICT r1 "what's weak" 1).

bench.py's config-2 step (B=1024, 2 global + 4 local views + the originals) runs the audio
conv1 kernels at N = 7 x 1024 = 7168 samples (student) and 2048 (teacher), and the mid-layer
weights-stationary kernels (conv_ws / wgrad_ws) at the same N.  Those kernels are persistent:
grid = min(tiles, resident blocks), so at bench size every block walks tens of tiles through
the cross-tile loop, the LDS-reuse barrier and the next-tile register prefetch -- paths the
small-N tests (one tile per block) never reach.  Here they run:

  * at bench size, against a float64 reference computed on the GPU with torch (a tap loop of
    f64 matmuls -- no MIOpen, no libavdino) from the SAME bf16 operands;
  * at small N with avd_options.grid_cap forcing a few blocks (many tiles each), against the
    uncapped launch: forward / dgrad tiles are independent of the block that computes them
    (bit-identical), weight gradients are fp32 sums in another order (rel 1e-6).

Tolerances: stored bf16 maps rel-L2 5e-3 (one bf16 rounding of the output); f32 reductions of
stored values (BN statistics, weight gradients) 1e-5 vs float64.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
F = pytest.importorskip("torch.nn.functional")

T = torch.bfloat16
F64 = torch.float64


@pytest.fixture(scope="module")
def ops():
    from avdino import ops as _ops
    return _ops


def grel(a, b):
    a, b = a.to(F64).reshape(-1), b.to(F64).reshape(-1)
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def rnd(g, shape, lo=-1.0, hi=1.0, dtype=torch.float32):
    return (torch.rand(*shape, generator=g, device="cuda") * (hi - lo) + lo).to(dtype)


def _chunks(N, per_sample_elems, budget=2 ** 27):
    step = max(1, budget // max(per_sample_elems, 1))
    return [(s, min(N, s + step)) for s in range(0, N, step)]


def conv_ref(x, w, pad):
    """NHWC float64 conv: x [N,H,W,Ci], w [Co,Ci,K,K] -> [N,Ho,Wo,Co] (tap loop of matmuls)."""
    N, H, W, Ci = x.shape
    Co, _, K, _ = w.shape
    Ho, Wo = H + 2 * pad - K + 1, W + 2 * pad - K + 1
    w = w.to(F64)
    y = torch.empty(N, Ho, Wo, Co, device="cuda", dtype=F64)
    for a, b in _chunks(N, (H + 2 * pad) * (W + 2 * pad) * max(Ci, Co) * 3):
        xp = F.pad(x[a:b].to(F64), (0, 0, pad, pad, pad, pad))
        acc = torch.zeros(b - a, Ho, Wo, Co, device="cuda", dtype=F64)
        for i in range(K):
            for j in range(K):
                acc += xp[:, i:i + Ho, j:j + Wo, :] @ w[:, :, i, j].T
        y[a:b] = acc
    return y


def wgrad_ref(x, dy, K, pad):
    """dW[o,c,i,j] = sum_{n,h,w} dy[n,h,w,o] x_pad[n,h+i,w+j,c], float64."""
    N, H, W, Ci = x.shape
    _, Ho, Wo, Co = dy.shape
    dw = torch.zeros(Co, Ci, K, K, device="cuda", dtype=F64)
    for a, b in _chunks(N, (H + 2 * pad) * (W + 2 * pad) * (Ci + Co) * 2):
        xp = F.pad(x[a:b].to(F64), (0, 0, pad, pad, pad, pad))
        d = dy[a:b].to(F64).reshape(-1, Co)
        for i in range(K):
            for j in range(K):
                dw[:, :, i, j] += d.T @ xp[:, i:i + Ho, j:j + Wo, :].reshape(-1, Ci)
    return dw


def dgrad_ref(dy, w, pad):
    """dX = conv(dy, w flipped and transposed, K-1-pad), float64."""
    K = w.shape[2]
    w2 = w.to(F64).flip(2, 3).transpose(0, 1).contiguous()
    return conv_ref(dy, w2, K - 1 - pad)


def layout(ops, w, dgrad):
    Co, Ci, K, _ = w.shape
    wk = torch.empty(ops.cl_weight_elems(Co, Ci, K, dgrad), device="cuda", dtype=T)
    ops.cl_weight_layout(w.float().contiguous(), wk, dgrad)
    return wk


# ---------------------------------------------------------------------------- audio conv1
N_STUDENT, N_TEACHER, B_BENCH = 7 * 1024, 2 * 1024, 1024


def test_conv1_forward_stats_bench_size(ops):
    """Audio conv1 (1->8, 5x5 p2, 112x112) forward + BN partial sums at N = 7168."""
    N, B, H, C, K, pad = N_STUDENT, B_BENCH, 112, 8, 5, 2
    G = N // B
    g = torch.Generator(device="cuda").manual_seed(1)
    x = rnd(g, (N, H, H, 1), 0, 1, T)
    w = rnd(g, (C, 1, K, K)).to(T).float() / 5
    bias = rnd(g, (C,), -0.1, 0.1)
    y = torch.empty(N, H, H, C, device="cuda", dtype=T)
    R = ops.cl_stat_rows(H, H, B, K, 1, C, T)
    st = torch.full((C * G * R * 2,), float("nan"), device="cuda")
    ops.cl_conv_fwd(x, layout(ops, w, 0), bias, y, st, N, B, 1, H, H, C, K, pad)
    y_ref = conv_ref(x, w, pad) + bias.to(F64)
    assert grel(y, y_ref) < 5e-3
    s = st.view(C, G, R, 2).to(F64).sum(2)
    yv = y.to(F64).view(G, B * H * H, C)
    assert grel(s[..., 0], yv.sum(1).T) < 1e-5
    assert grel(s[..., 1], (yv ** 2).sum(1).T) < 1e-5


def _bn_setup(g, G, C):
    scale = rnd(g, (G * C,), 0.5, 1.5)
    shift = rnd(g, (G * C,), -0.3, 0.3)
    coef = rnd(g, (G * C * 3,), -0.5, 0.5)
    return scale, shift, coef


def test_conv1_bwd_apply_wgrad_bench_size(ops):
    """c1p8_bwd_wgrad_kernel (BN-backward apply fused with conv1's weight gradient), the
    bench's dominant launch, at N = 7168: 65 tiles per persistent block on MI355X."""
    N, B, H, C, K, pad = N_STUDENT, B_BENCH, 112, 8, 5, 2
    G = N // B
    g = torch.Generator(device="cuda").manual_seed(2)
    x = rnd(g, (N, H, H, 1), 0, 1, T)
    y = (torch.randn(N, H, H, C, generator=g, device="cuda") * 0.8 + 0.1).to(T)
    gout = rnd(g, (N, H // 2, H // 2, C), dtype=T)
    scale, shift, coef = _bn_setup(g, G, C)
    ns = ops.cl_apply_wgrad_slabs(T, N, 1, H, H, C, K, pad)
    assert 0 < ns < N * (H // 16), "persistent grid expected at bench size"
    parts = torch.full((ns * C * K * K,), float("nan"), device="cuda")
    ops.cl_bn_bwd_apply_wgrad(y, gout, scale, shift, coef, x, parts, N, B, 1, H, H, C, K, pad)
    dw = torch.empty(C * K * K, device="cuda")
    ops.sum_rows(parts, ns, C * K * K, dw)
    # the same bf16 dy from the unfused apply kernel, then float64
    dy = torch.empty_like(y)
    ops.cl_bn_bwd_apply(y, gout, 0, scale, shift, coef, dy, N, B, C, H, H)
    dw64 = wgrad_ref(x, dy, K, pad)
    assert grel(dw, dw64) < 1e-5, grel(dw, dw64)


def test_conv1_recompute_bench_size(ops):
    """The stored-y-free conv1 passes the bench runs: teacher statistics (N = 2048, C1_STATS)
    and the student's BN -> ReLU -> pool recomputed from x (N = 7168, C1_APPLY) equal the
    stored-y kernels (bit-exact pooled maps, statistics to fp32 order)."""
    H, C, K, pad, B = 112, 8, 5, 2, B_BENCH
    g = torch.Generator(device="cuda").manual_seed(3)
    w = rnd(g, (C, 1, K, K)).to(T).float() / 5
    bias = rnd(g, (C,), -0.1, 0.1)
    wk = layout(ops, w, 0)
    for N, pas in ((N_TEACHER, ops.C1_STATS), (N_STUDENT, ops.C1_APPLY)):
        G = N // B
        x = rnd(g, (N, H, H, 1), 0, 1, T)
        y = torch.empty(N, H, H, C, device="cuda", dtype=T)
        R0 = ops.cl_stat_rows(H, H, B, K, 1, C, T)
        st0 = torch.empty(C * G * R0 * 2, device="cuda")
        ops.cl_conv_fwd(x, wk, bias, y, st0, N, B, 1, H, H, C, K, pad)
        if pas == ops.C1_STATS:
            R1 = ops.cl_c1_recompute_rows(ops.C1_STATS, T, N, B, 1, H, H, C, K, pad)
            st1 = torch.empty(C * G * R1 * 2, device="cuda")
            ops.cl_c1_recompute(ops.C1_STATS, x, wk, bias, N, B, 1, H, H, C, K, pad, out=st1)
            assert grel(st1.view(C, G, R1, 2).to(F64).sum(2), st0.view(C, G, R0, 2).to(F64).sum(2)) < 1e-6
        else:
            scale, shift, _ = _bn_setup(g, G, C)
            z0 = torch.empty(N, H // 2, H // 2, C, device="cuda", dtype=T)
            ops.cl_bn_relu_pool(y, scale, shift, z0, 0, N, B, C, H, H)
            z1 = torch.full_like(z0, float("nan"))
            ops.cl_c1_recompute(ops.C1_APPLY, x, wk, bias, N, B, 1, H, H, C, K, pad, scale=scale,
                                shift=shift, z=z1)
            assert torch.equal(z0, z1)


def test_conv1_moments_pass_bench_size(ops):
    """The training backward of the audio conv1 without a stored y (pass 4 of
    avd_cl_c1_recompute + combine) at N = 7168, ~100 tiles per block: its BN-backward sums equal
    avd_cl_bn_bwd_reduce's (fp32 order), its patch Gram matrix and patch sums equal float64, and
    dW is within the stored-y path's bf16 rounding of dy."""
    N, B, H, C, K, pad = N_STUDENT, B_BENCH, 112, 8, 5, 2
    G = N // B
    g = torch.Generator(device="cuda").manual_seed(7)
    x = rnd(g, (N, H, H, 1), 0, 1, T)
    w = rnd(g, (C, 1, K, K)).to(T).float() / 5
    bias = rnd(g, (C,), -0.1, 0.1)
    wk = layout(ops, w, 0)
    y = torch.empty(N, H, H, C, device="cuda", dtype=T)
    R0 = ops.cl_stat_rows(H, H, B, K, 1, C, T)
    st0 = torch.empty(C * G * R0 * 2, device="cuda")
    ops.cl_conv_fwd(x, wk, bias, y, st0, N, B, 1, H, H, C, K, pad)
    gamma, beta = rnd(g, (C,), 0.8, 1.2), rnd(g, (C,), -0.2, 0.2)
    bn = torch.empty(4, G * C, device="cuda")
    ops.bn_finalize(st0, G, R0, C, B * H * H, gamma, beta, bn[0], bn[1], bn[2], bn[3])
    gz = rnd(g, (N, H // 2, H // 2, C), dtype=T)
    Rb = ops.cl_bn_bwd_rows(B, C, H, H, T)
    p0 = torch.empty(C * G * Rb * 2, device="cuda")
    ops.cl_bn_bwd_reduce(y, gz, 0, bn[2], bn[3], bn[0], bn[1], p0, N, B, C, H, H)
    coef = torch.empty(G * C * 3, device="cuda")
    dg, dbt = torch.empty(C, device="cuda"), torch.empty(C, device="cuda")
    ops.bn_bwd_finalize(p0, G, Rb, C, B * H * H, gamma, bn[0], bn[1], coef, dg, dbt, None)
    ns = ops.cl_apply_wgrad_slabs(T, N, 1, H, H, C, K, pad)
    f0 = torch.empty(ns * C * K * K, device="cuda")
    ops.cl_bn_bwd_apply_wgrad(y, gz, bn[2], bn[3], coef, x, f0, N, B, 1, H, H, C, K, pad)
    d0 = torch.empty(C * K * K, device="cuda")
    ops.sum_rows(f0, ns, C * K * K, d0)
    R4 = ops.cl_c1_recompute_rows(ops.C1_REDUCE_MOMENTS, T, N, B, 1, H, H, C, K, pad)
    assert 0 < R4 and G * R4 * 8 < N * (H // 16), "blocks with many tiles each expected"
    mc = ops.c1_moment_cols(C, K)
    m4 = torch.full((C * G * R4 * 2 + R4 * G * mc,), float("nan"), device="cuda")
    ops.cl_c1_recompute(ops.C1_REDUCE_MOMENTS, x, wk, bias, N, B, 1, H, H, C, K, pad, scale=bn[2],
                        shift=bn[3], mean=bn[0], invstd=bn[1], gz=gz, out=m4)
    r4 = m4[:C * G * R4 * 2].view(C, G, R4, 2).to(F64).sum(2)
    r0 = p0.view(C, G, Rb, 2).to(F64).sum(2)
    assert grel(r4, r0) < 1e-5, grel(r4, r0)
    mom = torch.empty(G * mc, device="cuda")
    ops.sum_rows(m4, R4, G * mc, mom, off=C * G * R4 * 2)
    mh = mom.view(G, mc).to(F64)
    # float64 moments: M = sum dz x25 (dz routed at the first max of relu(bn(y)) of the same
    # bf16 y), Gram = sum x25 x25^T, S = sum x25, per BN group
    gram = torch.zeros(G, 25, 25, device="cuda", dtype=F64)
    sx = torch.zeros(G, 25, device="cuda", dtype=F64)
    mz = torch.zeros(G, C, 25, device="cuda", dtype=F64)
    sc, sf = bn[2].view(G, C).to(F64), bn[3].view(G, C).to(F64)
    for a, b in _chunks(N, H * H * 25 * 2):
        u = F.unfold(x[a:b].permute(0, 3, 1, 2).to(F64), K, padding=pad)     # [n, 25, H*H]
        for gi in range(a // B, (b - 1) // B + 1):
            lo, hi = max(a, gi * B) - a, min(b, (gi + 1) * B) - a
            n = hi - lo
            gram[gi] += torch.einsum("nip,njp->ij", u[lo:hi], u[lo:hi])
            sx[gi] += u[lo:hi].sum((0, 2))
            z = torch.relu(y[a + lo:a + hi].to(F64) * sc[gi] + sf[gi])
            zw = z.view(n, H // 2, 2, H // 2, 2, C).permute(0, 1, 3, 5, 2, 4).reshape(n, H // 2, H // 2, C, 4)
            best, am = zw.max(-1)
            gzw = gz[a + lo:a + hi].to(F64)
            dzw = torch.where((torch.arange(4, device="cuda") == am[..., None]) & (best[..., None] > 0),
                              gzw[..., None], torch.zeros((), device="cuda", dtype=F64))
            dz = dzw.view(n, H // 2, H // 2, C, 2, 2).permute(0, 1, 4, 2, 5, 3).reshape(n, H * H, C)
            mz[gi] += torch.einsum("npc,ntp->ct", dz, u[lo:hi])
    assert grel(mh[:, C * 25:C * 25 + 625].view(G, 25, 25), gram) < 1e-5
    assert grel(mh[:, C * 25 + 625:], sx) < 1e-5
    assert grel(mh[:, :C * 25].view(G, C, 25), mz) < 1e-5
    d4 = torch.empty(C * K * K, device="cuda")
    ops.cl_c1_recompute_combine(mom, coef, wk, bias, d4, G, C)
    # dW of the moments formula in float64 (y = w . x25 + b unrounded in the kx term)
    k3 = coef.view(G, C, 3).to(F64)
    w64 = w.view(C, 25).to(T).to(F64)          # the bf16 weights both paths compute with
    sy = torch.einsum("ct,gts->gcs", w64, gram) + bias.to(F64)[None, :, None] * sx[:, None, :]
    dw64 = (k3[..., 0:1] * mz + k3[..., 1:2] * sy + k3[..., 2:3] * sx[:, None, :]).sum(0)
    # the same formula on the kernel's moments (isolates the combine from the moment sums)
    km, kg, ks = mh[:, :C * 25].view(G, C, 25), mh[:, C * 25:C * 25 + 625].view(G, 25, 25), mh[:, C * 25 + 625:]
    ksy = torch.einsum("ct,gts->gcs", w64, kg) + bias.to(F64)[None, :, None] * ks[:, None, :]
    dwk = (k3[..., 0:1] * km + k3[..., 1:2] * ksy + k3[..., 2:3] * ks[:, None, :]).sum(0)
    print("moments rel: M", grel(km, mz), "Gram", grel(kg, gram), "S", grel(ks, sx),
          "| dW: combine vs f64 formula on kernel moments", grel(d4, dwk), "kernel-moment dW vs f64",
          grel(dwk, dw64), "vs stored-y", grel(d4, d0), "stored-y vs f64", grel(d0, dw64))
    assert grel(d4, dw64) < 1e-4, grel(d4, dw64)
    # the stored-y path rounds dy to bf16 before its weight gradient; dy is centred, so over
    # 90M pixels that rounding shows in dW amplified by the cancellation (2.5 % measured): the
    # moments pass is the more accurate of the two
    assert grel(d4, d0) < 5e-2, grel(d4, d0)
    assert grel(d0, dw64) < 5e-2


# ---------------------------------------------------------------------------- mid layers
# (Cin, H, Cout, K, pad, N): the CentralNet audio conv2-4 and image conv2 at bench-scale N
WS_BENCH = [(8, 56, 16, 5, 2, 2048), (16, 28, 32, 5, 2, 2048), (32, 14, 64, 5, 2, 4096),
            (32, 14, 64, 5, 0, 4096)]
# the 3x3 layers of the SimCLR / unimodal encoders at BASELINE config 4's B = 2048 (conv3.hip)
C3_BENCH = [(32, 56, 64, 3, 1, 2048), (64, 28, 128, 3, 1, 2048), (128, 14, 256, 3, 1, 2048),
            (32, 14, 64, 3, 1, 2048), (64, 7, 128, 3, 1, 2048)]


@pytest.mark.parametrize("shape", WS_BENCH + C3_BENCH)
def test_ws_kernels_bench_size(ops, shape):
    """conv_ws / conv3 forward (+ stats), dgrad and weight gradient at bench-scale N vs
    float64."""
    Ci, H, Co, K, pad, N = shape
    B = 1024
    G = N // B
    Ho = H + 2 * pad - K + 1
    g = torch.Generator(device="cuda").manual_seed(4 + H + pad)
    x = rnd(g, (N, H, H, Ci), dtype=T)
    w = (rnd(g, (Co, Ci, K, K)) / (Ci * K * K) ** 0.5).to(T).float()
    bias = rnd(g, (Co,), -0.1, 0.1)
    y = torch.empty(N, Ho, Ho, Co, device="cuda", dtype=T)
    R = ops.cl_stat_rows(Ho, Ho, B, K, Ci, Co, T)
    st = torch.full((Co * G * R * 2,), float("nan"), device="cuda")
    ops.cl_conv_fwd(x, layout(ops, w, 0), bias, y, st, N, B, Ci, H, H, Co, K, pad)
    assert grel(y, conv_ref(x, w, pad) + bias.to(F64)) < 5e-3
    s = st.view(Co, G, R, 2).to(F64).sum(2)
    yv = y.to(F64).view(G, B * Ho * Ho, Co)
    assert grel(s[..., 0], yv.sum(1).T) < 1e-5
    assert grel(s[..., 1], (yv ** 2).sum(1).T) < 1e-5
    dy = rnd(g, (N, Ho, Ho, Co), dtype=T)
    dx = torch.empty(N, H, H, Ci, device="cuda", dtype=T)
    ops.cl_conv_dgrad(dy, layout(ops, w, 1), dx, N, Ci, H, H, Co, K, pad)
    assert grel(dx, dgrad_ref(dy, w, pad)) < 5e-3
    nch = ops.cl_wgrad_chunks(N, Co, Ci, K)
    parts = torch.full((nch * Co * Ci * K * K,), float("nan"), device="cuda")
    ops.cl_conv_wgrad(x, dy, parts, N, Ci, H, H, Co, K, pad)
    dw = torch.empty(Co * Ci * K * K, device="cuda")
    ops.sum_rows(parts, nch, Co * Ci * K * K, dw)
    assert grel(dw, wgrad_ref(x, dy, K, pad)) < 1e-5


@pytest.mark.parametrize("HC", [(14, 64), (10, 64)])
def test_bn_bwd_reduce_pooled_mode2_bench_size(ops, HC, avd_opts):
    """The encoder tails' BN-backward sums from the (c, h, w)-flattened pooled map and gradient
    (bwd_reduce_pooled_m2_kernel: a wave per channel, coalesced planes) at N = 7168 against the
    generic pooled kernel and float64 of sum dz, sum dz * xhat."""
    H, C = HC
    N, B = N_STUDENT, B_BENCH
    G, Hp = N // B, H // 2
    g = torch.Generator(device="cuda").manual_seed(11 + H)
    y = (torch.randn(N, H, H, C, generator=g, device="cuda") * 0.8).to(T)
    gamma, beta = rnd(g, (C,), 0.5, 1.5), rnd(g, (C,), -0.2, 0.2)
    yf = y.to(F64).view(G, -1, C)
    mean = yf.mean(1).float().reshape(-1).contiguous()
    invstd = (yf.var(1, unbiased=False) + 1e-5).rsqrt().float().reshape(-1).contiguous()
    scale = (gamma.view(1, C) * invstd.view(G, C)).reshape(-1).contiguous()
    shift = (beta.view(1, C) - mean.view(G, C) * scale.view(G, C)).reshape(-1).contiguous()
    pooled = torch.empty(N * C * Hp * Hp, device="cuda")
    ops.cl_bn_relu_pool(y, scale, shift, pooled, 2, N, B, C, H, H)
    gout = torch.randn(N * C * Hp * Hp, generator=g, device="cuda")
    R = ops.cl_bn_bwd_rows(B, C, H, H, T)
    p1 = torch.full((C * G * R * 2,), float("nan"), device="cuda")
    ops.cl_bn_bwd_reduce_pooled(y, pooled, gout, 2, gamma, beta, mean, invstd, p1, N, B, C, H, H)
    avd_opts(generic_m2=1)
    p0 = torch.full((C * G * R * 2,), float("nan"), device="cuda")
    ops.cl_bn_bwd_reduce_pooled(y, pooled, gout, 2, gamma, beta, mean, invstd, p0, N, B, C, H, H)
    s1 = p1.view(C, G, R, 2).to(F64).sum(2)
    s0 = p0.view(C, G, R, 2).to(F64).sum(2)
    assert grel(s1, s0) < 1e-5, grel(s1, s0)
    pv, gv = pooled.to(F64).view(G, B, C, -1), gout.to(F64).view(G, B, C, -1)
    dz = torch.where(pv > 0, gv, torch.zeros_like(gv))
    xh = (pv - beta.to(F64).view(1, 1, C, 1)) / gamma.to(F64).view(1, 1, C, 1)
    assert grel(s1[..., 0], dz.sum((1, 3)).T) < 1e-5
    assert grel(s1[..., 1], (dz * xh).sum((1, 3)).T) < 1e-5


# ---------------------------------------------------------------------------- forced small grids
def _capped(avd_opts, cap, fn):
    avd_opts(grid_cap=0)
    a = fn()
    avd_opts(grid_cap=cap)
    b = fn()
    avd_opts(grid_cap=0)
    return a, b


@pytest.mark.parametrize("shape", [(8, 56, 16, 5, 2, 48), (16, 28, 32, 5, 2, 48),
                                   (32, 14, 64, 5, 2, 96), (32, 14, 64, 5, 0, 96)])
@pytest.mark.parametrize("cap", [1, 3, 7])
def test_ws_kernels_many_tiles_per_block(ops, shape, cap, avd_opts):
    Ci, H, Co, K, pad, N = shape
    B = N // 2
    G = 2
    Ho = H + 2 * pad - K + 1
    g = torch.Generator(device="cuda").manual_seed(50 + H)
    x = rnd(g, (N, H, H, Ci), dtype=T)
    w = (rnd(g, (Co, Ci, K, K)) / (Ci * K * K) ** 0.5).to(T).float()
    bias = rnd(g, (Co,), -0.1, 0.1)
    dy = rnd(g, (N, Ho, Ho, Co), dtype=T)
    wk, wd = layout(ops, w, 0), layout(ops, w, 1)

    def run():
        # the forward's partial rows are per resident block: the count follows the grid cap
        R = ops.cl_stat_rows(Ho, Ho, B, K, Ci, Co, T)
        y = torch.full((N, Ho, Ho, Co), float("nan"), device="cuda", dtype=T)
        st = torch.full((Co * G * R * 2,), float("nan"), device="cuda")
        ops.cl_conv_fwd(x, wk, bias, y, st, N, B, Ci, H, H, Co, K, pad)
        dx = torch.full((N, H, H, Ci), float("nan"), device="cuda", dtype=T)
        ops.cl_conv_dgrad(dy, wd, dx, N, Ci, H, H, Co, K, pad)
        nch = ops.cl_wgrad_chunks(N, Co, Ci, K)
        parts = torch.full((nch * Co * Ci * K * K,), float("nan"), device="cuda")
        ops.cl_conv_wgrad(x, dy, parts, N, Ci, H, H, Co, K, pad)
        dw = torch.empty(Co * Ci * K * K, device="cuda")
        ops.sum_rows(parts, nch, Co * Ci * K * K, dw)
        torch.cuda.synchronize()
        return y, st.view(Co, G, R, 2).to(F64).sum(2), dx, dw

    (y0, s0, dx0, dw0), (y1, s1, dx1, dw1) = _capped(avd_opts, cap, run)
    assert torch.equal(y0, y1) and torch.equal(dx0, dx1)
    # fp32 sum order: statistics are lane-local running sums over a block's tiles, so a cap of
    # one block sums ~10^4 values per lane (sum of signed values: 2.2e-6 measured at cap 1)
    assert grel(s1, s0) < 1e-5 and grel(dw1, dw0) < 5e-6
    assert grel(dw1, wgrad_ref(x, dy, K, pad)) < 1e-5


@pytest.mark.parametrize("cap", [1, 5])
def test_conv1_wgrad_many_tiles_per_block(ops, cap, avd_opts):
    N, B, H, C, K, pad = 12, 6, 112, 8, 5, 2
    G = N // B
    g = torch.Generator(device="cuda").manual_seed(60 + cap)
    x = rnd(g, (N, H, H, 1), 0, 1, T)
    y = torch.randn(N, H, H, C, generator=g, device="cuda").to(T)
    gout = rnd(g, (N, H // 2, H // 2, C), dtype=T)
    scale, shift, coef = _bn_setup(g, G, C)

    def run():
        ns = ops.cl_apply_wgrad_slabs(T, N, 1, H, H, C, K, pad)
        parts = torch.full((ns * C * K * K,), float("nan"), device="cuda")
        ops.cl_bn_bwd_apply_wgrad(y, gout, scale, shift, coef, x, parts, N, B, 1, H, H, C, K, pad)
        dw = torch.empty(C * K * K, device="cuda")
        ops.sum_rows(parts, ns, C * K * K, dw)
        torch.cuda.synchronize()
        return ns, dw

    (n0, dw0), (n1, dw1) = _capped(avd_opts, cap, run)
    assert n1 == cap < n0
    assert grel(dw1, dw0) < 1e-6


# ---------------------------------------------------------------------------- whole step
def _ref_grads(state, batch, E, D, P, autocast_dtype, dtype=torch.float32):
    """The reference's step (oracle/torch_port.py restates its modules and ops) on the GPU,
    fp32 or under torch.autocast(dtype) -- the reference's own mixed-precision mode is
    '16-mixed' (run_dino.py:360); bf16 autocast is the same recipe in our storage type.
    dtype=float64: the same step with float64 parameters and inputs (no autocast)."""
    from oracle import torch_port as TP
    torch.manual_seed(0)
    m = TP.DinoMSE(E, D, P, dropout=0.0, fusion_dropout=0.0).cuda().to(dtype)
    m.load_state_dict({k: torch.from_numpy(np.array(v)) for k, v in state.items()}, strict=True)
    b = {k: v.to(dtype) for k, v in batch.items()}
    with torch.autocast("cuda", dtype=autocast_dtype or torch.float32, enabled=autocast_dtype is not None):
        fi, fa, s_, t_ = m(b["image"], b["audio"], b["g_img"], b["g_aud"], b["l_img"], b["l_aud"])
        loss = TP.dino_loss(s_.to(dtype), t_.to(dtype)) + TP.mse_loss(fi.to(dtype), fa.to(dtype))
    loss.backward()
    return loss.item(), {k: p.grad.detach().to(F64).clone() for k, p in m.named_parameters()
                         if p.grad is not None}


@pytest.mark.parametrize("B,L", [(1024, 4), (512, 7), (256, 7)], ids=["config2", "B512_L7", "B256_L7"])
def test_bf16_step_vs_fp32_step_config2(capsys, B, L):
    """The benchmarked bf16 step at config-2 size (B = 1024, 2 global + 4 local views, mse,
    E = D = 256, P = 128: conv_ws / wgrad_ws mid layers, the Gram / routed / window-space conv1
    passes) against the ORACLE: the reference's step restated in torch ops (oracle/torch_port.py,
    pinned to the reference's own fixtures by tests/test_torch_port.py) in fp32 on the GPU, from
    identical parameters and inputs -- no HIP-vs-HIP link.  Per-tensor bounds come
    from the REFERENCE's own mixed precision: the same port under bf16 / fp16 autocast vs fp32.
    At initialisation the conv-weight / BN gradients are small sums of large cancelling terms,
    so one bf16 rounding of the stored maps moves them by ~10 % -- in the reference's recipe as
    in ours.  Bounds: loss 1e-3 relative; every tensor within 2x the reference's own
    mixed-precision error (the larger of its bf16-autocast and its fp16 '16-mixed' error, floor
    1e-2: on an 8-value BN tensor either one alone can sit far below the other by chance); the
    median within 1.25x of the bf16-autocast median.  The fp32 engine is checked against the same
    oracle (loss 1e-4; every tensor within half the reference's own autocast error, floor 5e-3
    rel-L2: bias gradients are sums over 6144-7168 rows that cancel, so fp32 summation order alone
    moves them by up to 4e-3 -- measured).  B512_L7 / B256_L7 run the student conv
    branches at 10 BN groups (2 global + 7 local views + the originals); B256_L7 is the case that
    failed the bf16-only bound in round 3 (audio bn1 weight)."""
    from avdino.engine import Hyper, MultiCentralEngine
    from avdino.params import ParamStore
    from avdino.spec import multimodal_dino_sd
    from oracle.params import make_state
    from oracle import spec as OS
    E = D = 256
    P, G = 128, 2
    state = make_state(OS.multimodal_dino_spec("mse", E, D, P), 301)
    g = torch.Generator(device="cuda").manual_seed(302)

    def px(*s):
        return torch.randint(0, 256, s, generator=g, device="cuda", dtype=torch.int32).float() / 255

    batch = dict(g_img=px(B, G, 1, 28, 28), g_aud=px(B, G, 1, 112, 112), l_img=px(B, L, 1, 28, 28),
                 l_aud=px(B, L, 1, 112, 112), image=px(B, 1, 28, 28), audio=px(B, 1, 112, 112))
    out = {}
    for name, act in (("f32", torch.float32), ("bf16", torch.bfloat16)):
        store = ParamStore(multimodal_dino_sd("mse", E, D, P), "cuda")
        store.load_state_dict({k: torch.from_numpy(np.array(v)) for k, v in state.items()})
        eng = MultiCentralEngine(store, "mse", E, D, P, Hyper(dropout=0.0, fusion_dropout=0.0),
                                 act_dtype=act)
        loss = eng.forward(batch).item()
        eng.backward()
        out[name] = (loss, {k: store.grad_of(k).detach().to(F64).clone() for k in store.live_keys})
    ref = {n: _ref_grads(state, batch, E, D, P, a) for n, a in
           (("f32", None), ("bf16", torch.bfloat16), ("f16", torch.float16))}
    (l32, g32), (l16, g16) = out["f32"], out["bf16"]
    r32 = ref["f32"][1]
    big = max(v.norm().item() for v in r32.values())
    keys = [k for k in g32 if r32[k].norm().item() > 1e-6 * big]
    ours = {k: grel(g16[k], r32[k]) for k in keys}          # bf16 engine vs the fp32 oracle
    e32 = {k: grel(g32[k], r32[k]) for k in keys}           # fp32 engine vs the fp32 oracle
    rbf = {k: grel(ref["bf16"][1][k], ref["f32"][1][k]) for k in keys}
    rfp = {k: grel(ref["f16"][1][k], ref["f32"][1][k]) for k in keys}
    ratio = sorted(((ours[k] / max(rbf[k], rfp[k], 1e-2), k) for k in keys), reverse=True)
    med = (float(np.median(list(ours.values()))), float(np.median(list(rbf.values()))),
           float(np.median(list(rfp.values()))))
    with capsys.disabled():
        print(f"\nbf16 vs fp32 step (B={B}, L={L}): loss {l16:.6f} vs {l32:.6f} "
              f"(rel {abs(l16 - l32) / abs(l32):.2e}); fp32 engine vs fp32 reference loss "
              f"{abs(l32 - ref['f32'][0]):.2e}")
        print(f"grad rel-L2 median: ours bf16 {med[0]:.3e}, reference bf16-autocast {med[1]:.3e}, "
              f"reference fp16-autocast {med[2]:.3e}")
        for r, k in ratio[:8]:
            print(f"  {k}: ours {ours[k]:.3e} ref-bf16 {rbf[k]:.3e} ref-fp16 {rfp[k]:.3e}")
        print(f"fp32 engine vs fp32 oracle: worst rel-L2 {max(e32.values()):.2e}")
    assert abs(l32 - ref["f32"][0]) < 1e-4
    bad32 = [(k, e32[k]) for k in keys if e32[k] > max(0.5 * max(rbf[k], rfp[k]), 5e-3)]
    assert not bad32, bad32
    assert abs(l16 - ref["f32"][0]) / abs(ref["f32"][0]) < 1e-3
    assert ratio[0][0] < 2.0, ratio[:4]
    assert med[0] < 1.25 * med[1], med


def test_fp32_step_vs_float64_port_config2(capsys):
    """fp32 parity at config-2 size against a FLOAT64 oracle.  The fp32
    engine (the parity mode: the same kernels on f32 maps, f32-accumulated MFMA) and the
    reference's step restated in torch ops in fp32 (torch_port) both differ from the float64
    port by their own fp32 rounding and summation order; the engine must not be worse than the
    reference's own fp32 recipe: per tensor, rel-L2(engine, f64) <= max(1.5 x rel-L2(port fp32,
    f64), 1e-4), where 1e-4 is SURVEY 8(c)'s per-tensor bound, and the median over tensors within
    1.1x the port's median.  Loss within 1e-5 of float64.  Measured (round 6): engine median 2.41e-5
    vs port 2.50e-5, worst 2.11e-3 (audio bn3 bias, 1.50x the port's 1.41e-3) vs the port's worst
    2.43e-3 -- the 2.9e-3 between the fp32 engine and the fp32 port is the two fp32 recipes'
    own rounding, not an engine error.
    Tensors whose float64 gradient is below 1e-6 of the largest (the conv / Linear biases that
    feed a BatchNorm: mathematically zero, rounding noise only) are excluded, as in SURVEY 8(c)."""
    from avdino.engine import Hyper, MultiCentralEngine
    from avdino.params import ParamStore
    from avdino.spec import multimodal_dino_sd
    from oracle.params import make_state
    from oracle import spec as OS
    E = D = 256
    P, G, L, B = 128, 2, 4, 1024
    state = make_state(OS.multimodal_dino_spec("mse", E, D, P), 301)
    g = torch.Generator(device="cuda").manual_seed(302)

    def px(*s):
        return torch.randint(0, 256, s, generator=g, device="cuda", dtype=torch.int32).float() / 255

    batch = dict(g_img=px(B, G, 1, 28, 28), g_aud=px(B, G, 1, 112, 112), l_img=px(B, L, 1, 28, 28),
                 l_aud=px(B, L, 1, 112, 112), image=px(B, 1, 28, 28), audio=px(B, 1, 112, 112))
    store = ParamStore(multimodal_dino_sd("mse", E, D, P), "cuda")
    store.load_state_dict({k: torch.from_numpy(np.array(v)) for k, v in state.items()})
    eng = MultiCentralEngine(store, "mse", E, D, P, Hyper(dropout=0.0, fusion_dropout=0.0),
                             act_dtype=torch.float32)
    l32 = eng.forward(batch).item()
    eng.backward()
    g32 = {k: store.grad_of(k).detach().to(F64).clone() for k in store.live_keys}
    del eng, store
    torch.cuda.empty_cache()
    lp, gp = _ref_grads(state, batch, E, D, P, None)
    l64, g64 = _ref_grads(state, batch, E, D, P, None, dtype=F64)
    big = max(v.norm().item() for v in g64.values())
    keys = [k for k in g32 if g64[k].norm().item() > 1e-6 * big]
    ours = {k: grel(g32[k], g64[k]) for k in keys}
    port = {k: grel(gp[k], g64[k]) for k in keys}
    ratio = sorted(((ours[k] / max(port[k], 1e-30), k) for k in keys), reverse=True)
    bad = [(k, ours[k], port[k]) for k in keys if ours[k] > max(1.5 * port[k], 1e-4)]
    with capsys.disabled():
        print(f"\nfp32 vs float64 (B={B}): loss engine {abs(l32 - l64):.2e}, port {abs(lp - l64):.2e}; "
              f"rel-L2 median engine {np.median(list(ours.values())):.2e}, "
              f"port {np.median(list(port.values())):.2e}; max engine {max(ours.values()):.2e}, "
              f"port {max(port.values()):.2e}")
        for r, k in ratio[:10]:
            print(f"  {k}: engine {ours[k]:.3e} port-fp32 {port[k]:.3e} (x{r:.2f})")
        worst = max(keys, key=lambda k: ours[k])
        print(f"  worst engine tensor {worst}: {ours[worst]:.3e} (port {port[worst]:.3e})")
    assert abs(l32 - l64) < 1e-5, (l32, l64)
    assert not bad, bad
    assert np.median(list(ours.values())) <= 1.1 * np.median(list(port.values()))


def _ref_curve(state, batches, E, D, P, autocast_dtype):
    """Losses of len(batches) full reference training steps (torch_port.train_step: forward,
    loss, update_teacher, backward, Adam -- dino.py:1214-1238 with Lightning's automatic
    optimisation), fp32 or under autocast, on the GPU."""
    from oracle import torch_port as TP
    torch.manual_seed(0)
    m = TP.DinoMSE(E, D, P, dropout=0.0, fusion_dropout=0.0).cuda()
    m.load_state_dict({k: torch.from_numpy(np.array(v)) for k, v in state.items()}, strict=True)
    opt = TP.make_optimizer(m)
    out = []
    for b in batches:
        with torch.autocast("cuda", dtype=autocast_dtype or torch.float32, enabled=autocast_dtype is not None):
            fi, fa, s_, t_ = m(b["image"], b["audio"], b["g_img"], b["g_aud"], b["l_img"], b["l_aud"])
            loss = TP.dino_loss(s_.float(), t_.float()) + TP.mse_loss(fi.float(), fa.float())
        m.update_teacher()
        opt.zero_grad()
        loss.backward()
        opt.step()
        out.append(loss.item())
    return np.array(out)


def test_bf16_three_step_loss_curve_config2(capsys):
    """Three full bf16 training steps of the benchmarked engine at config-2 size (B = 1024,
    2 + 4 views, mse, E = D = 256, P = 128; Adam, teacher EMA, centre update between steps)
    against the reference's own steps restated in torch ops (torch_port, the pinned oracle) in
    fp32 and under bf16 / fp16 autocast, from the same state over the same batches.  Band: every
    step's loss within max(2x the reference's own autocast deviation from fp32, 2e-4 relative)
    of the fp32 reference."""
    from avdino.engine import Hyper, MultiCentralEngine
    from avdino.params import ParamStore
    from avdino.spec import multimodal_dino_sd
    from oracle.params import make_state
    from oracle import spec as OS
    E = D = 256
    P, G, L, B = 128, 2, 4, 1024
    state = make_state(OS.multimodal_dino_spec("mse", E, D, P), 311)
    g = torch.Generator(device="cuda").manual_seed(312)

    def px(*s):
        return torch.randint(0, 256, s, generator=g, device="cuda", dtype=torch.int32).float() / 255

    batches = [dict(g_img=px(B, G, 1, 28, 28), g_aud=px(B, G, 1, 112, 112), l_img=px(B, L, 1, 28, 28),
                    l_aud=px(B, L, 1, 112, 112), image=px(B, 1, 28, 28), audio=px(B, 1, 112, 112))
               for _ in range(3)]
    store = ParamStore(multimodal_dino_sd("mse", E, D, P), "cuda")
    store.load_state_dict({k: torch.from_numpy(np.array(v)) for k, v in state.items()})
    eng = MultiCentralEngine(store, "mse", E, D, P, Hyper(dropout=0.0, fusion_dropout=0.0),
                             act_dtype=torch.bfloat16)
    ours = np.array([eng.step(b).item() for b in batches])
    r32 = _ref_curve(state, batches, E, D, P, None)
    rbf = _ref_curve(state, batches, E, D, P, torch.bfloat16)
    rfp = _ref_curve(state, batches, E, D, P, torch.float16)
    band = np.maximum(2 * np.maximum(np.abs(rbf - r32), np.abs(rfp - r32)), 2e-4 * np.abs(r32))
    with capsys.disabled():
        print(f"\nconfig-2 bf16 3-step curve: ours {ours}, reference fp32 {r32}, bf16-autocast {rbf}, "
              f"fp16-autocast {rfp}; |ours - fp32| {np.abs(ours - r32)} band {band}")
    assert np.all(np.abs(ours - r32) <= band), (ours, r32, band)


def test_simclr_conv1_bwd_apply_wgrad_bench_size(ops):
    """c1w3_kernel (the 3x3 encoders' conv1 1->32 p1 BN-backward apply fused with dW) at
    config 4's N = 2048 spectrograms (112x112): against the unfused apply + weight gradient
    (same bf16 dy) and float64."""
    N, B, H, C, K, pad = 2048, 2048, 112, 32, 3, 1
    G = N // B
    g = torch.Generator(device="cuda").manual_seed(21)
    x = rnd(g, (N, H, H, 1), 0, 1, T)
    y = (torch.randn(N, H, H, C, generator=g, device="cuda") * 0.8 + 0.1).to(T)
    gout = rnd(g, (N, H // 2, H // 2, C), dtype=T)
    scale, shift, coef = _bn_setup(g, G, C)
    ns = ops.cl_apply_wgrad_slabs(T, N, 1, H, H, C, K, pad)
    assert 0 < ns < N * (H // 4), "persistent grid expected at bench size"
    parts = torch.full((ns * C * K * K,), float("nan"), device="cuda")
    ops.cl_bn_bwd_apply_wgrad(y, gout, scale, shift, coef, x, parts, N, B, 1, H, H, C, K, pad)
    dw = torch.empty(C * K * K, device="cuda")
    ops.sum_rows(parts, ns, C * K * K, dw)
    dy = torch.empty_like(y)
    ops.cl_bn_bwd_apply(y, gout, 0, scale, shift, coef, dy, N, B, C, H, H)
    dw64 = wgrad_ref(x, dy, K, pad)
    assert grel(dw, dw64) < 1e-5, grel(dw, dw64)


# ---------------------------------------------------------------------------- off-centre BN statistics
# (kind, Cin, H, Cout, K, pad, N): every forward-statistics producer of the bench steps -- the
# audio/image conv1 (stored y, and the audio conv1's stored-y-free statistics pass), the
# weights-stationary mid layers, the 3x3 conv3p layers
OFFC = ([("cl", 1, 112, 8, 5, 2, N_STUDENT), ("c1s", 1, 112, 8, 5, 2, N_STUDENT), ("cl", 1, 28, 32, 5, 2, N_STUDENT)]
        + [("cl",) + s for s in WS_BENCH] + [("cl",) + s for s in C3_BENCH[:2]])


def _offc_stats(ops, st, G, R, Co, n, rm=None, rv=None, pivot=None):
    gamma, beta = torch.ones(Co, device="cuda"), torch.zeros(Co, device="cuda")
    bn = torch.empty(4, G * Co, device="cuda")
    ops.bn_finalize(st, G, R, Co, n, gamma, beta, bn[0], bn[1], bn[2], bn[3], rm, rv,
                    pivot=pivot, pivot_gs=0)
    return bn[0].view(G, Co).to(F64), 1.0 / bn[1].view(G, Co).to(F64) ** 2 - 1e-5


@pytest.mark.parametrize("cap", [None, 8])
@pytest.mark.parametrize("case", OFFC)
def test_bn_stats_off_centre_bench_size(ops, case, cap, avd_opts):
    """BatchNorm forward statistics where |mean| >> std: x in [0, 1], positive
    weights, bias +20, so every channel's |mean|/std is >= 10 (the regime where var = E[y^2] -
    mean^2 amplifies the error of the fp32 running sums by mean^2 / var).  avd_bn_finalize's mean
    and variance from the kernels' partials vs float64 statistics of the same stored bf16 maps, at
    bench N with the full persistent grid and with the grid capped at 8 blocks (thousands of
    tiles per lane-local running sum).

    Bounds: mean within 1e-4 std; variance rel 1e-4 (invstd within 5e-5: 1/80 of a bf16 ulp of
    the normalised output).  Without a pivot (the first step of a run) the bench's full grid
    meets them everywhere; the capped grid shows what long running sums cost there: up to 1e-1
    variance error on the weights-stationary layers (measured), so those producers
    (avd_cl_stat_pivot) sum about the layer's running mean, as the engine runs them -- after 20
    steps of the running-mean update (emulated here) they meet the bounds on the full grid and
    stay within 3e-4 capped (1.4e-4 measured: what remains is the fp32 rounding of ~6000-term
    lane sums)."""
    kind, Ci, H, Co, K, pad, N = case
    avd_opts(grid_cap=cap or 0)
    B = B_BENCH
    G = N // B
    Ho = H + 2 * pad - K + 1
    g = torch.Generator(device="cuda").manual_seed(100 + Ci + H + Co)
    x = rnd(g, (N, H, H, Ci), 0.0, 1.0, T)
    fan = Ci * K * K
    w = rnd(g, (Co, Ci, K, K), 0.0, 2.0 / fan ** 0.5).to(T).float()
    bias = torch.full((Co,), 20.0, device="cuda") + rnd(g, (Co,), -0.1, 0.1)
    wk = layout(ops, w, 0)
    y = torch.empty(N, Ho, Ho, Co, device="cuda", dtype=T)
    R = ops.cl_stat_rows(Ho, Ho, B, K, Ci, Co, T)
    st = torch.full((Co * G * R * 2,), float("nan"), device="cuda")
    ops.cl_conv_fwd(x, wk, bias, y, st, N, B, Ci, H, H, Co, K, pad)
    Rs = R
    if kind == "c1s":    # the stored-y-free statistics pass the training forward runs
        Rs = ops.cl_c1_recompute_rows(ops.C1_STATS, T, N, B, Ci, H, H, Co, K, pad)
        st = torch.full((Co * G * Rs * 2,), float("nan"), device="cuda")
        ops.cl_c1_recompute(ops.C1_STATS, x, wk, bias, N, B, Ci, H, H, Co, K, pad, out=st)
    mean, var = _offc_stats(ops, st, G, Rs, Co, B * Ho * Ho)
    yv = y.view(G, B * Ho * Ho, Co)
    m64 = torch.stack([yv[i].to(F64).mean(0) for i in range(G)])
    v64 = torch.stack([((yv[i].to(F64) - m64[i]) ** 2).mean(0) for i in range(G)])
    ratio = (m64.abs() / v64.sqrt()).min().item()

    def errs(mean, var):
        return (((mean - m64).abs() / v64.sqrt()).max().item(), ((var - v64).abs() / v64).max().item())

    em, ev = errs(mean, var)
    msg = f"{case} cap={cap}: min |mean|/std {ratio:.1f}, no pivot: mean err/std {em:.2e}, var rel {ev:.2e}"
    assert ratio >= 10, ratio
    if cap is None:
        assert em < 1e-4 and ev < 1e-4, msg
    if ops.cl_stat_pivot(Ho, Ho, B, K, Ci, Co, T):
        rm, rv = torch.zeros(Co, device="cuda"), torch.ones(Co, device="cuda")
        for _ in range(20):       # steps of training: the running mean tracks the batch means
            st.fill_(float("nan"))
            ops.cl_conv_fwd(x, wk, bias, y, st, N, B, Ci, H, H, Co, K, pad, pivot=rm)
            mean, var = _offc_stats(ops, st, G, R, Co, B * Ho * Ho, rm, rv, pivot=rm)
        em, ev = errs(mean, var)
        msg += f" | running-mean pivot: mean err/std {em:.2e}, var rel {ev:.2e}"
        # capped: ~6000-term fp32 lane sums remain (1.4e-4 measured, invstd within 7e-5)
        assert em < 1e-4 and ev < (1e-4 if cap is None else 3e-4), msg
    elif cap is not None:
        assert em < 1e-4 and ev < 1e-4, msg
    print(msg)


def test_conv1_routed_backward_bench_size(ops):
    """The audio conv1 training backward from the forward's routing codes (avd_cl_c1_apply_codes
    + avd_cl_c1_moments_codes + avd_cl_c1_codes_combine) at N = 7168: the pooled map of the
    codes-writing apply pass is bit-identical to the stored-y BN -> ReLU -> pool; the moments (M,
    Gram, S, sum dz) are within 1e-5 of float64 from the same routing; dW, dgamma, dbeta and the
    BN-backward coefficients are within 1e-5 / 1e-6 of the float64 formulas (sum dz y at the
    exact conv output w . x25 + b), and dW agrees with the recomputing moments pass (whose
    sum dz y uses the bf16-rounded y) to 1e-3."""
    N, B, H, C, K, pad = N_STUDENT, B_BENCH, 112, 8, 5, 2
    G = N // B
    Hp = H // 2
    g = torch.Generator(device="cuda").manual_seed(17)
    x = rnd(g, (N, H, H, 1), 0, 1, T)
    w = rnd(g, (C, 1, K, K)).to(T).float() / 5
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
    codes = torch.full((N * Hp * Hp,), -1, device="cuda", dtype=torch.int32)
    ops.c1_apply_codes(x, wk, bias, bn[2], bn[3], z1, codes, N, B, H, H)
    assert torch.equal(z0, z1)
    gz = rnd(g, (N, Hp, Hp, C), dtype=T)
    Rc, mc = ops.c1_codes_rows(N, B, H, H), ops.c1_codes_cols()
    assert Rc > 0 and mc == C * 25 + 625 + 25 + C
    parts = torch.full((Rc * G * mc,), float("nan"), device="cuda")
    ops.c1_moments_codes(x, gz, codes, parts, N, B, H, H)
    mom = torch.empty(G * mc, device="cuda")
    ops.sum_rows(parts, Rc, G * mc, mom)
    dw = torch.empty(C * 25, device="cuda")
    dg, db, dbi = (torch.empty(C, device="cuda") for _ in range(3))
    coef = torch.empty(G * C * 3, device="cuda")
    ops.c1_codes_combine(mom, wk, bias, gamma, bn[0], bn[1], B * H * H, dw, dg, db, dbi, coef, G)
    # float64 truth from the same routing (first max of relu(bn(y)) of the stored bf16 y)
    gram = torch.zeros(G, 25, 25, device="cuda", dtype=F64)
    sx = torch.zeros(G, 25, device="cuda", dtype=F64)
    mz = torch.zeros(G, C, 25, device="cuda", dtype=F64)
    s1 = torch.zeros(G, C, device="cuda", dtype=F64)
    sc, sf = bn[2].view(G, C).to(F64), bn[3].view(G, C).to(F64)
    for a, b in _chunks(N, H * H * 25 * 2):
        u = F.unfold(x[a:b].permute(0, 3, 1, 2).to(F64), K, padding=pad)     # [n, 25, H*H]
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
    assert grel(mh[:, :C * 25].view(G, C, 25), mz) < 1e-5
    assert grel(mh[:, C * 25:C * 25 + 625].view(G, 25, 25), gram) < 1e-5
    assert grel(mh[:, C * 25 + 625:C * 25 + 650], sx) < 1e-5
    assert grel(mh[:, C * 25 + 650:], s1) < 1e-5
    w64 = w.view(C, 25).to(T).to(F64)
    b64 = bias.to(F64)
    n = float(B * H * H)
    sy = torch.einsum("ct,gct->gc", w64, mz) + b64[None] * s1
    mu, iv, ga = bn[0].view(G, C).to(F64), bn[1].view(G, C).to(F64), gamma.to(F64)[None]
    s2 = (sy - mu * s1) * iv
    k1, kx, k0 = ga * iv, -ga * iv * iv * s2 / n, -ga * iv * s1 / n + ga * iv * iv * mu * s2 / n
    syg = torch.einsum("ct,gts->gcs", w64, gram) + b64[None, :, None] * sx[:, None, :]
    dw64 = (k1[..., None] * mz + kx[..., None] * syg + k0[..., None] * sx[:, None, :]).sum(0)
    k3 = coef.view(G, C, 3).to(F64)
    print("routed: dW vs f64", grel(dw, dw64), "coef", grel(k3, torch.stack([k1, kx, k0], -1)),
          "dgamma", grel(dg, s2.sum(0)), "dbeta", grel(db, s1.sum(0)))
    assert grel(k3, torch.stack([k1, kx, k0], -1)) < 1e-6
    assert grel(dg, s2.sum(0)) < 1e-5 and grel(db, s1.sum(0)) < 1e-5
    assert grel(dw, dw64) < 1e-5, grel(dw, dw64)
    # the recomputing moments pass (pass 4) on the same state
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
    d4 = torch.empty(C * 25, device="cuda")
    ops.cl_c1_recompute_combine(mom4, cf4, wk, bias, d4, G, C)
    print("routed vs recomputing moments pass: dW", grel(dw, d4), "dgamma", grel(dg, dg4))
    assert grel(dw, d4) < 3e-3 and grel(db, db4) < 1e-5


@pytest.mark.parametrize("N,B", [(24, 8), (320, 32), (N_STUDENT, B_BENCH)])
def test_image_conv1_routed_backward(ops, N, B):
    """The IMAGE conv1 (1->32, 5x5 pad 2 on 28x28) training backward from the forward's routing
    codes (avd_cl_c1r5_apply_codes + avd_cl_c1r5_moments_codes + avd_cl_c1r5_codes_combine): the
    codes-writing apply pass's pooled map is bit-identical to the stored-y BN -> ReLU -> pool; the
    moments (M, Gram, S, sum dz) are within 1e-5 of float64 from the same routing (first max of
    relu(bn(y)) of the stored bf16 y); dW, dgamma, dbeta and the coefficients within 1e-5 / 1e-6 of
    the float64 formulas; dW agrees with the recomputing moments pass (c1r3 pass 4) to 3e-3."""
    H, C, K, pad = 28, 32, 5, 2
    G = N // B
    Hp = H // 2
    g = torch.Generator(device="cuda").manual_seed(19)
    x = rnd(g, (N, H, H, 1), 0, 1, T)
    w = rnd(g, (C, 1, K, K)).to(T).float() / 5
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
    codes = torch.full((N * Hp * Hp * 8,), -1, device="cuda", dtype=torch.int16)
    ops.c1r5_apply_codes(x, wk, bias, bn[2], bn[3], z1, codes, N, B, H, H)
    assert torch.equal(z0, z1)
    z2 = torch.full_like(z0, float("nan"))
    ops.c1r5_apply_codes(x, wk, bias, bn[2], bn[3], z2, None, N, B, H, H)     # no codes: same map
    assert torch.equal(z0, z2)
    # the pixel-major statistics pass: per-group sums of the bf16 y within 1e-5 of float64
    Rs = ops.c1r5_stats_rows(N, B, H, H)
    sp = torch.full((C * G * Rs * 2,), float("nan"), device="cuda")
    ops.c1r5_stats(x, wk, bias, sp, N, B, H, H)
    s64 = sp.view(C, G, Rs, 2).to(F64).sum(2)
    y64 = y.to(F64).view(G, B * H * H, C)
    assert grel(s64[..., 0], y64.sum(1).T) < 1e-5 and grel(s64[..., 1], (y64 * y64).sum(1).T) < 1e-5
    bnp = torch.empty(4, G * C, device="cuda")
    ops.bn_finalize(sp, G, Rs, C, B * H * H, gamma, beta, bnp[0], bnp[1], bnp[2], bnp[3])
    assert grel(bnp, bn) < 1e-5
    gz = rnd(g, (N, Hp, Hp, C), dtype=T)
    Rc, mc = ops.c1r5_codes_rows(N, B, H, H), ops.c1r5_codes_cols()
    assert Rc > 0 and mc == C * 25 + 625 + 25 + C
    parts = torch.full((Rc * G * mc,), float("nan"), device="cuda")
    ops.c1r5_moments_codes(x, gz, codes, parts, N, B, H, H)
    mom = torch.empty(G * mc, device="cuda")
    ops.sum_rows(parts, Rc, G * mc, mom)
    dw = torch.empty(C * 25, device="cuda")
    dg, db, dbi = (torch.empty(C, device="cuda") for _ in range(3))
    coef = torch.empty(G * C * 3, device="cuda")
    ops.c1r5_codes_combine(mom, wk, bias, gamma, bn[0], bn[1], B * H * H, dw, dg, db, dbi, coef, G)
    gram = torch.zeros(G, 25, 25, device="cuda", dtype=F64)
    sx = torch.zeros(G, 25, device="cuda", dtype=F64)
    mz = torch.zeros(G, C, 25, device="cuda", dtype=F64)
    s1 = torch.zeros(G, C, device="cuda", dtype=F64)
    sc, sf = bn[2].view(G, C).to(F64), bn[3].view(G, C).to(F64)
    for a, b in _chunks(N, H * H * 25 * 2 * 8):
        u = F.unfold(x[a:b].permute(0, 3, 1, 2).to(F64), K, padding=pad)     # [n, 25, H*H]
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
    assert grel(mh[:, :C * 25].view(G, C, 25), mz) < 1e-5
    assert grel(mh[:, C * 25:C * 25 + 625].view(G, 25, 25), gram) < 1e-5
    assert grel(mh[:, C * 25 + 625:C * 25 + 650], sx) < 1e-5
    assert grel(mh[:, C * 25 + 650:], s1) < 1e-5
    w64 = w.view(C, 25).to(T).to(F64)
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
    dw4 = torch.empty(C * 25, device="cuda")
    ops.cl_c1_recompute_combine(mom4, cf4, wk, bias, dw4, G, C, K)
    # pass 4's sum dz y uses the bf16-rounded y: its dgamma sits ~2.5e-3 from the exact one
    assert grel(dw4, dw) < 3e-3 and grel(dg4, dg) < 6e-3 and grel(db4, db) < 1e-5
