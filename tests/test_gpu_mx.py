"""Block-scaled fp8 (MX) conv kernels of config 5's fp8 conv path (conv_ws8.hip,
avd_mx_conv_fwd / avd_mx_conv_dgrad) against float64 on the same inputs.

* Exact data: inputs are integers in [-8, 8] and weights integers x 2^-5, so every operand is
  an e4m3 value after the kernels' power-of-two scaling and every f32 accumulation is exact:
  y / dX must equal bf16(float64 conv) BIT FOR BIT -- this pins the operand layout (lane ->
  32 consecutive k), the tap / channel indexing of the staged strip, the per-strip scale, the
  per-block weight scales and the flipped input-gradient weights, at test size with a capped
  grid (every block walks several strips) and uncapped.  The forward's BatchNorm partial sums
  equal the float64 sums of the stored y.
* The weight gradient (avd_mx_conv_wgrad, K = output pixels): exact data -> the slab sum equals
  float64 dW bit for bit.
* Random data: the error against float64 of the unquantised operands is the e4m3 rounding's
  (rel-L2 < 0.06; 3 mantissa bits give ~3.6 % rms per operand)."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

# forward conv (Cin, Cout, K, pad, H): audio conv2-4, image conv2; their input gradients
LAYERS = [(8, 16, 5, 2, 56), (16, 32, 5, 2, 28), (32, 64, 5, 2, 14), (32, 64, 5, 0, 14)]


def _bf(t):
    return t.to(torch.bfloat16)


def _ref_fwd(x, w, b, pad):
    xd = x.double().permute(0, 3, 1, 2)
    y = torch.nn.functional.conv2d(xd, w.double(), b.double(), padding=pad)
    return y.permute(0, 2, 3, 1).contiguous()


def _ref_dgrad(dy, w, pad):
    d = dy.double().permute(0, 3, 1, 2)
    dx = torch.nn.functional.conv_transpose2d(d, w.double(), padding=pad)
    return dx.permute(0, 2, 3, 1).contiguous()


def _weights(w, dgrad):
    from avdino import ops
    Co, Ci, K, _ = w.shape
    wq = torch.empty(ops.mx_weight_bytes(Co, Ci, K, dgrad), dtype=torch.uint8, device="cuda")
    wsc = torch.empty(ops.mx_scale_bytes(Co, Ci, K, dgrad), dtype=torch.uint8, device="cuda")
    ops.mx_weight_layout(w, wq, wsc, dgrad)
    return wq, wsc


@pytest.fixture(params=[None, "5"], ids=["grid", "capped"])
def capped(request, avd_opts):
    if request.param:
        avd_opts(grid_cap=int(request.param))
    return request.param


@pytest.mark.parametrize("layer", LAYERS, ids=[f"{l[0]}to{l[1]}@{l[4]}p{l[3]}" for l in LAYERS])
def test_mx_conv_exact_data(layer, capped):
    from avdino import ops
    Cin, Cout, K, pad, H = layer
    Ho = H + 2 * pad - K + 1
    G, B = 2, 4
    N = G * B
    g = torch.Generator().manual_seed(Cin * 100 + H)
    x = _bf(torch.randint(-8, 9, (N, H, H, Cin), generator=g).float()).cuda()
    w = (torch.randint(-8, 9, (Cout, Cin, K, K), generator=g).float() * 2.0 ** -5).cuda()
    b = (torch.randint(-4, 5, (Cout,), generator=g).float() * 0.125).cuda()
    wq, wsc = _weights(w, 0)
    y = torch.empty(N, Ho, Ho, Cout, dtype=torch.bfloat16, device="cuda")
    R = ops.mx_stat_rows(H, B, K, Cin, Cout, pad)
    assert R > 0
    stats = torch.full((Cout * G * R * 2,), float("nan"), device="cuda")
    ops.mx_conv_fwd(x, wq, wsc, b, y, stats, N, B, Cin, H, H, Cout, K, pad)
    ref = _ref_fwd(x.float(), w, b, pad)
    assert torch.equal(y, _bf(ref.float())), (y.float() - ref.float()).abs().max()
    st = stats.view(Cout, G, R, 2).double().sum(2).cpu()
    yd = y.double().view(G, B * Ho * Ho, Cout).cpu()
    np.testing.assert_allclose(st[..., 0].T.numpy(), yd.sum(1).numpy(), rtol=1e-6, atol=1e-3)
    np.testing.assert_allclose(st[..., 1].T.numpy(), (yd ** 2).sum(1).numpy(), rtol=1e-6, atol=1e-3)
    # input gradient: dX of the same conv from an integer dY
    dy = _bf(torch.randint(-8, 9, (N, Ho, Ho, Cout), generator=g).float()).cuda()
    wqd, wscd = _weights(w, 1)
    dx = torch.empty(N, H, H, Cin, dtype=torch.bfloat16, device="cuda")
    ops.mx_conv_dgrad(dy, wqd, wscd, dx, N, Cin, H, H, Cout, K, pad)
    dref = _ref_dgrad(dy.float(), w, pad)
    assert torch.equal(dx, _bf(dref.float())), (dx.float() - dref.float()).abs().max()


@pytest.mark.parametrize("layer", LAYERS, ids=[f"{l[0]}to{l[1]}@{l[4]}p{l[3]}" for l in LAYERS])
def test_mx_conv_random_data_error_is_e4m3_rounding(layer):
    from avdino import ops
    Cin, Cout, K, pad, H = layer
    Ho = H + 2 * pad - K + 1
    N = 8
    g = torch.Generator().manual_seed(7 + Cin)
    x = _bf(torch.randn(N, H, H, Cin, generator=g) * 3.0).cuda()
    w = (torch.randn(Cout, Cin, K, K, generator=g) * 0.05).cuda()
    b = torch.zeros(Cout, device="cuda")
    wq, wsc = _weights(w, 0)
    y = torch.empty(N, Ho, Ho, Cout, dtype=torch.bfloat16, device="cuda")
    ops.mx_conv_fwd(x, wq, wsc, b, y, None, N, N, Cin, H, H, Cout, K, pad)
    ref = _ref_fwd(x.float(), w, b, pad)
    err = ((y.double() - ref).norm() / ref.norm()).item()
    assert 0.005 < err < 0.06, err
    dy = _bf(torch.randn(N, Ho, Ho, Cout, generator=g) * 1e-4).cuda()   # gradient-sized values
    wqd, wscd = _weights(w, 1)
    dx = torch.empty(N, H, H, Cin, dtype=torch.bfloat16, device="cuda")
    ops.mx_conv_dgrad(dy, wqd, wscd, dx, N, Cin, H, H, Cout, K, pad)
    dref = _ref_dgrad(dy.float(), w, pad)
    derr = ((dx.double() - dref).norm() / dref.norm()).item()
    assert 0.005 < derr < 0.06, derr


def _ref_wgrad(x, dy, w_shape, pad):
    return torch.nn.grad.conv2d_weight(x.double().permute(0, 3, 1, 2), w_shape,
                                       dy.double().permute(0, 3, 1, 2), padding=pad)


def _wgrad(x, dy, N, Cin, H, Cout, K, pad):
    from avdino import ops
    nch = ops.mx_wgrad_chunks(N, Cin, H, Cout, K, pad)
    assert nch > 0
    parts = torch.full((nch * Cout * Cin * K * K,), float("nan"), device="cuda")
    ops.mx_conv_wgrad(x, dy, parts, N, Cin, H, H, Cout, K, pad)
    return parts.view(nch, Cout, Cin, K, K).double().sum(0)


@pytest.mark.parametrize("layer", LAYERS, ids=[f"{l[0]}to{l[1]}@{l[4]}p{l[3]}" for l in LAYERS])
def test_mx_wgrad_exact_data(layer, capped):
    Cin, Cout, K, pad, H = layer
    Ho = H + 2 * pad - K + 1
    N = 6
    g = torch.Generator().manual_seed(Cout * 10 + H)
    x = _bf(torch.randint(-8, 9, (N, H, H, Cin), generator=g).float()).cuda()
    dy = _bf(torch.randint(-8, 9, (N, Ho, Ho, Cout), generator=g).float()).cuda()
    dw = _wgrad(x, dy, N, Cin, H, Cout, K, pad)
    ref = _ref_wgrad(x.float(), dy.float(), (Cout, Cin, K, K), pad)
    assert torch.equal(dw, ref), (dw - ref).abs().max()


@pytest.mark.parametrize("layer", LAYERS, ids=[f"{l[0]}to{l[1]}@{l[4]}p{l[3]}" for l in LAYERS])
def test_mx_wgrad_random_data_error_is_e4m3_rounding(layer):
    Cin, Cout, K, pad, H = layer
    Ho = H + 2 * pad - K + 1
    N = 8
    g = torch.Generator().manual_seed(70 + Cin)
    x = _bf(torch.randn(N, H, H, Cin, generator=g).abs()).cuda()        # post-ReLU/pool-like
    dy = _bf(torch.randn(N, Ho, Ho, Cout, generator=g) * 1e-5).cuda()   # gradient-sized
    dw = _wgrad(x, dy, N, Cin, H, Cout, K, pad)
    ref = _ref_wgrad(x.float(), dy.float(), (Cout, Cin, K, K), pad)
    err = ((dw - ref).norm() / ref.norm()).item()
    assert 0.002 < err < 0.06, err


# ------------------------------------------------------------------ config 5 at its size
N5, B5 = 7 * 4096, 4096          # config 5: B = 4096 per GPU, 2 global + 4 local views + originals


def _pm1(shape, gen):
    """Random {-1, 0, 1} bf16 operands on the device: exact in e4m3 under any power-of-two
    scale, and every partial sum of their products is an integer far below 2^24 (a random
    walk over <= 9e7 terms), so the MX kernels' f32 accumulation is exact at any N."""
    return (torch.randint(-1, 2, shape, generator=gen, device="cuda", dtype=torch.int8)).to(torch.bfloat16)


def _ref_conv64(x, w, b, pad):
    """NHWC float64 conv of a few samples (tap loop of f64 matmuls)."""
    N, H, W, Ci = x.shape
    Co, _, K, _ = w.shape
    Ho = H + 2 * pad - K + 1
    xp = torch.nn.functional.pad(x.double(), (0, 0, pad, pad, pad, pad))
    y = torch.zeros(N, Ho, Ho, Co, dtype=torch.float64, device="cuda")
    wd = w.double()
    for i in range(K):
        for j in range(K):
            y += xp[:, i:i + Ho, j:j + Ho, :] @ wd[:, :, i, j].T
    return y if b is None else y + b.double()


def _ref_wgrad64(x, dy, K, pad, per=1024):
    """dW[o, c, i, j] = sum dy[n, h, w, o] x_pad[n, h + i, w + j, c] in float64 over the whole
    batch: per tap a batched f64 matmul over pixel blocks, summed (exact for integer data)."""
    N, H, W, Ci = x.shape
    _, Ho, _, Co = dy.shape
    dw = torch.zeros(Co, Ci, K, K, dtype=torch.float64, device="cuda")
    for a in range(0, N, per):
        xp = torch.nn.functional.pad(x[a:a + per].double(), (0, 0, pad, pad, pad, pad))
        n = xp.shape[0]
        d = dy[a:a + per].double().reshape(n, Ho * Ho, Co).transpose(1, 2)        # [n, Co, pix]
        for i in range(K):
            for j in range(K):
                xs = xp[:, i:i + Ho, j:j + Ho, :].reshape(n, Ho * Ho, Ci)        # [n, pix, Ci]
                dw[:, :, i, j] += torch.bmm(d, xs).sum(0)
    return dw


@pytest.mark.parametrize("layer", LAYERS, ids=[f"{l[0]}to{l[1]}@{l[4]}p{l[3]}" for l in LAYERS])
def test_mx_kernels_config5_size(layer, capsys):
    """The three MX kernels at config 5's N = 28672 (B = 4096, 7 BN groups), every persistent
    block walking many strips, against float64 of the same operands:
    {-1, 0, 1} activations / gradients and integer x 2^-5 weights are exact e4m3 values and
    every f32 accumulation is exact, so
      * the forward map equals bf16(float64 conv) bit for bit on 56 sampled samples spread over
        all groups (first / last of each group included), and the BN partial sums of every
        (group, channel) equal float64 sums of the stored map (1e-5 of the sum of |y| / of y^2: f32 running sums over
        B * Ho^2 = 1.3e7 / 3.2e6 / 8e5 / 4e5 pixels);
      * the input gradient equals bf16(float64) bit for bit on the same samples;
      * the weight gradient (slab sum in float64) equals the float64 dW over all 28672
        samples bit for bit."""
    from avdino import ops
    Cin, Cout, K, pad, H = layer
    Ho = H + 2 * pad - K + 1
    N, B = N5, B5
    G = N // B
    gen = torch.Generator(device="cuda").manual_seed(5000 + Cin * 10 + pad)
    assert ops.mx_conv_serves(Cin, H, Cout, K, pad, 0, N, B) and ops.mx_conv_serves(Cin, H, Cout, K, pad, 1, N)
    x = _pm1((N, H, H, Cin), gen)
    w = torch.randint(-8, 9, (Cout, Cin, K, K), generator=gen, device="cuda").float() * 2.0 ** -5
    b = torch.randint(-4, 5, (Cout,), generator=gen, device="cuda").float() * 0.125
    samp = sorted({s for gi in range(G) for s in (gi * B, gi * B + B - 1)} |
                  set(torch.randint(0, N, (42,), generator=gen, device="cuda").tolist()))
    sidx = torch.tensor(samp, device="cuda")
    # forward + BN partial sums
    wq, wsc = _weights(w, 0)
    y = torch.empty(N, Ho, Ho, Cout, dtype=torch.bfloat16, device="cuda")
    R = ops.mx_stat_rows(H, B, K, Cin, Cout, pad)
    stats = torch.full((Cout * G * R * 2,), float("nan"), device="cuda")
    ops.mx_conv_fwd(x, wq, wsc, b, y, stats, N, B, Cin, H, H, Cout, K, pad)
    ref = _ref_conv64(x[sidx], w, b, pad)
    ys = y[sidx]
    assert torch.equal(ys, ref.to(torch.bfloat16)), (ys.double() - ref).abs().max()
    st = stats.view(Cout, G, R, 2).double().sum(2)
    yd = torch.stack([y[gi * B:(gi + 1) * B].double().reshape(-1, Cout).sum(0) for gi in range(G)])
    y2 = torch.stack([(y[gi * B:(gi + 1) * B].double().reshape(-1, Cout) ** 2).sum(0) for gi in range(G)])
    ya = torch.stack([y[gi * B:(gi + 1) * B].double().reshape(-1, Cout).abs().sum(0) for gi in range(G)])
    e1 = ((st[..., 0].T - yd).abs() / ya).max().item()     # relative to the sum of |y|
    e2 = ((st[..., 1].T - y2).abs() / y2).max().item()
    del y
    # input gradient
    dy = _pm1((N, Ho, Ho, Cout), gen)
    wqd, wscd = _weights(w, 1)
    dx = torch.empty(N, H, H, Cin, dtype=torch.bfloat16, device="cuda")
    ops.mx_conv_dgrad(dy, wqd, wscd, dx, N, Cin, H, H, Cout, K, pad)
    w2 = w.flip(2, 3).transpose(0, 1).contiguous()
    dref = _ref_conv64(dy[sidx], w2, None, K - 1 - pad)
    assert torch.equal(dx[sidx], dref.to(torch.bfloat16)), (dx[sidx].double() - dref).abs().max()
    del dx
    # weight gradient over the whole batch
    dw = _wgrad(x, dy, N, Cin, H, Cout, K, pad)
    dwr = _ref_wgrad64(x, dy, K, pad)
    with capsys.disabled():
        print(f"\nMX {Cin}->{Cout}@{H} N={N}: BN sums rel {e1:.1e} / {e2:.1e}, dW max |.| "
              f"{dwr.abs().max().item():.0f}, max |dW - f64| {(dw - dwr).abs().max().item():.1e}")
    assert e1 < 1e-5 and e2 < 1e-5, (e1, e2)
    assert torch.equal(dw, dwr), (dw - dwr).abs().max()
