"""TEST INFRASTRUCTURE ONLY -- the CPU checker for avd_augment_views (csrc/augment.hip).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.

Numpy restatement, in float32 with the kernel's operation order, of the per-pixel chain the
device applies to one (sample, view) record (layout: include/avdino.h AVD_AUG_*):
RandomResizedCrop (bilinear, get_data.py:123/128/139/166) -> TimeWarpWithStretch (|phase
vocoder| of a zero-phase spectrogram, get_data.py:29-58) -> Frequency/TimeMasking (148-149,
180-182) -> RandomRotation (124/129) -> RandomAffine (nearest, 125/130/152/185) -> RandomErasing
(131) -> GaussianNoise (21-27, 189) -> GroupedMasking (60-108, 157/191).

augment_one_seq restates the same stages for a chain in ANY order (transforms.Compose: each
stage reads its predecessor's whole output), which avd_augment_views_seq follows; for a chain in
the fixed order both restatements agree bit for bit (tests/test_augment_data.py).

Parity status: pinned to the reference's own code where that code is plain torch
(tests/test_augment_golden.py, fixtures by tests/golden/gen_augment_golden.py): the chain
structure MultiModalAugmentation builds (default and from the shipped config's best_augments),
__call__'s view/chain control flow, and the pixels of GroupedMasking and GaussianNoise ->
GroupedMasking given the reference's randperm / randn draws (bit-identical).  The stages that
call torchvision / torchaudio kernels (RandomResizedCrop, RandomRotation, RandomAffine,
RandomErasing, TimeStretch, Frequency/TimeMasking) stay "parity unpinned": those libraries are
not installed here; this oracle restates their published algorithms and pins the device
kernels to that maths (bit-exact outside the noise term, whose log/cos may differ by a few ulp).
"""
import numpy as np

f32 = np.float32


def _mix64(x):
    x = x ^ (x >> np.uint64(30))
    x = x * np.uint64(0xBF58476D1CE4E5B9)
    x = x ^ (x >> np.uint64(27))
    x = x * np.uint64(0x94D049BB133111EB)
    return x ^ (x >> np.uint64(31))


def gauss(seed, rec, pix):
    """csrc/augment.hip gauss2(): one Box-Muller draw over a counter hash of (seed, record,
    pixel pair pix >> 1) -- its cosine for the even pixel, its sine for the odd one."""
    pix = np.asarray(pix)
    with np.errstate(over="ignore"):
        key = (np.uint64(rec) << np.uint64(32)) | (pix >> 1).astype(np.uint64)
        r = _mix64(np.uint64(seed) ^ _mix64(key))
    u1 = ((r >> np.uint64(40)) + np.uint64(1)).astype(f32) * f32(5.9604644775390625e-8)
    u2 = ((r >> np.uint64(16)) & np.uint64(0xFFFFFF)).astype(f32) * f32(5.9604644775390625e-8)
    mag, ang = np.sqrt(f32(-2.0) * np.log(u1)), f32(6.2831855) * u2
    return np.where((pix & 1) == 0, mag * np.cos(ang), mag * np.sin(ang)).astype(f32)


def _affine_nearest(m, x, y, H, W):
    cx, cy = f32((W - 1) * 0.5), f32((H - 1) * 0.5)
    dx, dy = x.astype(f32) - cx, y.astype(f32) - cy
    m = m.astype(f32)
    sx = ((m[0] * dx + m[1] * dy) + m[2]) + cx
    sy = ((m[3] * dx + m[4] * dy) + m[5]) + cy
    rx, ry = np.rint(sx), np.rint(sy)
    ok = (rx >= 0) & (rx <= W - 1) & (ry >= 0) & (ry <= H - 1)
    return ok, np.where(ok, rx, 0).astype(np.int64), np.where(ok, ry, 0).astype(np.int64)


def _crop_sample(img, rec, r, c):
    H, W = img.shape
    if not (int(rec[23]) & 1):
        return img[r, c]
    top, left, ch, cw = (int(v) for v in rec[0:4])
    sh, sw = f32(ch) / f32(H), f32(cw) / f32(W)
    sy = (r.astype(f32) + f32(0.5)) * sh - f32(0.5)
    sx = (c.astype(f32) + f32(0.5)) * sw - f32(0.5)
    sy, sx = np.maximum(sy, f32(0)), np.maximum(sx, f32(0))
    y0, x0 = sy.astype(np.int64), sx.astype(np.int64)
    y1, x1 = np.minimum(y0 + 1, ch - 1), np.minimum(x0 + 1, cw - 1)
    ly, lx = sy - y0.astype(f32), sx - x0.astype(f32)
    hy, hx = f32(1) - ly, f32(1) - lx
    p00, p01 = img[top + y0, left + x0], img[top + y0, left + x1]
    p10, p11 = img[top + y1, left + x0], img[top + y1, left + x1]
    return hy * (hx * p00 + lx * p01) + ly * (hx * p10 + lx * p11)


def augment_one(img, rec, gm, seed, rid, group=4):
    """One output view [H, W] f32 from the normalised source img [H, W] f32 and its record."""
    H, W = img.shape
    img = img.astype(f32)
    y, x = np.meshgrid(np.arange(H), np.arange(W), indexing="ij")
    flags = int(rec[23])
    qx, qy, ok = x.copy(), y.copy(), np.ones((H, W), bool)
    if flags & 2:
        o, qx, qy = _affine_nearest(rec[4:10], qx, qy, H, W)
        ok &= o
    if flags & 4:
        o, qx2, qy2 = _affine_nearest(rec[10:16], qx, qy, H, W)
        ok &= o
        qx, qy = np.where(ok, qx2, 0), np.where(ok, qy2, 0)
    qx, qy = np.where(ok, qx, 0), np.where(ok, qy, 0)
    f0, f1, t0, t1 = (int(v) for v in rec[17:21])
    ok &= ~((qy >= f0) & (qy < f1)) & ~((qx >= t0) & (qx < t1))
    if flags & 8:
        t = qx.astype(f32) * f32(rec[16])
        inr = t < f32(W)
        tt = np.where(inr, t, f32(0))
        i0 = tt.astype(np.int64)
        a = tt - i0.astype(f32)
        s0 = np.abs(_crop_sample(img, rec, qy, i0))
        has1 = i0 + 1 < W
        s1 = np.where(has1, np.abs(_crop_sample(img, rec, qy, np.minimum(i0 + 1, W - 1))), f32(0))
        v = a * s1 + (f32(1) - a) * s0
        val = np.where(ok & inr, v, f32(0))
    else:
        val = np.where(ok, _crop_sample(img, rec, qy, qx), f32(0))
    et, el, eh, ew = (int(v) for v in rec[24:28])
    if eh > 0:
        val = np.where((y >= et) & (y < et + eh) & (x >= el) & (x < el + ew), f32(0), val)
    std = f32(rec[21])
    if std != 0:
        pix = (y * W + x).reshape(-1)
        val = val + gauss(seed, rid, pix).reshape(H, W) * std
    row = int(rec[22])
    if gm is not None and row >= 0:
        g = (y // group) * (W // group) + x // group
        bit = (gm[row][g >> 5].astype(np.uint32) >> (g & 31).astype(np.uint32)) & 1
        val = np.where(bit == 1, val * f32(0), val)
    return val.astype(f32)


# stage kinds (avd_augment_records numbering, avdino/augment.py _SK)
K_CROP, K_TWARP, K_FMASK, K_TMASK, K_ROT, K_AFF, K_ERASE, K_NOISE, K_GMASK = range(9)


def augment_one_seq(img, rec, gm, seed, rid, kinds, group=4, noise=None):
    """One view through a chain in ANY order, one transform at a time over the whole image --
    transforms.Compose semantics (get_data.py:134-231: each module reads its predecessor's
    output), the restatement avd_augment_views_seq follows.  ``noise`` [H, W] replaces the
    counter-hash normals (tests inject the reference's own torch.randn_like draws)."""
    H, W = img.shape
    cur = img.astype(f32).copy()
    y, x = np.meshgrid(np.arange(H), np.arange(W), indexing="ij")
    flags = int(rec[23])
    for k in kinds:
        if k == K_CROP and flags & 1:
            cur = _crop_sample(cur, rec, y, x).astype(f32)
        elif k == K_TWARP and flags & 8:
            # |phase_vocoder| of a zero-phase spectrogram (get_data.py:42-58)
            t = x.astype(f32) * f32(rec[16])
            inr = t < f32(W)
            tt = np.where(inr, t, f32(0))
            i0 = tt.astype(np.int64)
            a = tt - i0.astype(f32)
            s0 = np.abs(cur[y, i0])
            s1 = np.where(i0 + 1 < W, np.abs(cur[y, np.minimum(i0 + 1, W - 1)]), f32(0))
            cur = np.where(inr, a * s1 + (f32(1) - a) * s0, f32(0)).astype(f32)
        elif k in (K_ROT, K_AFF) and flags & (4 if k == K_ROT else 2):
            m = rec[10:16] if k == K_ROT else rec[4:10]
            ok, qx, qy = _affine_nearest(m, x, y, H, W)
            cur = np.where(ok, cur[qy, qx], f32(0)).astype(f32)
        elif k == K_FMASK and rec[18] > rec[17]:
            cur = np.where((y >= int(rec[17])) & (y < int(rec[18])), f32(0), cur)
        elif k == K_TMASK and rec[20] > rec[19]:
            cur = np.where((x >= int(rec[19])) & (x < int(rec[20])), f32(0), cur)
        elif k == K_ERASE and rec[26] > 0:
            et, el, eh, ew = (int(v) for v in rec[24:28])
            cur = np.where((y >= et) & (y < et + eh) & (x >= el) & (x < el + ew), f32(0), cur)
        elif k == K_NOISE and rec[21] != 0:
            # GaussianNoise.forward: x + randn_like(x) * std (get_data.py:26-27)
            g = (gauss(seed, rid, (y * W + x).reshape(-1)).reshape(H, W) if noise is None
                 else np.asarray(noise, f32))
            cur = (cur + g * f32(rec[21])).astype(f32)
        elif k == K_GMASK and gm is not None and rec[22] >= 0:
            # GroupedMasking.forward: spectrogram * mask over 4x4 groups (get_data.py:98-106)
            row = int(rec[22])
            gi = (y // group) * (W // group) + x // group
            bit = (gm[row][gi >> 5].astype(np.uint32) >> (gi & 31).astype(np.uint32)) & 1
            cur = np.where(bit == 1, cur * f32(0), cur)
    return cur.astype(f32)


def augment_views(src_u8, idx, lut, rec, gm, V, H, W, seed, order=0, group=4, kinds=None):
    """All records: out [B, V, H, W] (order 0) or [V, B, H, W] (order 1).  kinds: the chain's
    stage order (augment_one_seq) instead of the fixed gather order (augment_one)."""
    B = len(idx)
    out = np.zeros((B, V, H, W) if order == 0 else (V, B, H, W), f32)
    lut = np.asarray(lut, f32)
    for b in range(B):
        img = lut[src_u8[idx[b]]].reshape(H, W)
        for v in range(V):
            rid = b * V + v
            o = (augment_one(img, rec[rid], gm, seed, rid, group) if kinds is None else
                 augment_one_seq(img, rec[rid], gm, seed, rid, kinds, group))
            if order == 0:
                out[b, v] = o
            else:
                out[v, b] = o
    return out


def normalise_lut(kind, mean=0.0, std=1.0):
    """The dataset's per-byte normalisation (BaseAVMNISTDataset._process_image_audio,
    get_data.py:464-467): image u/255, audio (u/255 - mean)/std, float64 then float32."""
    u = np.arange(256, dtype=np.float64)
    v = u / 255.0 if kind == "image" else (u / 255.0 - mean) / std
    return v.astype(f32)
