"""CPU restatement (numpy, float64) of the reference's multimodal-DINO training step,
with an explicit backward pass.

TEST INFRASTRUCTURE ONLY -- the checker, never the thing measured or shipped.
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use it.
Pinned against golden vectors produced by running the reference itself
(tests/golden/gen_golden.py -> tests/golden/*.npz; tests/test_oracle_golden.py).

Each function cites the reference code (paths relative to
/root/reference/AVMNIST_Experiments) whose math it restates.

Conventions: activations of a conv stack are [N, C, H, W] with N = G*B, rows
ordered group-major (group g owns rows g*B .. g*B+B-1).  Train-mode BatchNorm
statistics are taken per (group, channel) because the reference calls the
encoder once per view (models/dino.py:680-704), giving each view its own batch
statistics.
"""
import math

import numpy as np
from numpy.lib.stride_tricks import sliding_window_view
from scipy.special import erf

F64 = np.float64
BN_EPS = 1e-5
BN_MOMENTUM = 0.1
NORM_EPS = 1e-12


# --------------------------------------------------------------------------- conv
def conv2d_fwd(x, w, b, pad):
    """nn.Conv2d(stride 1) forward -- models/unimodal.py:113-176, models/dino.py:20-61."""
    k = w.shape[-1]
    xp = np.pad(x, ((0, 0), (0, 0), (pad, pad), (pad, pad)))
    win = sliding_window_view(xp, (k, k), axis=(2, 3))  # N,C,Ho,Wo,k,k
    y = np.einsum("nchwij,ocij->nohw", win, w, optimize=True) + b[None, :, None, None]
    return y, win


def conv2d_bwd(dy, win, w, x_shape, pad):
    k = w.shape[-1]
    dw = np.einsum("nohw,nchwij->ocij", dy, win, optimize=True)
    db = dy.sum(axis=(0, 2, 3))
    N, C, H, W = x_shape
    dwin = np.einsum("nohw,ocij->nchwij", dy, w, optimize=True)
    Ho, Wo = dy.shape[2], dy.shape[3]
    dxp = np.zeros((N, C, H + 2 * pad, W + 2 * pad), F64)
    for i in range(k):
        for j in range(k):
            dxp[:, :, i:i + Ho, j:j + Wo] += dwin[..., i, j]
    dx = dxp[:, :, pad:pad + H, pad:pad + W]
    return dx, dw, db


# --------------------------------------------------------------------------- batchnorm
def bn_train_fwd(x, gamma, beta, G, axes):
    """Train-mode BatchNorm (biased var for normalisation) per group.

    x: [G*B, C, ...]; statistics over the rows of each group and the spatial axes.
    Restates nn.BatchNorm2d/1d train mode (unimodal.py:114,130; dino.py:1245).
    """
    N = x.shape[0]
    B = N // G
    xs = x.reshape((G, B) + x.shape[1:])
    red = (1,) + tuple(a + 1 for a in axes)
    mean = xs.mean(axis=red, keepdims=True)
    var = ((xs - mean) ** 2).mean(axis=red, keepdims=True)
    invstd = 1.0 / np.sqrt(var + BN_EPS)
    xhat = (xs - mean) * invstd
    shape = (1, 1, -1) + (1,) * (x.ndim - 2)
    y = xhat * gamma.reshape(shape) + beta.reshape(shape)
    n = xs.size // (G * x.shape[1])
    cache = (xhat, invstd, gamma, G, red, shape, x.shape)
    stats = (mean.reshape(G, -1), var.reshape(G, -1), n)
    return y.reshape(x.shape), cache, stats


def bn_eval_fwd(x, gamma, beta, rm, rv):
    """nn.BatchNorm2d/1d in eval mode: running statistics, channel axis 1."""
    shape = (1, -1) + (1,) * (x.ndim - 2)
    return (x - rm.reshape(shape)) / np.sqrt(rv.reshape(shape) + BN_EPS) * gamma.reshape(shape) \
        + beta.reshape(shape)


def bn_train_bwd(dy, cache):
    xhat, invstd, gamma, G, red, shape, xshape = cache
    dys = dy.reshape(xhat.shape)
    n = xhat.size // (G * xhat.shape[2])
    dbeta = dys.sum(axis=red).sum(axis=0)
    dgamma = (dys * xhat).sum(axis=red).sum(axis=0)
    dxhat = dys * gamma.reshape(shape)
    s1 = dxhat.sum(axis=red, keepdims=True)
    s2 = (dxhat * xhat).sum(axis=red, keepdims=True)
    dx = invstd / n * (n * dxhat - s1 - xhat * s2)
    return dx.reshape(xshape), dgamma, dbeta


def bn_running_update(rm, rv, stats):
    """Sequential per-group running-stat update: group order = call order in the
    reference (views 0..V-1, then originals).  Unbiased variance, momentum 0.1."""
    mean, var, n = stats
    rm = rm.astype(F64).copy()
    rv = rv.astype(F64).copy()
    for g in range(mean.shape[0]):
        rm = (1 - BN_MOMENTUM) * rm + BN_MOMENTUM * mean[g]
        rv = (1 - BN_MOMENTUM) * rv + BN_MOMENTUM * var[g] * n / (n - 1)
    return rm, rv


# --------------------------------------------------------------------------- relu / maxpool
def maxpool2_fwd(x):
    """F.max_pool2d(x, 2) (floor mode); ties resolved to the first element in
    row-major window order, as ATen's CPU kernel does (scan with '>')."""
    N, C, H, W = x.shape
    Ho, Wo = H // 2, W // 2
    xc = x[:, :, :2 * Ho, :2 * Wo].reshape(N, C, Ho, 2, Wo, 2).transpose(0, 1, 2, 4, 3, 5)
    xc = xc.reshape(N, C, Ho, Wo, 4)
    arg = xc.argmax(axis=-1)
    y = np.take_along_axis(xc, arg[..., None], axis=-1)[..., 0]
    return y, (arg, x.shape)


def maxpool2_bwd(dy, cache):
    arg, xshape = cache
    N, C, H, W = xshape
    Ho, Wo = dy.shape[2], dy.shape[3]
    d = np.zeros((N, C, Ho, Wo, 4), F64)
    np.put_along_axis(d, arg[..., None], dy[..., None], axis=-1)
    d = d.reshape(N, C, Ho, Wo, 2, 2).transpose(0, 1, 2, 4, 3, 5).reshape(N, C, 2 * Ho, 2 * Wo)
    dx = np.zeros(xshape, F64)
    dx[:, :, :2 * Ho, :2 * Wo] = d
    return dx


# --------------------------------------------------------------------------- dense ops
def linear_fwd(x, w, b):
    return x @ w.T + b


def linear_bwd(dy, x, w):
    return dy @ w, dy.T @ x, dy.sum(axis=0)


def gelu_fwd(x):
    """nn.GELU() (erf form) -- ProjectionHead dino.py:1246."""
    return 0.5 * x * (1.0 + erf(x / math.sqrt(2.0)))


def gelu_bwd(dy, x):
    cdf = 0.5 * (1.0 + erf(x / math.sqrt(2.0)))
    pdf = np.exp(-0.5 * x * x) / math.sqrt(2.0 * math.pi)
    return dy * (cdf + x * pdf)


def l2norm_fwd(x):
    """F.normalize(x, p=2, dim=-1): x / max(||x||, 1e-12)."""
    n = np.sqrt((x * x).sum(axis=-1, keepdims=True))
    d = np.maximum(n, NORM_EPS)
    return x / d, (x, n, d)


def l2norm_bwd(dy, cache):
    x, n, d = cache
    y = x / d
    proj = (dy * y).sum(axis=-1, keepdims=True)
    dx = (dy - y * proj * (n > NORM_EPS)) / d
    return dx


def log_softmax(z):
    m = z.max(axis=-1, keepdims=True)
    return z - m - np.log(np.exp(z - m).sum(axis=-1, keepdims=True))


def softmax(z):
    return np.exp(log_softmax(z))


# --------------------------------------------------------------------------- encoders
class ConvStack:
    """[conv -> BN(train) -> ReLU -> maxpool2] x L, optional global average pool.

    CentralUnimodalImage/Audio (unimodal.py:127-153, 185-211) and the 3x3 CNNs
    (dino.py:18-73: the AdaptiveAvgPool2d(1) tail)."""

    def __init__(self, arch, prefix_fmt):
        self.arch = arch
        self.prefix_fmt = prefix_fmt  # callable(i) -> (conv_key, bn_key)

    def forward(self, P, x, G, eval_mode=False):
        """eval_mode: BatchNorm from the running statistics (nn.Module.eval()); forward only."""
        caches, stats = [], []
        h = x
        for i, (ci, co, k, pad) in enumerate(self.arch["convs"]):
            ck, bk = self.prefix_fmt(i)
            y, win = conv2d_fwd(h, P[ck + ".weight"], P[ck + ".bias"], pad)
            if eval_mode:
                z = bn_eval_fwd(y, P[bk + ".weight"], P[bk + ".bias"], P[bk + ".running_mean"],
                                P[bk + ".running_var"])
                h, _ = maxpool2_fwd(np.maximum(z, 0.0))
                continue
            z, bnc, st = bn_train_fwd(y, P[bk + ".weight"], P[bk + ".bias"], G, axes=(2, 3))
            r = np.maximum(z, 0.0)
            p, pc = maxpool2_fwd(r)
            caches.append((win, h.shape, pad, ck, bk, bnc, z, pc))
            stats.append((bk, st))
            h = p
        if self.arch["gap"]:
            feat = h.mean(axis=(2, 3))
            caches.append(("gap", h.shape))
        else:
            feat = h.reshape(h.shape[0], -1)
            caches.append(("flat", h.shape))
        return feat, (caches, stats)

    def backward(self, P, dfeat, cache, grads):
        caches, _ = cache
        kind, hshape = caches[-1]
        if kind == "gap":
            dh = np.broadcast_to(dfeat[:, :, None, None] / (hshape[2] * hshape[3]), hshape).copy()
        else:
            dh = dfeat.reshape(hshape)
        for i in reversed(range(len(self.arch["convs"]))):
            win, xshape, pad, ck, bk, bnc, z, pc = caches[i]
            dr = maxpool2_bwd(dh, pc)
            dz = dr * (z > 0)
            dy, dg, dbt = bn_train_bwd(dz, bnc)
            dx, dw, db = conv2d_bwd(dy, win, P[ck + ".weight"], xshape, pad)
            _acc(grads, ck + ".weight", dw)
            _acc(grads, ck + ".bias", db)
            _acc(grads, bk + ".weight", dg)
            _acc(grads, bk + ".bias", dbt)
            dh = dx
        return dh


def _acc(grads, k, v):
    if k in grads:
        grads[k] = grads[k] + v
    else:
        grads[k] = v


def lenet_stack(arch, prefix):
    return ConvStack(arch, lambda i: (f"{prefix}.conv{i + 1}", f"{prefix}.bn{i + 1}"))


def cnn3_stack(arch, prefix):
    return ConvStack(arch, lambda i: (f"{prefix}.{4 * i}", f"{prefix}.{4 * i + 1}"))


class Branch:
    """Conv stack followed by the Linear that maps its flattened output to E
    (CentralMultiModalEncoder image_encoder/audio_encoder, dino.py:459-468)."""

    def __init__(self, stack, lin_key):
        self.stack = stack
        self.lin = lin_key

    def forward(self, P, x, G, eval_mode=False):
        feat, sc = self.stack.forward(P, x, G, eval_mode)
        out = linear_fwd(feat, P[self.lin + ".weight"], P[self.lin + ".bias"])
        return out, (feat, sc)

    def backward(self, P, dout, cache, grads):
        feat, sc = cache
        dfeat, dw, db = linear_bwd(dout, feat, P[self.lin + ".weight"])
        _acc(grads, self.lin + ".weight", dw)
        _acc(grads, self.lin + ".bias", db)
        return self.stack.backward(P, dfeat, sc, grads)


class CentralMultiModal:
    """CentralMultiModalEncoder / SimpleMultiModalEncoder forward (SimpleMultiModalEncoder.forward,
    dino.py:229-234): cat(image_branch, audio_branch) -> Linear -> ReLU -> Dropout -> Linear.
    encoder "multi_central": CentralNet LeNets + Linear (dino.py:454-468); "multi_simple": the
    3x3 image_encoder / audio_encoder (dino.py:18-73, 214-227), whose Linear is Sequential index
    14 / 18."""

    def __init__(self, prefix, encoder="multi_central"):
        from .spec import CENTRAL_IMAGE, CENTRAL_AUDIO, CNN3_AUDIO, CNN3_IMAGE
        self.p = prefix
        if encoder == "multi_central":
            self.img = Branch(lenet_stack(CENTRAL_IMAGE, f"{prefix}.image_encoder.0"), f"{prefix}.image_encoder.1")
            self.aud = Branch(lenet_stack(CENTRAL_AUDIO, f"{prefix}.audio_encoder.0"), f"{prefix}.audio_encoder.1")
        elif encoder == "multi_simple":
            self.img = Branch(cnn3_stack(CNN3_IMAGE, f"{prefix}.image_encoder"), f"{prefix}.image_encoder.14")
            self.aud = Branch(cnn3_stack(CNN3_AUDIO, f"{prefix}.audio_encoder"), f"{prefix}.audio_encoder.18")
        else:
            raise ValueError(encoder)

    def forward(self, P, img, aud, G, drop_mask=None, eval_mode=False):
        fi, ci = self.img.forward(P, img, G, eval_mode)
        fa, ca = self.aud.forward(P, aud, G, eval_mode)
        cat = np.concatenate([fi, fa], axis=1)
        h = linear_fwd(cat, P[self.p + ".fusion.0.weight"], P[self.p + ".fusion.0.bias"])
        r = np.maximum(h, 0.0)
        if drop_mask is not None:
            r = r * drop_mask
        out = linear_fwd(r, P[self.p + ".fusion.3.weight"], P[self.p + ".fusion.3.bias"])
        return out, (ci, ca, cat, h, r, drop_mask)

    def backward(self, P, dout, cache, grads):
        ci, ca, cat, h, r, drop_mask = cache
        dr, dw, db = linear_bwd(dout, r, P[self.p + ".fusion.3.weight"])
        _acc(grads, self.p + ".fusion.3.weight", dw)
        _acc(grads, self.p + ".fusion.3.bias", db)
        if drop_mask is not None:
            dr = dr * drop_mask
        dh = dr * (h > 0)
        dcat, dw, db = linear_bwd(dh, cat, P[self.p + ".fusion.0.weight"])
        _acc(grads, self.p + ".fusion.0.weight", dw)
        _acc(grads, self.p + ".fusion.0.bias", db)
        E = dcat.shape[1] // 2
        self.img.backward(P, dcat[:, :E], ci, grads)
        self.aud.backward(P, dcat[:, E:], ca, grads)


class ProjHead:
    """ProjectionHead (dino.py:1240-1254): Linear -> BN1d(train) -> GELU -> Dropout -> Linear."""

    def __init__(self, prefix):
        self.p = prefix

    def forward(self, P, x, G=1, drop_mask=None):
        p = self.p
        h = linear_fwd(x, P[p + ".mlp.0.weight"], P[p + ".mlp.0.bias"])
        z, bnc, st = bn_train_fwd(h, P[p + ".mlp.1.weight"], P[p + ".mlp.1.bias"], G, axes=())
        a = gelu_fwd(z)
        if drop_mask is not None:
            a = a * drop_mask
        out = linear_fwd(a, P[p + ".mlp.4.weight"], P[p + ".mlp.4.bias"])
        return out, (x, h, bnc, z, a, drop_mask, st)

    def backward(self, P, dout, cache, grads):
        p = self.p
        x, h, bnc, z, a, drop_mask, _ = cache
        da, dw, db = linear_bwd(dout, a, P[p + ".mlp.4.weight"])
        _acc(grads, p + ".mlp.4.weight", dw)
        _acc(grads, p + ".mlp.4.bias", db)
        if drop_mask is not None:
            da = da * drop_mask
        dz = gelu_bwd(da, z)
        dh, dg, dbt = bn_train_bwd(dz, bnc)
        _acc(grads, p + ".mlp.1.weight", dg)
        _acc(grads, p + ".mlp.1.bias", dbt)
        dx, dw, db = linear_bwd(dh, x, P[p + ".mlp.0.weight"])
        _acc(grads, p + ".mlp.0.weight", dw)
        _acc(grads, p + ".mlp.0.bias", db)
        return dx


# --------------------------------------------------------------------------- losses
def dino_loss(s, t, tau_s, tau_t, center_teacher=False):
    """MultiModalDINOLightning.dino_loss (dino.py:822-854); with center_teacher=True
    the UniModalDINOLightning variant that subtracts the per-view batch mean of the
    normalised teacher (dino.py:1606-1617).  Returns (loss, d_loss/d_s)."""
    V, B, _ = s.shape
    T = t.shape[0]
    sn, sc = l2norm_fwd(s)
    tn, _ = l2norm_fwd(t)
    if center_teacher:
        tn = tn - tn.mean(axis=1, keepdims=True)
    pt = softmax(tn / tau_t)          # [T,B,K]
    ls = log_softmax(sn / tau_s)      # [V,B,K]
    # sum over all (student view, teacher view) pairs, each a batch mean, / (V*T)
    ptsum = pt.sum(axis=0)            # [B,K]
    loss = -(ptsum[None] * ls).sum() / (B * V * T)
    # d/d(ls) = -ptsum/(B V T); log-softmax backward: g - softmax * sum(g)
    g = np.broadcast_to(-ptsum[None] / (B * V * T), ls.shape)
    dz = g - np.exp(ls) * g.sum(axis=-1, keepdims=True)
    dsn = dz / tau_s
    ds = l2norm_bwd(dsn, sc)
    return loss, ds


def mse_loss(i, a):
    """MultiModalDINOWithMSELightning.mse_loss (dino.py:1193-1211)."""
    inn, ic = l2norm_fwd(i)
    an, ac = l2norm_fwd(a)
    d = inn - an
    loss = (d * d).mean()
    g = 2.0 * d / d.size
    return loss, l2norm_bwd(g, ic), l2norm_bwd(-g, ac)


def cross_entropy(logits, labels):
    """F.cross_entropy mean reduction; returns (loss, dlogits)."""
    n = logits.shape[0]
    ls = log_softmax(logits)
    loss = -ls[np.arange(n), labels].mean()
    d = np.exp(ls)
    d[np.arange(n), labels] -= 1.0
    return loss, d / n


def infonce_loss(i, a, temperature=0.07):
    """infoNCE_loss (dino.py:1091-1128; other_ssl/info_nce/info_nce.py:75-112)."""
    B = i.shape[0]
    inn, ic = l2norm_fwd(i)
    an, ac = l2norm_fwd(a)
    S = inn @ an.T / temperature
    lab = np.arange(B)
    l1, d1 = cross_entropy(S, lab)
    l2, d2 = cross_entropy(S.T, lab)
    dS = (d1 + d2.T) / 2.0
    loss = (l1 + l2) / 2.0
    dinn = dS @ an / temperature
    dan = dS.T @ inn / temperature
    return loss, l2norm_bwd(dinn, ic), l2norm_bwd(dan, ac)


def nt_xent_loss(reps, temperature=0.07):
    """MultiModalSimCLRLightning.nt_xent_loss (multimodal_simclr.py:74-89)."""
    N = reps.shape[0]
    B = N // 2
    rn, rc = l2norm_fwd(reps)
    S = rn @ rn.T / temperature
    np.fill_diagonal(S, -np.inf)
    lab = np.concatenate([np.arange(B) + B, np.arange(B)])
    loss, dS = cross_entropy(S, lab)
    np.fill_diagonal(dS, 0.0)
    drn = (dS + dS.T) @ rn / temperature
    return loss, l2norm_bwd(drn, rc)


# --------------------------------------------------------------------------- optimiser / EMA
def adam_step(p, g, m, v, step, lr, wd, b1=0.9, b2=0.999, eps=1e-8):
    """torch.optim.Adam (L2 weight decay added to the gradient), configure_optimizers
    dino.py:953-962."""
    g = g + wd * p
    m = b1 * m + (1 - b1) * g
    v = b2 * v + (1 - b2) * g * g
    bc1 = 1 - b1 ** step
    bc2 = 1 - b2 ** step
    denom = np.sqrt(v) / math.sqrt(bc2) + eps
    p = p - (lr / bc1) * m / denom
    return p, m, v


def adamw_step(p, g, m, v, step, lr, wd=0.01, b1=0.9, b2=0.999, eps=1e-8):
    """torch.optim.AdamW (decoupled weight decay, default wd 0.01): the epoch-end linear
    probe's optimiser (dino.py:898, 1678)."""
    p = p * (1 - lr * wd)
    m = b1 * m + (1 - b1) * g
    v = b2 * v + (1 - b2) * g * g
    denom = np.sqrt(v) / math.sqrt(1 - b2 ** step) + eps
    return p - (lr / (1 - b1 ** step)) * m / denom, m, v


def ema(teacher, student, m):
    """MultiModalDINO.update_teacher (dino.py:635-646)."""
    return m * teacher + (1 - m) * student


# --------------------------------------------------------------------------- full step
def _views_to_rows(v):
    """[B, V, 1, H, W] -> [V*B, 1, H, W] (view-major, matching torch.cat of the
    per-view features, dino.py:695)."""
    B, V = v.shape[:2]
    return np.ascontiguousarray(v.transpose(1, 0, 2, 3, 4).reshape(V * B, *v.shape[2:]))


def multimodal_step(P, batch, mode, hp, masks=None, aux_fn=None, encoder="multi_central"):
    """One MultiModalDINO* training step in the reference's order:
    forward -> losses -> EMA (pre-step student) -> backward -> Adam.

    P: dict key -> float64 ndarray (full state dict, incl. teacher / BN buffers / center).
    Returns dict with losses, outputs, grads (live student params), new state.
    masks: optional dropout masks (already scaled by 1/(1-p)) for the fusion of the
    student ('fusion_s' [V*B,E]), teacher ('fusion_t' [G*B,E]), heads ('fusion_o' [B,E])
    and the student projection ('proj_s' [V*B,512]); None = p 0.
    aux_fn: optional (zi, za) -> (aux loss, d zi, d za) replacing the mode's own head loss
    (multimodal_step_ddp's global-negative InfoNCE).
    """
    masks = masks or {}
    P = {k: np.asarray(v, F64) if np.asarray(v).dtype != np.int64 else np.asarray(v) for k, v in P.items()}
    g_img, g_aud, l_img, l_aud = batch["g_img"], batch["g_aud"], batch["l_img"], batch["l_aud"]
    B, G = g_img.shape[:2]
    L = l_img.shape[1]
    V = G + L
    img_v = np.concatenate([_views_to_rows(g_img), _views_to_rows(l_img)]).astype(F64)
    aud_v = np.concatenate([_views_to_rows(g_aud), _views_to_rows(l_aud)]).astype(F64)

    stu = CentralMultiModal("student", encoder)
    tea = CentralMultiModal("teacher", encoder)
    sproj, tproj = ProjHead("student_projection"), ProjHead("teacher_projection")

    # student: all views (each view its own BN group)
    s_feat, s_cache = stu.forward(P, img_v, aud_v, V, masks.get("fusion_s"))
    # teacher: global views, no grad, train mode (batch-stat BN)
    t_feat, t_cache = tea.forward(P, img_v[:G * B], aud_v[:G * B], G, masks.get("fusion_t"))
    s_proj, sp_cache = sproj.forward(P, s_feat, 1, masks.get("proj_s"))
    t_proj, tp_cache = tproj.forward(P, t_feat, 1)
    center = P["center"]
    t_c = t_proj - center
    new_center = center * hp["center_momentum"] + t_proj.mean(axis=0, keepdims=True) * (1 - hp["center_momentum"])
    s_out = s_proj.reshape(V, B, -1)
    t_out = t_c.reshape(G, B, -1)

    dino, ds = dino_loss(s_out, t_out, hp["tau_s"], hp["tau_t"])
    out = {"dino_loss": dino, "s_out": s_out, "t_out": t_out, "center_after": new_center}
    grads = {}
    bn_stats = []  # (bn key, stats) in call order
    bn_stats += [(k, st) for k, st in _stack_stats(s_cache)]
    bn_stats += [("student_projection.mlp.1", sp_cache[-1])]
    bn_stats += [(k, st) for k, st in _stack_stats(t_cache)]
    bn_stats += [("teacher_projection.mlp.1", tp_cache[-1])]

    aux = 0.0
    if mode in ("mse", "infonce", "semi_supervised"):
        img_o = batch["image"].astype(F64)
        aud_o = batch["audio"].astype(F64)
        fi, ci = stu.img.forward(P, img_o, 1)
        fa, ca = stu.aud.forward(P, aud_o, 1)
        hi = {"mse": "image_projection_head", "infonce": "image_projection_head",
              "semi_supervised": "image_classifier"}[mode]
        ha = hi.replace("image", "audio")
        hI, hA = ProjHead(hi), ProjHead(ha)
        zi, zic = hI.forward(P, fi)
        za, zac = hA.forward(P, fa)
        if aux_fn is not None:
            aux, dzi, dza = aux_fn(zi, za)
        elif mode == "mse":
            aux, dzi, dza = mse_loss(zi, za)
        elif mode == "infonce":
            aux, dzi, dza = infonce_loss(zi, za)
        else:
            li, dzi = cross_entropy(zi, batch["label"])
            la, dza = cross_entropy(za, batch["label"])
            aux = li + la
        out["f_img"], out["f_aud"] = zi, za
        bn_stats += [(k, st) for k, st in _branch_stats(ci)]
        bn_stats += [(k, st) for k, st in _branch_stats(ca)]
        bn_stats += [(hi + ".mlp.1", zic[-1]), (ha + ".mlp.1", zac[-1])]
        dfi = hI.backward(P, dzi, zic, grads)
        dfa = hA.backward(P, dza, zac, grads)
        stu.img.backward(P, dfi, ci, grads)
        stu.aud.backward(P, dfa, ca, grads)
    out["aux_loss"] = aux
    out["loss"] = dino + aux

    # backward of the DINO branch
    dsf = sproj.backward(P, ds.reshape(V * B, -1), sp_cache, grads)
    stu.backward(P, dsf, s_cache, grads)

    # new state: EMA uses the pre-step student (update_teacher precedes backward/step)
    new = dict(P)
    m = hp["momentum"]
    for k in P:
        if k.startswith("teacher") and not (k.endswith("running_mean") or k.endswith("running_var")
                                            or k.endswith("num_batches_tracked")):
            new[k] = ema(P[k], P["student" + k[len("teacher"):]], m)
    new["center"] = new_center
    # BN running stats, group order per call order
    for bk, st in bn_stats:
        rm, rv = bn_running_update(new[bk + ".running_mean"], new[bk + ".running_var"], st)
        new[bk + ".running_mean"], new[bk + ".running_var"] = rm, rv
        new[bk + ".num_batches_tracked"] = np.asarray(new[bk + ".num_batches_tracked"]) + st[0].shape[0]
    out["grads"] = grads
    out["state"] = new
    return out


def multimodal_step_ddp(P, batch, mode, hp, world, global_negatives=True):
    """The reference's DDP step over ``world`` ranks, simulated in one process (SURVEY 8(e)
    "parity for N ranks"): rank r owns batch rows r*B..(r+1)*B (DistributedSampler shards),
    runs the forward with its OWN BatchNorm statistics (no SyncBN), updates its own centre and
    running statistics, and the gradients are averaged (DDP all-reduce / world) before Adam;
    every rank starts from rank 0's buffers (broadcast_buffers).  InfoNCE with
    global_negatives: each rank's loss is the mean over ITS rows of the InfoNCE over the
    all-gathered batch, and its head gradient is the one the all-gather's adjoint delivers, so
    the averaged gradient is the single-device gradient of the global-batch InfoNCE.
    Returns per-rank step dicts and the averaged gradients."""
    Bt = batch["g_img"].shape[0]
    B = Bt // world
    shard = [{k: v[r * B:(r + 1) * B] for k, v in batch.items()} for r in range(world)]
    aux = [None] * world
    if mode == "infonce" and global_negatives and world > 1:
        zs = [multimodal_step(P, shard[r], mode, hp) for r in range(world)]
        Zi = np.concatenate([z["f_img"] for z in zs])
        Za = np.concatenate([z["f_aud"] for z in zs])
        _, dZi, dZa = infonce_loss(Zi, Za)
        inn, _ = l2norm_fwd(Zi)
        an, _ = l2norm_fwd(Za)
        S = inn @ an.T / 0.07
        lab = np.arange(Bt)
        ls1 = -log_softmax(S)[lab, lab]
        ls2 = -log_softmax(S.T)[lab, lab]
        for r in range(world):
            sl = slice(r * B, (r + 1) * B)
            lr_ = 0.5 * (ls1[sl].mean() + ls2[sl].mean())
            aux[r] = (lambda a, b, lr_=lr_, sl=sl: (lr_, world * dZi[sl], world * dZa[sl]))
    outs = [multimodal_step(P, shard[r], mode, hp, aux_fn=aux[r]) for r in range(world)]
    grads = {k: sum(o["grads"][k] for o in outs) / world for k in outs[0]["grads"]}
    return outs, grads


def _stack_stats(enc_cache):
    ci, ca = enc_cache[0], enc_cache[1]
    return list(_branch_stats(ci)) + list(_branch_stats(ca))


def _branch_stats(branch_cache):
    _feat, (_caches, stats) = branch_cache
    return stats


def adam_update_state(state, grads, opt, step, hp):
    """Apply Adam to every parameter with a gradient; opt holds (m, v) per key."""
    new = dict(state)
    for k, g in grads.items():
        m, v = opt.get(k, (np.zeros_like(g), np.zeros_like(g)))
        p, m, v = adam_step(state[k], g, m, v, step, hp["lr"], hp["wd"])
        new[k] = p
        opt[k] = (m, v)
    return new


def cosine_consistency_loss(emb):
    """UniModalDINOLightning._cosine_consistency_loss (dino.py:1575-1594): mean over view
    pairs i<j of batch-mean (1 - n_i . n_j)^2 with n = F.normalize(emb).  emb [V,B,D].
    Returns (loss, d loss / d emb)."""
    V, B, _ = emb.shape
    n, c = l2norm_fwd(emb)
    count = V * (V - 1) // 2
    if count == 0:
        return 0.0, np.zeros_like(emb)
    loss = 0.0
    dn = np.zeros_like(n)
    for i in range(V):
        for j in range(i + 1, V):
            sim = (n[i] * n[j]).sum(-1)
            loss += ((1 - sim) ** 2).mean()
            g = (-2.0 * (1 - sim) / (B * count))[:, None]
            dn[i] += g * n[j]
            dn[j] += g * n[i]
    return loss / count, l2norm_bwd(dn, c)


UNI_KINDS = {"image": "image_simple", "audio": "spectrogram_simple"}


def uni_encoder(kind, prefix):
    """Unimodal student/teacher encoders of UNIMODAL_MODEL_MAP (run_dino.py:542-550):
    image_simple = ImageEncoder (dino.py:483-499: image_encoder(512) + projection Linear(512,D)),
    spectrogram_simple = SpectrogramEncoder (502-513: audio_encoder(D)),
    spectrogram_central = SpectrogramEncoderCentral (515-523: CentralUnimodalAudio + Linear(3136,D)).
    Returns (forward, backward)."""
    from .spec import CNN3_IMAGE, CNN3_AUDIO, CENTRAL_AUDIO
    kind = UNI_KINDS.get(kind, kind)
    lin = None
    if kind == "image_simple":
        br = Branch(cnn3_stack(CNN3_IMAGE, f"{prefix}.encoder"), f"{prefix}.encoder.14")
        lin = f"{prefix}.projection.0"
    elif kind == "spectrogram_simple":
        br = Branch(cnn3_stack(CNN3_AUDIO, f"{prefix}.encoder"), f"{prefix}.encoder.18")
    elif kind == "spectrogram_central":
        br = Branch(lenet_stack(CENTRAL_AUDIO, f"{prefix}.encoder.0"), f"{prefix}.encoder.1")
    else:
        raise ValueError(kind)

    def fwd(P, x, G, eval_mode=False):
        f, c = br.forward(P, x, G, eval_mode)
        if lin is None:
            return f, (f, c)
        return linear_fwd(f, P[lin + ".weight"], P[lin + ".bias"]), (f, c)

    def bwd(P, dout, cache, grads):
        f, c = cache
        if lin is not None:
            dout, dw, db = linear_bwd(dout, f, P[lin + ".weight"])
            _acc(grads, lin + ".weight", dw)
            _acc(grads, lin + ".bias", db)
        return br.backward(P, dout, c, grads)

    return fwd, bwd


def unimodal_step(P, batch, hp, modality="image", cos_alpha=0.0, masks=None, encoder=None):
    """One UniModalDINO training step (UniModalDINO.forward dino.py:1319-1398,
    UniModalDINOLightning.dino_loss 1596-1635 + cosine consistency 1575-1594 when
    cos_alpha > 0, training_step 1637-1668): forward -> loss -> EMA -> backward.
    Views: g_* [B,G,1,H,W] (+ l_* [B,L,...]) of the chosen modality.  Returns loss, outputs,
    live-student grads, centre and the new state (EMA, centre, BN running stats)."""
    masks = masks or {}
    P = {k: np.asarray(v, F64) if np.asarray(v).dtype != np.int64 else np.asarray(v) for k, v in P.items()}
    key = "img" if UNI_KINDS.get(modality, modality) == "image_simple" else "aud"
    g = batch["g_" + key]
    B, G = g.shape[:2]
    l = batch.get("l_" + key)
    L = 0 if l is None else l.shape[1]
    V = G + L
    x = _views_to_rows(g).astype(F64)
    if L:
        x = np.concatenate([x, _views_to_rows(l).astype(F64)])
    kind = encoder or modality
    sf, sb = uni_encoder(kind, "student")
    tf, _ = uni_encoder(kind, "teacher")
    s_feat, s_cache = sf(P, x, V)
    t_feat, t_cache = tf(P, x[:G * B], G)
    sp, tp = ProjHead("student_projection"), ProjHead("teacher_projection")
    s_proj, spc = sp.forward(P, s_feat, 1, masks.get("proj_s"))
    t_proj, tpc = tp.forward(P, t_feat)
    t_c = t_proj - P["center"]
    s_out = s_proj.reshape(V, B, -1)
    t_out = t_c.reshape(G, B, -1)
    dino, ds = dino_loss(s_out, t_out, hp["tau_s"], hp["tau_t"], center_teacher=True)
    grads = {}
    dsf = sp.backward(P, ds.reshape(V * B, -1), spc, grads)
    cos = 0.0
    if cos_alpha > 0:
        cos, demb = cosine_consistency_loss(s_feat.reshape(V, B, -1))
        dsf = dsf + cos_alpha * demb.reshape(V * B, -1)
    sb(P, dsf, s_cache, grads)
    new_center = P["center"] * hp["center_momentum"] + t_proj.mean(axis=0, keepdims=True) * (1 - hp["center_momentum"])
    new = dict(P)
    m = hp["momentum"]
    for k in P:
        if k.startswith("teacher") and not (k.endswith("running_mean") or k.endswith("running_var")
                                            or k.endswith("num_batches_tracked")):
            new[k] = ema(P[k], P["student" + k[len("teacher"):]], m)
    new["center"] = new_center
    bn_stats = (list(_branch_stats(s_cache[1])) + [("student_projection.mlp.1", spc[-1])]
                + list(_branch_stats(t_cache[1])) + [("teacher_projection.mlp.1", tpc[-1])])
    for bk, st in bn_stats:
        rm, rv = bn_running_update(new[bk + ".running_mean"], new[bk + ".running_var"], st)
        new[bk + ".running_mean"], new[bk + ".running_var"] = rm, rv
        new[bk + ".num_batches_tracked"] = np.asarray(new[bk + ".num_batches_tracked"]) + st[0].shape[0]
    return {"loss": dino + cos_alpha * cos, "dino_loss": dino, "cos_loss": cos, "s_out": s_out,
            "t_out": t_out, "emb": s_feat.reshape(V, B, -1), "grads": grads,
            "center_after": new_center, "state": new}


def pretrain_dino(P, batches, epochs, lr=1e-4, hp=None, wd=0.01, modality="image"):
    """training_structures/dino_train.py:104-186 (BASELINE config 1's CPU path): AdamW over
    every parameter with a gradient (torch default weight_decay 0.01), and per batch
    forward -> dino_loss(tau_s 0.1, tau_t 0.04; the unimodal loss) -> backward -> AdamW.step ->
    update_teacher, i.e. the teacher EMA sees the POST-step student (the Lightning path EMAs
    before backward).  batches: per epoch, the same list of unimodal batch dicts.  Returns the
    per-step losses, per-epoch mean losses and the final state."""
    hp = dict(hp or {})
    hp.setdefault("tau_s", 0.1)
    hp.setdefault("tau_t", 0.04)
    P = {k: np.asarray(v, F64) if np.asarray(v).dtype != np.int64 else np.asarray(v) for k, v in P.items()}
    opt, t, losses, epoch_losses = {}, 0, [], []
    for _ in range(epochs):
        el = []
        for b in batches:
            r = unimodal_step(P, b, hp, modality, 0.0)
            new = r["state"]
            t += 1
            for k, g in r["grads"].items():
                m, v = opt.get(k, (np.zeros_like(g), np.zeros_like(g)))
                new[k], m, v = adamw_step(P[k], g, m, v, t, lr, wd)
                opt[k] = (m, v)
            for k in P:     # EMA after the optimizer step: old teacher, NEW student
                if k.startswith("teacher") and not k.endswith(("running_mean", "running_var",
                                                                "num_batches_tracked")):
                    new[k] = ema(P[k], new["student" + k[len("teacher"):]], hp["momentum"])
            P = new
            losses.append(r["loss"])
            el.append(r["loss"])
        epoch_losses.append(float(np.mean(el)))
    return {"step_losses": np.array(losses), "epoch_losses": np.array(epoch_losses), "state": P}


def unimodal_image_step(P, batch, hp):
    """UniModalDINO(ImageEncoder), 2 global / 0 local views, no cosine term (BASELINE config 1)."""
    return unimodal_step(P, batch, hp, "image", 0.0)


def simclr_step(P, batch, mode, temperature=0.07, shards=1):
    """MultiModalSimCLRModel.forward + nt_xent_loss (multimodal_simclr.py:22-47, 74-89)
    for a pinned modality mode (0 img/img, 1 aud/aud, 2 img/aud, 3 aud/img).

    shards > 1 restates the data-parallel run with GLOBAL negatives: the batch
    is split into `shards` rank-local batches, each encoded with its own BatchNorm statistics,
    NT-Xent is taken over the concatenated global [z1 of all shards; z2 of all shards], and
    the parameter gradient is the sum over shards (= DDP's average of per-rank local-mean
    losses).  bn_stats lists, per encoder call in call order, (bn key, stats) pairs."""
    from .spec import CNN3_IMAGE, CNN3_AUDIO
    P = {k: np.asarray(v, F64) if np.asarray(v).dtype != np.int64 else np.asarray(v) for k, v in P.items()}
    grads = {}
    stats = []

    def image_enc(x):
        e = Branch(cnn3_stack(CNN3_IMAGE, "image_encoder.encoder"), "image_encoder.encoder.14")
        f, c = e.forward(P, x, 1)
        o = linear_fwd(f, P["image_encoder.projection.0.weight"], P["image_encoder.projection.0.bias"])
        h = ProjHead("image_projection_head")
        z, hc = h.forward(P, o)
        stats.append(list(_branch_stats(c)) + [("image_projection_head.mlp.1", hc[-1])])

        def bwd(dz):
            do = h.backward(P, dz, hc, grads)
            df, dw, db = linear_bwd(do, f, P["image_encoder.projection.0.weight"])
            _acc(grads, "image_encoder.projection.0.weight", dw)
            _acc(grads, "image_encoder.projection.0.bias", db)
            e.backward(P, df, c, grads)
        return z, bwd

    def audio_enc(x):
        e = Branch(cnn3_stack(CNN3_AUDIO, "audio_encoder.encoder"), "audio_encoder.encoder.18")
        f, c = e.forward(P, x, 1)
        h = ProjHead("audio_projection_head")
        z, hc = h.forward(P, f)
        stats.append(list(_branch_stats(c)) + [("audio_projection_head.mlp.1", hc[-1])])

        def bwd(dz):
            do = h.backward(P, dz, hc, grads)
            e.backward(P, do, c, grads)
        return z, bwd

    f1 = image_enc if mode in (0, 2) else audio_enc
    f2 = image_enc if mode in (0, 3) else audio_enc
    Bt = batch["img1"].shape[0]
    B = Bt // shards
    z1s, z2s, bw = [], [], []
    for r in range(shards):
        sl = slice(r * B, (r + 1) * B)
        i1, s1 = batch["img1"][sl].astype(F64), batch["spec1"][sl].astype(F64)
        i2, s2 = batch["img2"][sl].astype(F64), batch["spec2"][sl].astype(F64)
        z1, b1 = f1(i1 if f1 is image_enc else s1)
        z2, b2 = f2(i2 if f2 is image_enc else s2)
        z1s.append(z1)
        z2s.append(z2)
        bw.append((b1, b2))
    Z1, Z2 = np.concatenate(z1s), np.concatenate(z2s)
    loss, dr = nt_xent_loss(np.concatenate([Z1, Z2]), temperature)
    # per-shard local-mean losses averaged by DDP == the global mean: dr is already global
    for r, (b1, b2) in enumerate(bw):
        b1(dr[r * B:(r + 1) * B])
        b2(dr[Bt + r * B:Bt + (r + 1) * B])
    return {"loss": loss, "z1": Z1, "z2": Z2, "grads": grads, "bn_stats": stats}


class _ProbeModel:
    """DownstreamClassifier (models/dino.py:1764-1814) over a deep copy of the student:
    ``features(b, eval_mode)`` runs the copy (train mode updates its BN running statistics),
    the classifier is Linear(D,128)-ReLU-Linear(128,10) trained with AdamW."""

    def __init__(self, P, kind, cls):
        self.P = {k: np.asarray(v, F64) if np.asarray(v).dtype != np.int64 else np.asarray(v)
                  for k, v in P.items()}
        self.C = {k: np.asarray(v, F64) for k, v in cls.items()}
        self.m = {k: np.zeros_like(v) for k, v in self.C.items()}
        self.v = {k: np.zeros_like(x) for k, x in self.C.items()}
        self.t = 0
        if kind == "multi_central":
            enc = CentralMultiModal("student")

            def run(b, eval_mode):
                out, cache = enc.forward(self.P, b["image"].astype(F64), b["audio"].astype(F64), 1,
                                         eval_mode=eval_mode)
                return out, (None if eval_mode else _stack_stats(cache))
        else:
            fwd, _ = uni_encoder(kind, "student")
            img = UNI_KINDS.get(kind, kind) == "image_simple"

            def run(b, eval_mode):
                x = (b["image"] if img else b["audio"]).astype(F64)
                out, cache = fwd(self.P, x, 1, eval_mode)
                return out, (None if eval_mode else _branch_stats(cache[1]))
        self.run = run

    def features(self, b, eval_mode):
        feat, stats = self.run(b, eval_mode)
        if not eval_mode:
            for bk, st in stats:   # the copy's running statistics (train-mode forward)
                self.P[bk + ".running_mean"], self.P[bk + ".running_var"] = bn_running_update(
                    self.P[bk + ".running_mean"], self.P[bk + ".running_var"], st)
        return feat

    def logits(self, feat):
        C = self.C
        h = linear_fwd(feat, C["classifier.0.weight"], C["classifier.0.bias"])
        return h, linear_fwd(np.maximum(h, 0), C["classifier.2.weight"], C["classifier.2.bias"])

    def train_batch(self, b, lr, wd):
        """One optimizer step on the classifier; returns the batch's mean CE."""
        C = self.C
        feat = self.features(b, False)
        h, logits = self.logits(feat)
        r = np.maximum(h, 0)
        loss, dl = cross_entropy(logits, b["label"])
        dr, dw2, db2 = linear_bwd(dl, r, C["classifier.2.weight"])
        _, dw0, db0 = linear_bwd(dr * (h > 0), feat, C["classifier.0.weight"])
        g = {"classifier.0.weight": dw0, "classifier.0.bias": db0, "classifier.2.weight": dw2,
             "classifier.2.bias": db2}
        self.t += 1
        for k in C:
            C[k], self.m[k], self.v[k] = adamw_step(C[k], g[k], self.m[k], self.v[k], self.t, lr, wd)
        return loss

    def evaluate(self, batches):
        """evaluate() in eval mode: (mean per-batch CE, accuracy %, logits, predictions)."""
        ev_loss, correct, total, all_logits = 0.0, 0, 0, []
        for b in batches:
            _, logits = self.logits(self.features(b, True))
            ev_loss += cross_entropy(logits, b["label"])[0]
            correct += int((logits.argmax(1) == b["label"]).sum())
            total += len(b["label"])
            all_logits.append(logits)
        lg = np.concatenate(all_logits)
        return ev_loss / len(batches), 100.0 * correct / total, lg, lg.argmax(1)

    def running(self):
        return {k: self.P[k].copy() for k in self.P
                if k.endswith(("running_mean", "running_var")) and k.startswith("student.")}


def linear_probe(P, kind, train_batches, valid_batches, cls, lr, wd=0.01):
    """on_train_epoch_end's linear probe (multimodal dino.py:878-951, unimodal 1670-1735) with
    DownstreamClassifier (1764-1814): a frozen deep copy of the student encoder, run in TRAIN
    mode during the probe epoch (batch-stat BatchNorm whose running statistics update the copy;
    fusion dropout p=0 here), classifier Linear(D,128)-ReLU-Linear(128,10) trained with
    AdamW(lr, weight_decay=wd) one step per batch, then evaluate() with the copy in eval mode
    (running statistics).  kind: "multi_central" or an UNIMODAL_MODEL_MAP key.
    batches: lists of dicts image [B,1,28,28], audio [B,1,112,112], label [B].
    cls: classifier.{0,2}.{weight,bias}.  Returns per-batch train losses, val_loss (their mean),
    eval loss / accuracy / logits, the final classifier and the copy's running statistics."""
    pm = _ProbeModel(P, kind, cls)
    losses = [pm.train_batch(b, lr, wd) for b in train_batches]
    ev_loss, acc, logits, _ = pm.evaluate(valid_batches)
    return {"train_losses": np.array(losses), "val_loss": float(np.mean(losses)),
            "eval_loss": ev_loss, "mlp_acc": acc, "logits": logits, "classifier": pm.C,
            "running": pm.running()}


def cosine_annealing_lr(base_lr, epoch, T_max, eta_min=0.0):
    """torch.optim.lr_scheduler.CosineAnnealingLR's value after ``epoch`` steps (closed form)."""
    return eta_min + (base_lr - eta_min) * (1 + math.cos(math.pi * epoch / T_max)) / 2


def train_downstream(P, kind, train_batches, valid_batches, test_batches, cls, num_epochs=10,
                     lr=1e-3, wd=0.01):
    """training_structures/dino_train.py:188-329: DownstreamClassifier trained num_epochs with
    AdamW(classifier, lr) (torch default weight_decay 0.01) + CosineAnnealingLR(T_max=num_epochs)
    stepped per epoch; the copy in train mode for training epochs, eval mode for evaluate();
    the checkpoint of the first epoch with the highest validation accuracy (strict >, starting
    from 0) -- classifier AND the copy's running statistics -- is reloaded for the test set."""
    import copy
    pm = _ProbeModel(P, kind, cls)
    best_acc, best, history = 0.0, None, []
    for epoch in range(num_epochs):
        lr_e = cosine_annealing_lr(lr, epoch, num_epochs)
        losses = [pm.train_batch(b, lr_e, wd) for b in train_batches]
        val_loss, val_acc, _, _ = pm.evaluate(valid_batches)
        history.append((float(np.mean(losses)), val_loss, val_acc))
        if val_acc > best_acc:
            best_acc, best = val_acc, (epoch, copy.deepcopy(pm.C), copy.deepcopy(pm.P))
    if best is not None:
        pm.C, pm.P = best[1], best[2]
    test_loss, test_acc, logits, preds = pm.evaluate(test_batches)
    return {"history": np.array(history), "best_epoch": -1 if best is None else best[0],
            "test_loss": test_loss, "test_acc": test_acc, "test_logits": logits,
            "test_preds": preds, "classifier": pm.C, "running": pm.running()}


def knn_classify(train_x, train_y, test_x, k=5):
    """sklearn KNeighborsClassifier(n_neighbors=k).fit(train_x, train_y).predict(test_x) as
    train_knn_classifier uses it (dino_train.py:362-366): brute-force euclidean distances in
    float64, the k nearest with ties to the smaller train index, uniform-weight vote with ties
    to the smallest class (argmax over sorted classes_).  Returns (predictions, neighbours)."""
    tx, qx = np.asarray(train_x, F64), np.asarray(test_x, F64)
    d = (qx * qx).sum(1)[:, None] - 2 * qx @ tx.T + (tx * tx).sum(1)[None, :]
    nbr = np.argsort(d, axis=1, kind="stable")[:, :k]
    classes, yi = np.unique(np.asarray(train_y), return_inverse=True)
    votes = np.zeros((len(qx), len(classes)), np.int64)
    np.add.at(votes, (np.repeat(np.arange(len(qx)), k), yi[nbr].ravel()), 1)
    return classes[votes.argmax(1)], nbr
