"""Global-negative contrastive losses at the configs' GATHERED sizes, one
rank of the 8-GPU run on one GPU:

* config 3, InfoNCE (dino.py:1091-1128): this rank's B = 1024 rows against C = 8 x 1024 = 8192
  gathered rows per modality (S = [1024 x 8192], twice);
* config 4, NT-Xent (multimodal_simclr.py:74-89): this rank's 2B = 4096 rows [z1; z2] against
  the C = 2 x 8 x 2048 = 32768 gathered rows (S = [4096 x 32768]).

The product functions (avdino.contrastive.infonce / nt_xent) run unchanged; only the two
collectives are replaced by a fake world of 8 (this rank r = 3): the all-gather places this
rank's normalised rows at its slot among fixed synthetic unit rows of the other ranks, and the
reduce-scatter records the full column gradient d(gathered rows) and hands back this rank's own
slice (the other ranks' contributions to it are theirs to send).  Against float64 autograd of
the same per-rank loss (the reference's formula over the global batch, restricted to this
rank's rows): per-row CE terms, d loss / d(local rows) (row side + this rank's column side) and
the column gradient of every other rank's rows.  fp32 operands (the parity mode: GEMMs and
softmax-CE over a stored S): loss 1e-6 relative, gradients 1e-4 rel-L2; bf16 MFMA operands (the
bench mode: the fused kernel avd_xent_fused, S never stored): within 2x the torch
fp16-autocast error of the same loss (the reference's '16-mixed'), floor 1e-3 / 1e-2."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
F64 = torch.float64

W, RANK = 8, 3


class _FakeWorld:
    """avdino.dist with a world of W ranks of which this process is RANK."""

    def __init__(self, monkeypatch, others):
        from avdino import dist as AD
        self.others = others          # {tag: [C, P] f32 unit rows used for the other ranks}
        self.cols = []
        monkeypatch.setattr(AD, "distributed", lambda group=None: True)
        monkeypatch.setattr(AD, "world", lambda group=None: W)
        monkeypatch.setattr(AD, "rank", lambda group=None: RANK)
        monkeypatch.setattr(AD, "gather_rows", self.gather)
        monkeypatch.setattr(AD, "scatter_rows_grad", self.scatter)
        self.k = 0

    def gather(self, x, group=None, out=None):
        B = x.shape[0]
        src = self.others[self.k % len(self.others)]
        self.k += 1
        out.copy_(src)
        out[RANK * B:(RANK + 1) * B] = x
        return out

    def scatter(self, dx_all, group=None, out=None):
        B = dx_all.shape[0] // W
        self.cols.append(dx_all.detach().clone())
        out.copy_(dx_all[RANK * B:(RANK + 1) * B])
        return out


def _unit(g, n, P):
    x = torch.randn(n, P, generator=g, device="cuda", dtype=F64)
    return (x / x.norm(dim=1, keepdim=True)).float()


def _rel(a, b):
    return ((a.double() - b).norm() / b.norm()).item()


def _infonce_ref(zi, za, oi, oa, B, tau, cast=None):
    """Per-rank InfoNCE in float64 autograd: rows = this rank's, columns = all W*B rows."""
    zi = zi.detach().to(F64).requires_grad_()
    za = za.detach().to(F64).requires_grad_()
    oi_, oa_ = oi.to(F64).requires_grad_(), oa.to(F64).requires_grad_()
    ni, na = torch.nn.functional.normalize(zi, dim=1), torch.nn.functional.normalize(za, dim=1)
    sl = slice(RANK * B, (RANK + 1) * B)
    ni_all = torch.cat([oi_[:sl.start], ni, oi_[sl.stop:]])
    na_all = torch.cat([oa_[:sl.start], na, oa_[sl.stop:]])
    tgt = torch.arange(RANK * B, (RANK + 1) * B, device="cuda")
    a, b_ = (ni, na_all) if cast is None else (ni.to(cast), na_all.to(cast))
    S1 = (a @ b_.T).to(F64) / tau
    a, b_ = (na, ni_all) if cast is None else (na.to(cast), ni_all.to(cast))
    S2 = (a @ b_.T).to(F64) / tau
    ce1 = torch.nn.functional.cross_entropy(S1, tgt, reduction="none")
    ce2 = torch.nn.functional.cross_entropy(S2, tgt, reduction="none")
    loss = 0.5 * (ce1.mean() + ce2.mean())
    loss.backward()
    return dict(parts=torch.cat([ce1, ce2]).detach(), loss=loss.item(), dzi=zi.grad,
                dza=za.grad, d_oa=oa_.grad, d_oi=oi_.grad)


@pytest.mark.parametrize("mode", ["f32", "bf16"])
def test_infonce_config3_gathered_size(monkeypatch, mode, capsys):
    from avdino import contrastive, ops
    from avdino.engine import Workspace
    B, P, tau = 1024, 128, 0.07
    C = W * B
    g = torch.Generator(device="cuda").manual_seed(31)
    zi = torch.randn(B, P, generator=g, device="cuda") * 3
    za = torch.randn(B, P, generator=g, device="cuda") * 3
    oi, oa = _unit(g, C, P), _unit(g, C, P)
    fw = _FakeWorld(monkeypatch, [oi, oa])          # gathers: image rows, then audio rows
    ws = Workspace(torch.device("cuda"))
    dzi, dza = torch.empty(B * P, device="cuda"), torch.empty(B * P, device="cuda")
    parts = torch.empty(2 * B, device="cuda")
    gm = ops.GEMM_F32_MFMA if mode == "f32" else ops.GEMM_BF16_MFMA
    scale = contrastive.infonce(ws, zi.reshape(-1), za.reshape(-1), B, P, dzi, dza, parts, tau, gm)
    torch.cuda.synchronize()
    assert scale == 0.5 / B and len(fw.cols) == 2
    ref = _infonce_ref(zi, za, oi, oa, B, tau)
    loss = parts.double().sum().item() * scale       # parts: per-row CE, loss = sum * scale
    sl = np.r_[0:RANK * B, (RANK + 1) * B:C]
    err = dict(loss=abs(loss - ref["loss"]) / ref["loss"], parts=_rel(parts, ref["parts"]),
               dzi=_rel(dzi.view(B, P), ref["dzi"]), dza=_rel(dza.view(B, P), ref["dza"]),
               col_a=_rel(fw.cols[0][sl], ref["d_oa"][sl]),      # dS carries the 0.5 / B
               col_i=_rel(fw.cols[1][sl], ref["d_oi"][sl]))
    if mode == "f32":
        tol = dict(loss=1e-6, parts=1e-5, dzi=1e-4, dza=1e-4, col_a=1e-4, col_i=1e-4)
    else:
        r16 = _infonce_ref(zi, za, oi, oa, B, tau, cast=torch.float16)
        band = dict(loss=abs(r16["loss"] - ref["loss"]) / ref["loss"], parts=_rel(r16["parts"], ref["parts"]),
                    dzi=_rel(r16["dzi"], ref["dzi"]), dza=_rel(r16["dza"], ref["dza"]),
                    col_a=_rel(r16["d_oa"][sl], ref["d_oa"][sl]), col_i=_rel(r16["d_oi"][sl], ref["d_oi"][sl]))
        tol = {k: max(2 * v, 1e-3 if k in ("loss", "parts") else 1e-2) for k, v in band.items()}
    with capsys.disabled():
        print(f"\nInfoNCE [{B} x {C}] {mode}: " + ", ".join(f"{k} {v:.2e} (tol {tol[k]:.1e})" for k, v in err.items()))
    assert all(err[k] <= tol[k] for k in err), (err, tol)


def _ntxent_ref(reps, o, B, tau, cast=None):
    """Per-rank NT-Xent in float64: rows [z1; z2] of this rank, columns [z1 of every rank;
    z2 of every rank], own column masked, positive = the other view of the same sample."""
    reps = reps.detach().to(F64).requires_grad_()
    o_ = o.to(F64).requires_grad_()
    n = torch.nn.functional.normalize(reps, dim=1)
    WB = W * B
    s1, s2 = slice(RANK * B, (RANK + 1) * B), slice(WB + RANK * B, WB + (RANK + 1) * B)
    n_all = torch.cat([o_[:s1.start], n[:B], o_[s1.stop:s2.start], n[B:], o_[s2.stop:]])
    a, b_ = (n, n_all) if cast is None else (n.to(cast), n_all.to(cast))
    S = (a @ b_.T).to(F64) / tau
    own = torch.cat([torch.arange(s1.start, s1.stop), torch.arange(s2.start, s2.stop)]).cuda()
    S = S.masked_fill(torch.nn.functional.one_hot(own, 2 * WB).bool(), float("-inf"))
    tgt = torch.cat([torch.arange(s2.start, s2.stop), torch.arange(s1.start, s1.stop)]).cuda()
    ce = torch.nn.functional.cross_entropy(S, tgt, reduction="none")
    loss = ce.mean()
    loss.backward()
    return dict(parts=ce.detach(), loss=loss.item(), dreps=reps.grad, d_o=o_.grad)


@pytest.mark.parametrize("mode", ["f32", "bf16"])
def test_ntxent_config4_gathered_size(monkeypatch, mode, capsys):
    from avdino import contrastive, ops
    from avdino.engine import Workspace
    B, P, tau = 2048, 256, 0.07
    C = 2 * W * B
    g = torch.Generator(device="cuda").manual_seed(41)
    reps = torch.randn(2 * B, P, generator=g, device="cuda") * 2
    o = _unit(g, C, P)
    WB = W * B
    fw = _FakeWorld(monkeypatch, [o[:WB], o[WB:]])   # gathers: z1 rows, then z2 rows
    ws = Workspace(torch.device("cuda"))
    dreps, parts = torch.empty(2 * B * P, device="cuda"), torch.empty(2 * B, device="cuda")
    gm = ops.GEMM_F32_MFMA if mode == "f32" else ops.GEMM_BF16_MFMA
    scale = contrastive.nt_xent(ws, reps.reshape(-1), B, P, dreps, parts, tau, gm)
    torch.cuda.synchronize()
    assert scale == 1.0 / (2 * B) and len(fw.cols) == 2
    ref = _ntxent_ref(reps, o, B, tau)
    col = torch.cat(fw.cols)                         # [z1 of every rank; z2 of every rank]
    keep = torch.ones(C, dtype=torch.bool)
    keep[RANK * B:(RANK + 1) * B] = False
    keep[WB + RANK * B:WB + (RANK + 1) * B] = False
    keep = keep.cuda()
    loss = parts.double().sum().item() * scale
    err = dict(loss=abs(loss - ref["loss"]) / ref["loss"], parts=_rel(parts, ref["parts"]),
               dreps=_rel(dreps.view(2 * B, P), ref["dreps"]), col=_rel(col[keep], ref["d_o"][keep]))
    if mode == "f32":
        tol = dict(loss=1e-6, parts=1e-5, dreps=1e-4, col=1e-4)
    else:
        r16 = _ntxent_ref(reps, o, B, tau, cast=torch.float16)
        band = dict(loss=abs(r16["loss"] - ref["loss"]) / ref["loss"], parts=_rel(r16["parts"], ref["parts"]),
                    dreps=_rel(r16["dreps"], ref["dreps"]), col=_rel(r16["d_o"][keep], ref["d_o"][keep]))
        tol = {k: max(2 * v, 1e-3 if k in ("loss", "parts") else 1e-2) for k, v in band.items()}
    with capsys.disabled():
        print(f"\nNT-Xent [{2 * B} x {C}] {mode}: " + ", ".join(f"{k} {v:.2e} (tol {tol[k]:.1e})" for k, v in err.items()))
    assert all(err[k] <= tol[k] for k in err), (err, tol)


def _xent_ref(q, k, Bh, tgt, msk, inv_t, g, cast=None):
    """float64 autograd of the per-row CE over S = inv_t q k^T with per-half targets / masks."""
    q = q.detach().to(F64).requires_grad_()
    k = k.detach().to(F64).requires_grad_()
    R, C = q.shape[0], k.shape[0]
    a, b = (q, k) if cast is None else (q.to(cast), k.to(cast))
    S = (a @ b.T).to(F64) * inv_t
    i = torch.arange(R, device="cuda")
    h = (i >= Bh).long()
    ii = i - h * Bh
    t = torch.tensor(tgt, device="cuda")[h] + ii
    m = torch.tensor(msk, device="cuda")[h]
    mask = torch.zeros(R, C, dtype=torch.bool, device="cuda")
    has = m >= 0
    mask[i[has], (m + ii)[has]] = True
    S = S.masked_fill(mask, float("-inf"))
    ce = torch.nn.functional.cross_entropy(S, t, reduction="none")
    (ce.sum() * g).backward()
    return ce.detach(), q.grad, k.grad


XCASES = [  # R, C, P, Bh, tgt, msk  (NT-Xent: R = 2 Bh, C = 2 W Bh; InfoNCE: R = Bh, C = W Bh)
    (10, 10, 128, 5, (5, 0), (0, 5)),                 # NT-Xent, world 1, tails everywhere
    (6, 24, 256, 3, (15, 3), (3, 15)),                # NT-Xent, a rank of world 4
    (7, 21, 256, 7, (7, 0), (-1, -1)),                # InfoNCE, rank 1 of world 3
    (200, 200, 128, 100, (100, 0), (0, 100)),         # several row / column blocks
    (96, 768, 128, 96, (288, 0), (-1, -1)),           # InfoNCE rank 3 of 8, column splits
]


@pytest.mark.parametrize("case", XCASES, ids=[f"R{c[0]}C{c[1]}P{c[2]}" for c in XCASES])
def test_xent_fused_against_float64(case, capsys):
    """avd_xent_fused (xent.hip) on edge shapes -- rows / columns not multiples of the 64-row
    block or the 32-column step, one or two halves, with and without a masked own column --
    against float64 autograd of the same loss; bands as above (2x the fp16-operand error of the
    same float64 computation, floors 1e-3 / 1e-2)."""
    from avdino import ops
    R, C, P, Bh, tgt, msk = case
    g_ = torch.Generator(device="cuda").manual_seed(R * 1000 + C)
    q, k = _unit(g_, R, P), _unit(g_, C, P)
    inv_t, gs = 1.0 / 0.07, 1.0 / R
    loss = torch.empty(R, device="cuda")
    dq, dk = torch.empty(R, P, device="cuda"), torch.empty(C, P, device="cuda")
    ws = torch.empty(ops.xent_fused_ws(R, C, P), device="cuda")
    ops.xent_fused(q, k, R, C, P, Bh, tgt, msk, inv_t, gs, loss, dq, dk, ws)
    torch.cuda.synchronize()
    ce, gq, gk = _xent_ref(q, k, Bh, tgt, msk, inv_t, gs)
    c16, q16, k16 = _xent_ref(q, k, Bh, tgt, msk, inv_t, gs, cast=torch.float16)
    err = dict(loss=_rel(loss, ce), dq=_rel(dq, gq), dk=_rel(dk, gk))
    band = dict(loss=_rel(c16, ce), dq=_rel(q16, gq), dk=_rel(k16, gk))
    tol = {n: max(2 * band[n], 1e-3 if n == "loss" else 1e-2) for n in err}
    with capsys.disabled():
        print(f"\nxent R={R} C={C} P={P}: " + ", ".join(f"{n} {err[n]:.2e} (tol {tol[n]:.1e})" for n in err))
    assert all(err[n] <= tol[n] for n in err), (err, tol)
    # deterministic: a second launch is bit-identical
    loss2, dq2, dk2 = torch.empty_like(loss), torch.empty_like(dq), torch.empty_like(dk)
    ops.xent_fused(q, k, R, C, P, Bh, tgt, msk, inv_t, gs, loss2, dq2, dk2, ws)
    assert torch.equal(loss, loss2) and torch.equal(dq, dq2) and torch.equal(dk, dk2)
