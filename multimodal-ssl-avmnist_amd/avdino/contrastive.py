"""Contrastive heads with local or GLOBAL negatives.

* InfoNCE of MultiModalDINOWithINFONCELightning.infoNCE_loss (dino.py:1091-1128; same math
  other_ssl/info_nce/info_nce.py:75-112): S = n(i) n(a)^T / tau, (CE(S, diag) + CE(S^T, diag))/2.
* NT-Xent of MultiModalSimCLRLightning.nt_xent_loss (multimodal_simclr.py:74-89):
  reps = [z1; z2], S = n n^T / tau with the diagonal masked, targets (i + B) mod 2B.

With world W > 1 (one process per GPU, torch.distributed over RCCL) every rank keeps its own
B rows and all-gathers the L2-normalised rows of the other ranks as negatives, so rank r's rows
of S are exactly rows r*B.. of the single-device S over the global W*B batch.  Each rank's
loss is the mean over ITS rows; DDP's gradient averaging (x 1/W) then yields the gradient of
the global-batch loss.  The column side of dS (how my rows act as other ranks' negatives /
positives) is reduce-scattered back to the owning rank (avdino.dist).  W == 1 is the
reference's single-device loss exactly.  The collectives are host points (avdino.capture) on
fixed workspace buffers, so a global-negative step is still a captured graph -- three
segments around the gather and the scatter.

Compute is libavdino: l2norm, then -- with bf16 MFMA operands (the bench precision) and P = 128
or 256 -- the fused softmax-CE avd_xent_fused (xent.hip: S never stored; rows then columns,
flash-style), else (the fp32 parity mode) MFMA GEMMs into f32 S / dS and avd_softmax_xent with
offset targets / masks; axpy.
"""
from . import dist, ops
from .capture import host_point


class _Norm:
    def __init__(self, ws, tag, x, rows, P):
        self.y = ws.get(tag + ".n", rows * P)
        self.r = ws.get(tag + ".r", rows)
        self.rows, self.P = rows, P
        ops.l2norm_fwd(x, self.y, self.r, rows, P)

    def backward(self, dy, dx):
        ops.l2norm_bwd(self.y, self.r, dy, dx, self.rows, self.P)


def _world(local, group):
    """(world, rank, exchange?) of the negatives: exchange = the gathered path (world > 1, or
    the world-1 collectives forced by dist.forced())."""
    if local or not dist.distributed(group):
        return 1, 0, False
    return dist.world(group), dist.rank(group), True


# the bf16 step's contrastive losses on the fused kernel (False: GEMMs + softmax-CE over S)
FUSED = True


def _fused(gm, P):
    return FUSED and gm == ops.GEMM_BF16_MFMA and P in (128, 256)


def infonce(ws, zi, za, B, P, dzi, dza, loss_parts, temperature=0.07, gm=ops.GEMM_F32_MFMA,
            group=None, local=False):
    """zi, za [B, P] (this rank's rows) -> loss_parts [2B] per-row CE (this rank's loss =
    sum(loss_parts) * 0.5 / B), dzi, dza [B, P] (d of that loss).  Returns the scale."""
    W, r, xg = _world(local, group)
    inv_t = 1.0 / temperature
    ni, na = _Norm(ws, "nce.i", zi, B, P), _Norm(ws, "nce.a", za, B, P)
    C = W * B
    if not xg:
        ni_all, na_all = ni.y, na.y
    else:   # host point: the all-gathers write fixed buffers the next graph segment reads
        ni_all, na_all = ws.get("nce.ni_all", C * P), ws.get("nce.na_all", C * P)
        host_point(lambda: (dist.gather_rows(ni.y.view(B, P), group, out=ni_all.view(C, P)),
                            dist.gather_rows(na.y.view(B, P), group, out=na_all.view(C, P))))
    if _fused(gm, P):
        # rows of S1 = n(i) n(a_all)^T / tau and S2 = n(a) n(i_all)^T / tau, targets r*B + i
        xw = ws.get("nce.xws", ops.xent_fused_ws(B, C, P))
        dni, dna = ws.get("nce.dni", B * P), ws.get("nce.dna", B * P)
        cA, cI = ws.get("nce.colA", C * P), ws.get("nce.colI", C * P)
        ops.xent_fused(ni.y, na_all, B, C, P, B, (r * B, 0), (-1, -1), inv_t, 0.5 / B, loss_parts[:B],
                       dni, cA, xw)
        ops.xent_fused(na.y, ni_all, B, C, P, B, (r * B, 0), (-1, -1), inv_t, 0.5 / B,
                       loss_parts[B:2 * B], dna, cI, xw)
        return _infonce_tail(ws, ni, na, dni, dna, cA, cI, dzi, dza, B, P, C, xg, group)
    S1, S2 = ws.get("nce.S1", B * C), ws.get("nce.S2", B * C)
    ops.gemm(B, C, P, ni.y, P, 1, na_all, 1, P, S1, C, alpha=inv_t, mode=gm)   # image rows
    ops.gemm(B, C, P, na.y, P, 1, ni_all, 1, P, S2, C, alpha=inv_t, mode=gm)   # audio rows
    dS1, dS2 = ws.get("nce.dS1", B * C), ws.get("nce.dS2", B * C)
    ops.softmax_xent(S1, C, B, C, None, 1, False, False, 0.5 / B, loss_parts[:B], dS1, C, False,
                     tgt_off=r * B)
    ops.softmax_xent(S2, C, B, C, None, 1, False, False, 0.5 / B, loss_parts[B:2 * B], dS2, C,
                     False, tgt_off=r * B)
    dni, dna = ws.get("nce.dni", B * P), ws.get("nce.dna", B * P)
    ops.gemm(B, P, C, dS1, C, 1, na_all, P, 1, dni, P, alpha=inv_t, mode=gm)   # row side
    ops.gemm(B, P, C, dS2, C, 1, ni_all, P, 1, dna, P, alpha=inv_t, mode=gm)
    # column side: d(na_all) from S1, d(ni_all) from S2, each [C, P], owned rows scattered home
    cA, cI = ws.get("nce.colA", C * P), ws.get("nce.colI", C * P)
    ops.gemm(C, P, B, dS1, 1, C, ni.y, P, 1, cA, P, alpha=inv_t, mode=gm)
    ops.gemm(C, P, B, dS2, 1, C, na.y, P, 1, cI, P, alpha=inv_t, mode=gm)
    return _infonce_tail(ws, ni, na, dni, dna, cA, cI, dzi, dza, B, P, C, xg, group)


def _infonce_tail(ws, ni, na, dni, dna, cA, cI, dzi, dza, B, P, C, xg, group):
    """Column gradients home (added, or reduce-scattered to their owners), then the l2norm
    backward."""
    if not xg:
        ops.axpy(dna, cA)
        ops.axpy(dni, cI)
    else:
        rA, rI = ws.get("nce.rA", B * P), ws.get("nce.rI", B * P)
        host_point(lambda: (dist.scatter_rows_grad(cA.view(C, P), group, out=rA.view(B, P)),
                            dist.scatter_rows_grad(cI.view(C, P), group, out=rI.view(B, P))))
        ops.axpy(dna, rA)
        ops.axpy(dni, rI)
    ni.backward(dni, dzi)
    na.backward(dna, dza)
    return 0.5 / B


def nt_xent(ws, reps, B, P, dreps, loss_parts, temperature=0.07, gm=ops.GEMM_F32_MFMA, group=None,
            local=False):
    """reps [2B, P] = [z1; z2] of this rank -> loss_parts [2B] per-row CE (this rank's loss =
    sum(loss_parts) / 2B), dreps [2B, P].  Returns the scale."""
    W, r, xg = _world(local, group)
    inv_t = 1.0 / temperature
    n = _Norm(ws, "ntx", reps, 2 * B, P)
    nv = n.y.view(2 * B, P)
    if not xg:
        n_all = n.y
    else:   # global layout [z1 of every rank; z2 of every rank]; host point as in infonce
        n_all = ws.get("ntx.all", 2 * W * B * P)
        av = n_all.view(2, W * B, P)
        host_point(lambda: (dist.gather_rows(nv[:B], group, out=av[0]),
                            dist.gather_rows(nv[B:], group, out=av[1])))
    C = 2 * W * B
    g = 1.0 / (2 * B)
    dn = ws.get("ntx.dn", 2 * B * P)
    col = ws.get("ntx.col", C * P)
    if _fused(gm, P):
        # z1 rows: target W*B + r*B + i, own column r*B + i masked; z2 rows the other way round
        xw = ws.get("ntx.xws", ops.xent_fused_ws(2 * B, C, P))
        ops.xent_fused(n.y, n_all, 2 * B, C, P, B, (W * B + r * B, r * B), (r * B, W * B + r * B), inv_t, g,
                       loss_parts, dn, col, xw)
        return _ntxent_tail(ws, n, dn, col, dreps, B, P, W, xg, group, g)
    S = ws.get("ntx.S", 2 * B * C)
    ops.gemm(2 * B, C, P, n.y, P, 1, n_all, 1, P, S, C, alpha=inv_t, mode=gm)
    dS = ws.get("ntx.dS", 2 * B * C)
    # z1 rows: global row r*B + i, positive W*B + r*B + i; z2 rows: W*B + r*B + i -> r*B + i
    ops.softmax_xent(S, C, B, C, None, 1, False, True, g, loss_parts[:B], dS, C, False,
                     tgt_off=W * B + r * B, mask_off=r * B)
    ops.softmax_xent(S[B * C:], C, B, C, None, 1, False, True, g, loss_parts[B:2 * B], dS[B * C:],
                     C, False, tgt_off=r * B, mask_off=W * B + r * B)
    ops.gemm(2 * B, P, C, dS, C, 1, n_all, P, 1, dn, P, alpha=inv_t, mode=gm)   # row side
    ops.gemm(C, P, 2 * B, dS, 1, C, n.y, P, 1, col, P, alpha=inv_t, mode=gm)   # column side
    return _ntxent_tail(ws, n, dn, col, dreps, B, P, W, xg, group, g)


def _ntxent_tail(ws, n, dn, col, dreps, B, P, W, xg, group, g):
    if not xg:
        ops.axpy(dn, col)
    else:
        cv = col.view(2, W * B, P)
        rc = ws.get("ntx.rc", 2 * B * P)
        rv = rc.view(2, B, P)
        host_point(lambda: (dist.scatter_rows_grad(cv[0], group, out=rv[0]),
                            dist.scatter_rows_grad(cv[1], group, out=rv[1])))
        ops.axpy(dn, rc)
    n.backward(dn, dreps)
    return g
