"""Tensor-level wrappers over the C ABI (include/avdino.h).

Every function takes torch tensors that live on the HIP device, checks shapes/dtypes on the
host, and launches on torch's current stream.  PyTorch is used here only for device memory
and streams; all arithmetic happens in libavdino.so.
"""
import contextlib
import ctypes

import torch

from ._lib import BF16, F32, call, lib

_DT = {torch.float32: F32, torch.bfloat16: BF16}


def dtcode(t):
    try:
        return _DT[t.dtype]
    except KeyError:
        raise TypeError(f"unsupported dtype {t.dtype}") from None


def p(t):
    """Device pointer of a (contiguous) tensor, or None."""
    if t is None:
        return None
    if not t.is_contiguous():
        raise ValueError("tensor must be contiguous")
    return t.data_ptr()


def stream():
    return torch.cuda.current_stream().cuda_stream


class _Options(ctypes.Structure):
    """avd_options (include/avdino.h)."""
    _fields_ = [("grid_cap", ctypes.c_int), ("generic_conv", ctypes.c_int), ("generic_m2", ctypes.c_int)]


def get_options():
    o = _Options()
    call("avd_get_options", ctypes.byref(o))
    return {k: getattr(o, k) for k, _ in _Options._fields_}


@contextlib.contextmanager
def options(**kw):
    """The library's launch options (avd_set_options: grid_cap, generic_conv, generic_m2 -- test
    hooks; the library reads no environment variables) set for the duration of the block."""
    old = _Options()
    call("avd_get_options", ctypes.byref(old))
    new = _Options(old.grid_cap, old.generic_conv, old.generic_m2)
    for k, v in kw.items():
        if k not in dict(_Options._fields_):
            raise KeyError(f"avd_options has no field {k!r}")
        setattr(new, k, int(v))
    call("avd_set_options", ctypes.byref(new))
    try:
        yield
    finally:
        call("avd_set_options", ctypes.byref(old))


class KernelTimer:
    """Optional HIP-event timing of selected launches (bench.py's live roofline).

    Each instrumented op reports a key (op name + shape), its algorithmic HBM bytes and
    FLOPs; events are recorded on the launching stream around the launch.  ``only`` limits
    timing to one key (the dominant kernel) so the timed region stays undisturbed."""

    def __init__(self, only=None):
        # None: every instrumented launch; else one key or a set of keys
        self.only = {only} if isinstance(only, str) else (set(only) if only is not None else None)
        self.rec = []  # (key, bytes, flops, start_event, end_event)
        self.replay = None  # last launch closure of the ``only`` key (bench --probe-dominant)
        self.fns = {}       # key -> last launch closure (tools/opbench.py replays them)

    def wrap(self, key, nbytes, flops, fn):
        # launches of one op and shape from different streams are different call sites (e.g.
        # the audio conv3 and image conv1 BN-backward apply share a shape): keyed apart
        if torch.cuda.current_stream() != torch.cuda.default_stream():
            key += " @side"
        if self.only is not None and key not in self.only:
            return fn()
        if self.only is not None:
            self.replay = fn
        self.fns[key] = (fn, nbytes, flops)
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        s.record()
        out = fn()
        e.record()
        self.rec.append((key, nbytes, flops, s, e))
        return out

    def summary(self):
        torch.cuda.synchronize()
        agg = {}
        for key, nb, fl, s, e in self.rec:
            a = agg.setdefault(key, [0, 0.0, 0, 0])
            a[0] += 1
            a[1] += s.elapsed_time(e)
            a[2] += nb
            a[3] += fl
        return {k: dict(calls=v[0], ms=v[1], bytes=v[2], flops=v[3]) for k, v in agg.items()}


TIMER = None


def _timed(key, nbytes, flops, fn):
    if SPANS is not None:
        return SPANS.wrap(key, nbytes, flops, fn)
    if TIMER is None:
        return fn()
    return TIMER.wrap(key, nbytes, flops, fn)


class SpanTimer:
    """In-graph duration of selected launch sites (bench.py's live roofline of a replayed step):
    span marks (avd_mark_span, the device real-time counter) on the launching stream before and
    after each launch of a watched key, captured into the step's graph with it, so every
    replay of the timed region adds its duration.  Keys are matched without KernelTimer's
    " @side" suffix (inside a capture every launch is on a non-default stream)."""

    def __init__(self, device, keys, cap=64):
        self.keys = {k.replace(" @side", "") for k in keys}
        self.slots = {}
        self.info = {}
        self.buf = torch.zeros(3 * cap, dtype=torch.int64, device=device)

    def wrap(self, key, nbytes, flops, fn):
        if key not in self.keys:
            return fn()
        st = torch.cuda.current_stream().cuda_stream
        # one begin/end slot per (key, stream): the same launch key queued on two streams of
        # one captured step would otherwise overwrite the other's begin mark
        sk = (key, st)
        if sk not in self.slots and len(self.slots) >= self.buf.numel() // 3:
            return fn()
        slot = self.slots.setdefault(sk, len(self.slots))
        self.info[key] = (nbytes, flops)
        call("avd_mark_span", p(self.buf), slot, 0, st)
        out = fn()
        call("avd_mark_span", p(self.buf), slot, 1, st)
        return out

    def reset(self):
        self.buf.zero_()

    def read(self):
        """{key: (launches, total us, bytes per launch, flops per launch)} since reset(), summed
        over the streams the key ran on."""
        torch.cuda.synchronize()
        b = self.buf.view(-1, 3).cpu().tolist()
        out = {}
        for (k, _st), s in self.slots.items():
            if b[s][2]:
                n, us = out.get(k, (0, 0.0))[:2]
                out[k] = (n + b[s][2], us + b[s][1] / 100.0) + self.info[k]
        return out


SPANS = None


# Scratch allocation epoch: bumped whenever a workspace / scratch buffer is (re)allocated.  A
# captured hipGraph bakes in the device pointers it saw, so a graph captured in an earlier epoch
# may address freed memory and must not be replayed (capture.GraphedStep checks this).
_ALLOC_EPOCH = [0]


def bump_alloc_epoch():
    _ALLOC_EPOCH[0] += 1


def alloc_epoch():
    return _ALLOC_EPOCH[0]


def _need(cond, msg):
    if not cond:
        raise ValueError(msg)


# ---------------------------------------------------------------- BatchNorm statistics
def bn_finalize(parts, G, R, C, count, gamma, beta, mean, invstd, scale, shift, rm=None, rv=None,
                eps=1e-5, momentum=0.1, pivot=None, pivot_gs=None):
    """pivot [G, C] (pivot_gs = C, avd_colstats) or [C] (pivot_gs = 0, avd_cl_conv_fwd_pv)."""
    if pivot is not None:
        pivot_gs = C if pivot_gs is None else pivot_gs
        _need(pivot.numel() >= (G - 1) * pivot_gs + C, "bn_finalize pivot size")
    call("avd_bn_finalize", p(parts), G, R, C, count, p(gamma), p(beta), eps, momentum, p(mean),
         p(invstd), p(scale), p(shift), p(rm), p(rv), p(pivot), int(pivot_gs or 0), stream())


def bn_bwd_finalize(parts, G, R, C, count, gamma, mean, invstd, coef, dgamma, dbeta, dbias,
                    accumulate=0):
    call("avd_bn_bwd_finalize", p(parts), G, R, C, count, p(gamma), p(mean), p(invstd), p(coef),
         p(dgamma), p(dbeta), p(dbias), accumulate, stream())


# ---------------------------------------------------------------- dense
GEMM_F32_VALU, GEMM_F32_MFMA, GEMM_BF16_MFMA = 0, 1, 2


def gemm(M, N, K, A, sam, sak, B, sbk, sbn, C, ldc, bias=None, alpha=1.0, beta=0.0,
         a_off=0, b_off=0, c_off=0, mode=GEMM_F32_MFMA):
    """C[m,n] = alpha*sum_k A[m,k]B[k,n] (+bias[n]) (+beta*C).  *_off are element offsets into
    the (flat, f32) storage of A/B/C so row/column slices need no copies."""
    for t in (A, B, C):
        _need(t.dtype == torch.float32 and t.is_contiguous(), "gemm operands are contiguous f32")
    # every element the kernel may touch must lie inside the tensors (no device OOB)
    _need(a_off >= 0 and a_off + (M - 1) * sam + (K - 1) * sak < A.numel(), "gemm A bounds")
    _need(b_off >= 0 and b_off + (K - 1) * sbk + (N - 1) * sbn < B.numel(), "gemm B bounds")
    _need(c_off >= 0 and c_off + (M - 1) * ldc + (N - 1) < C.numel(), "gemm C bounds")
    _need(bias is None or bias.numel() >= N, "gemm bias")
    nws = lib.avd_gemm_ws_elems(M, N, K, mode)
    ws = _gemm_workspace(C.device, nws) if nws > 0 else None
    _timed(f"gemm[{M}x{N}x{K} m{mode}]", 4 * (M * K + K * N + M * N), 2 * M * N * K,
           lambda: call("avd_gemm", M, N, K, A.data_ptr() + 4 * a_off, sam, sak,
                        B.data_ptr() + 4 * b_off, sbk, sbn, C.data_ptr() + 4 * c_off, ldc, p(bias),
                        alpha, beta, mode, p(ws), nws, stream()))


_GEMM_WS = {}


def _gemm_workspace(device, n):
    """Split-K partial-tile scratch, one per (device, stream), grown on demand (stream-ordered
    reuse: every GEMM on a stream finishes its reduce before the next one writes; engines that
    run branches on side streams get their own)."""
    key = (device, torch.cuda.current_stream(device).cuda_stream)
    t = _GEMM_WS.get(key)
    if t is None or t.numel() < n:
        t = torch.empty(max(n, 1 << 20), device=device, dtype=torch.float32)
        _GEMM_WS[key] = t
        bump_alloc_epoch()
    return t


def linear_fwd(x, w, b, out, rows, x_ld=None, x_off=0, out_ld=None, out_off=0, mode=GEMM_F32_MFMA):
    """out[rows, O] = x[rows, I] W^T + b   (W [O, I])."""
    O, In = w.shape
    x_ld = In if x_ld is None else x_ld
    out_ld = O if out_ld is None else out_ld
    gemm(rows, O, In, x, x_ld, 1, w, 1, In, out, out_ld, bias=b, a_off=x_off, c_off=out_off,
         mode=mode)


# Linear backward's dW and dX GEMMs in one launch (avd_linear_bwd); False: two GEMM launches
PAIR_BWD = True


def linear_bwd(dout, x, w, dw, db, dx, rows, dout_ld=None, dout_off=0, x_ld=None, x_off=0,
               dx_ld=None, dx_off=0, mode=GEMM_F32_MFMA):
    """dW = dout^T x ; db = sum_rows dout ; dx = dout W  (dx or dw optional)."""
    O, In = w.shape
    dout_ld = O if dout_ld is None else dout_ld
    x_ld = In if x_ld is None else x_ld
    dx_ld = In if dx_ld is None else dx_ld
    if dw is None:                  # the input gradient alone
        _need(dx is not None, "linear_bwd: nothing to compute")
        gemm(rows, In, O, dout, dout_ld, 1, w, In, 1, dx, dx_ld, a_off=dout_off, c_off=dx_off, mode=mode)
        return
    if dx is not None and mode in (GEMM_F32_MFMA, GEMM_BF16_MFMA) and PAIR_BWD:
        # dW, dX and the bias gradient on the same launches (avd_linear_bwd)
        for t in (dout, x, w, dw, dx):
            _need(t.dtype == torch.float32 and t.is_contiguous(), "linear_bwd operands are contiguous f32")
        _need(dout_off + (rows - 1) * dout_ld + O <= dout.numel(), "linear_bwd dout bounds")
        _need(x_off + (rows - 1) * x_ld + In <= x.numel(), "linear_bwd x bounds")
        _need(dx_off + (rows - 1) * dx_ld + In <= dx.numel(), "linear_bwd dx bounds")
        _need(dw.numel() >= O * In, "linear_bwd dw size")
        nws = lib.avd_linear_bwd_ws_elems(rows, O, In, mode)   # > 0: includes the bias partials
        ws = _gemm_workspace(dout.device, nws)
        _need(db is None or db.numel() >= O, "linear_bwd db size")
        _timed(f"linear_bwd[{rows}x{O}x{In} m{mode}]",
               4 * (2 * rows * O + rows * In + O * In + O * In + rows * In), 4 * rows * O * In,
               lambda: call("avd_linear_bwd", rows, O, In, dout.data_ptr() + 4 * dout_off, dout_ld,
                            x.data_ptr() + 4 * x_off, x_ld, p(w), p(dw),
                            dx.data_ptr() + 4 * dx_off, dx_ld, p(db), mode, 3, p(ws), nws, stream()))
        return
    if dx is None and mode in (GEMM_F32_MFMA, GEMM_BF16_MFMA) and PAIR_BWD:
        # the weight gradient alone (+ db) on the paired launch's dW grid and its reduce
        for t in (dout, x, dw):
            _need(t.dtype == torch.float32 and t.is_contiguous(), "linear_bwd operands are contiguous f32")
        _need(dout_off + (rows - 1) * dout_ld + O <= dout.numel(), "linear_bwd dout bounds")
        _need(x_off + (rows - 1) * x_ld + In <= x.numel(), "linear_bwd x bounds")
        _need(dw.numel() >= O * In and (db is None or db.numel() >= O), "linear_bwd dw / db size")
        nws = lib.avd_linear_bwd_ws_elems(rows, O, In, mode)
        ws = _gemm_workspace(dout.device, nws)
        _timed(f"linear_bwd_dw[{rows}x{O}x{In} m{mode}]", 4 * (rows * O + rows * In + O * In),
               2 * rows * O * In,
               lambda: call("avd_linear_bwd", rows, O, In, dout.data_ptr() + 4 * dout_off, dout_ld,
                            x.data_ptr() + 4 * x_off, x_ld, None, p(dw), None, In, p(db), mode, 1,
                            p(ws), nws, stream()))
        return
    # dW[o, i] = sum_r dout[r, o] x[r, i]: A = dout^T (M=O, K=rows), B = x (K=rows, N=In)
    gemm(O, In, rows, dout, 1, dout_ld, x, x_ld, 1, dw, In, a_off=dout_off, b_off=x_off, mode=mode)
    if db is not None:
        sum_rows(dout, rows, O, db, ld=dout_ld, off=dout_off)
    if dx is not None:
        gemm(rows, In, O, dout, dout_ld, 1, w, In, 1, dx, dx_ld, a_off=dout_off, c_off=dx_off,
             mode=mode)


# ---- the encoder Linear over NHWC bf16 features (include/avdino.h "encoder Linear ... NHWC")
def linear_weight_hwc(entries):
    """entries: [(W f32 [O, C*HW] in (c,h,w) column order, Wp bf16 [O*HW*C], C, HW)] (<= 4) ->
    Wp = W with its columns in (h, w, c) order, one launch."""
    import ctypes as _ct
    n = len(entries)
    _need(0 < n <= 4, "linear_weight_hwc batch size")
    for W, Wp, C, HW in entries:
        _need(W.dtype == torch.float32 and W.is_contiguous() and W.shape[1] == C * HW, "hwc W")
        _need(Wp.dtype == torch.bfloat16 and Wp.numel() >= W.numel(), "hwc Wp")
    ws = (_ct.c_void_p * n)(*[e[0].data_ptr() for e in entries])
    wps = (_ct.c_void_p * n)(*[e[1].data_ptr() for e in entries])
    Os = (_ct.c_int * n)(*[e[0].shape[0] for e in entries])
    Cs = (_ct.c_int * n)(*[e[2] for e in entries])
    HWs = (_ct.c_int * n)(*[e[3] for e in entries])
    call("avd_linear_weight_hwc", n, ws, wps, Os, Cs, HWs, stream())


def linear_fwd_hwc(feat, wp, b, out, rows, O, C, HW, out_ld=None, out_off=0):
    """out[rows, O] (+out_ld/off) = feat_hwc[rows, HW*C] Wp^T + b on the bf16 MFMA (the encoder
    Linear over the last conv block's NHWC pooled map)."""
    In = C * HW
    out_ld = O if out_ld is None else out_ld
    _need(feat.dtype == torch.bfloat16 and feat.numel() >= rows * In, "hwc fwd feat")
    _need(wp.dtype == torch.bfloat16 and wp.numel() >= O * In, "hwc fwd Wp")
    _need(out.dtype == torch.float32 and out_off + (rows - 1) * out_ld + O <= out.numel(), "hwc fwd out")
    nws = lib.avd_linear_hwc_ws_elems(rows, O, In)
    ws = _gemm_workspace(out.device, nws)
    _timed(f"linear_fwd_hwc[{rows}x{O}x{In}]", 2 * rows * In + 2 * O * In + 4 * rows * O,
           2 * rows * O * In,
           lambda: call("avd_linear_fwd_hwc", rows, O, C, HW, p(feat), p(wp), p(b),
                        out.data_ptr() + 4 * out_off, out_ld, p(ws), nws, stream()))


def linear_bwd_hwc(dout, feat, wp, dw, db, dx, rows, O, C, HW, dout_ld=None, dout_off=0, which=3):
    """dW (reference (c,h,w) columns) = dout^T feat_hwc; db = sum_rows dout; dx (bf16 NHWC) =
    dout Wp -- one paired launch + split-K reduces (avd_linear_bwd_hwc; which 1 / 2: dW + db /
    dX alone)."""
    In = C * HW
    dout_ld = O if dout_ld is None else dout_ld
    _need(dout.dtype == torch.float32 and dout_off + (rows - 1) * dout_ld + O <= dout.numel(), "hwc bwd dout")
    _need(feat.dtype == torch.bfloat16 and feat.numel() >= rows * In, "hwc bwd feat")
    _need(wp.dtype == torch.bfloat16 and wp.numel() >= O * In, "hwc bwd Wp")
    _need(dw.dtype == torch.float32 and dw.numel() >= O * In, "hwc bwd dW")
    _need(dx.dtype == torch.bfloat16 and dx.numel() >= rows * In, "hwc bwd dX")
    _need(db is None or db.numel() >= O, "hwc bwd db")
    nws = lib.avd_linear_hwc_ws_elems(rows, O, In)
    ws = _gemm_workspace(dout.device, nws)
    part = {3: "", 2: "_dx", 1: "_dw"}[which]
    nb = {3: 4 * 2 * rows * O + 2 * 2 * rows * In + 2 * O * In + 4 * O * In,
          2: 4 * rows * O + 2 * rows * In + 2 * O * In, 1: 4 * rows * O + 2 * rows * In + 4 * O * In}[which]
    _timed(f"linear_bwd_hwc{part}[{rows}x{O}x{In}]", nb, (4 if which == 3 else 2) * rows * O * In,
           lambda: call("avd_linear_bwd_hwc", rows, O, C, HW, dout.data_ptr() + 4 * dout_off, dout_ld,
                        p(feat), p(wp), p(dw), p(db), p(dx), which, p(ws), nws, stream()))


# ---------------------------------------------------------------- channels-last conv blocks
def cl_weight_elems(Cout, Cin, K, dgrad):
    return lib.avd_cl_weight_elems(Cout, Cin, K, int(dgrad))


def cl_weight_layout(w, wk, dgrad):
    """w [Cout,Cin,K,K] f32 -> MFMA layout in wk's dtype (forward, or input-grad if dgrad)."""
    Cout, Cin, K, _ = w.shape
    _need(w.dtype == torch.float32 and wk.numel() >= cl_weight_elems(Cout, Cin, K, dgrad), "cl wk")
    call("avd_cl_weight_layout", p(w), p(wk), dtcode(wk), Cout, Cin, K, int(dgrad), stream())


def cl_weight_layout_batch(entries):
    """entries: [(w f32 [Cout,Cin,K,K], wk, dgrad)] (<= 16, one dtype) -> one launch
    (avd_cl_weight_layout_batch)."""
    import ctypes as _ct
    n = len(entries)
    _need(0 < n <= 16, "weight layout batch size")
    dt = entries[0][1].dtype
    for w, wk, dg in entries:
        Co, Ci, K, _ = w.shape
        _need(w.dtype == torch.float32 and w.is_contiguous(), "layout batch w")
        _need(wk.dtype == dt and wk.numel() >= cl_weight_elems(Co, Ci, K, dg), "layout batch wk")
    PA, IA = _ct.c_void_p * n, _ct.c_int * n
    ws = PA(*[w.data_ptr() for w, _, _ in entries])
    wks = PA(*[wk.data_ptr() for _, wk, _ in entries])
    co = IA(*[w.shape[0] for w, _, _ in entries])
    ci = IA(*[w.shape[1] for w, _, _ in entries])
    kk = IA(*[w.shape[2] for w, _, _ in entries])
    dg = IA(*[int(d) for _, _, d in entries])
    call("avd_cl_weight_layout_batch", n, ws, wks, co, ci, kk, dg, _DT[dt], stream())


def cl_stat_rows(Ho, Wo, B, K, Cin, Cout, dtype):
    return lib.avd_cl_stat_rows(Ho, Wo, B, K, Cin, Cout, _DT[dtype])


# ---- MX (block-scaled e4m3) conv forward + input gradient (config 5): include/avdino.h "MX"
def mx_weight_bytes(Cout, Cin, K, dgrad):
    return int(lib.avd_mx_weight_bytes(Cout, Cin, K, int(dgrad)))


def mx_scale_bytes(Cout, Cin, K, dgrad):
    return int(lib.avd_mx_scale_bytes(Cout, Cin, K, int(dgrad)))


def mx_weight_layout(w, wq, wsc, dgrad):
    """w f32 [Cout, Cin, K, K] -> e4m3 rows wq (uint8) + E8M0 block scales wsc (uint8)."""
    Cout, Cin, K, _ = w.shape
    _need(w.dtype == torch.float32 and w.is_contiguous(), "mx layout w")
    _need(wq.dtype == torch.uint8 and wq.numel() >= mx_weight_bytes(Cout, Cin, K, dgrad), "mx layout wq")
    _need(wsc.dtype == torch.uint8 and wsc.numel() >= mx_scale_bytes(Cout, Cin, K, dgrad), "mx layout wsc")
    call("avd_mx_weight_layout", p(w), p(wq), p(wsc), Cout, Cin, K, int(dgrad), stream())


def mx_weight_layout_batch(entries):
    """entries: [(w f32 [Cout,Cin,K,K], wq, wsc, dgrad)] (<= 16) -> one launch."""
    import ctypes as _ct
    n = len(entries)
    _need(0 < n <= 16, "mx layout batch size")
    for w, wq, wsc, dg in entries:
        Co, Ci, K, _ = w.shape
        _need(w.dtype == torch.float32 and w.is_contiguous(), "mx batch w")
        _need(wq.dtype == torch.uint8 and wq.numel() >= mx_weight_bytes(Co, Ci, K, dg), "mx batch wq")
        _need(wsc.dtype == torch.uint8 and wsc.numel() >= mx_scale_bytes(Co, Ci, K, dg), "mx batch wsc")
    PA, IA = _ct.c_void_p * n, _ct.c_int * n
    call("avd_mx_weight_layout_batch", n, PA(*[e[0].data_ptr() for e in entries]),
         PA(*[e[1].data_ptr() for e in entries]), PA(*[e[2].data_ptr() for e in entries]),
         IA(*[e[0].shape[0] for e in entries]), IA(*[e[0].shape[1] for e in entries]),
         IA(*[e[0].shape[2] for e in entries]), IA(*[int(e[3]) for e in entries]), stream())


def mx_conv_serves(Cin, H, Cout, K, pad, dgrad, N=None, B=None):
    """An MX kernel for this layer shape; with N (and B for a forward with BN partials) also
    that the strip size divides them (else the caller runs the bf16 kernels)."""
    ns = lib.avd_mx_conv_ns(Cin, H, H, Cout, K, pad, int(dgrad))
    if ns <= 0:
        return False
    return (N is None or N % ns == 0) and (B is None or B % ns == 0)


def mx_stat_rows(H, B, K, Cin, Cout, pad):
    return lib.avd_mx_stat_rows(H, H, B, K, Cin, Cout, pad)


def mx_conv_fwd(x, wq, wsc, bias, y, stats, N, B, Cin, H, W, Cout, K, pad, pivot=None):
    """bf16 NHWC x -> bf16 NHWC y on the block-scaled e4m3 MFMA (+bias, + BN partial rows
    [Cout][N/B][R][2], sums about ``pivot`` when given)."""
    Ho, Wo = H + 2 * pad - K + 1, W + 2 * pad - K + 1
    _need(H == W and mx_conv_serves(Cin, H, Cout, K, pad, 0), f"mx conv: no kernel for {Cin}->{Cout} @{H}")
    _need(x.dtype == y.dtype == torch.bfloat16, "mx conv dtypes (bf16 maps)")
    _need(x.numel() == N * H * W * Cin and y.numel() == N * Ho * Wo * Cout, "mx conv sizes")
    _need(wq.numel() >= mx_weight_bytes(Cout, Cin, K, 0) and wsc.numel() >= mx_scale_bytes(Cout, Cin, K, 0),
          "mx conv weights")
    if stats is not None:
        R = mx_stat_rows(H, B, K, Cin, Cout, pad)
        _need(R > 0 and stats.numel() >= Cout * (N // B) * R * 2, "mx conv stats size")
    _need(pivot is None or (stats is not None and pivot.numel() >= Cout and pivot.dtype == torch.float32),
          "mx conv pivot")
    nb = x.numel() * 2 + y.numel() * 2
    fl = 2 * y.numel() * Cin * K * K
    _timed(f"mx_conv_fwd[{N}x{H}x{W}x{Cin}->{Cout} k{K}p{pad}]", nb, fl,
           lambda: call("avd_mx_conv_fwd", p(x), p(wq), p(wsc), p(bias), p(pivot), p(y), p(stats),
                        N, B, Cin, H, W, Cout, K, pad, stream()))


def mx_conv_dgrad(dy, wq_d, wsc_d, dx, N, Cin, H, W, Cout, K, pad):
    Ho, Wo = H + 2 * pad - K + 1, W + 2 * pad - K + 1
    _need(H == W and mx_conv_serves(Cin, H, Cout, K, pad, 1), f"mx dgrad: no kernel for {Cin}->{Cout} @{H}")
    _need(dy.dtype == dx.dtype == torch.bfloat16, "mx dgrad dtypes (bf16 maps)")
    _need(dy.numel() == N * Ho * Wo * Cout and dx.numel() == N * H * W * Cin, "mx dgrad sizes")
    _need(wq_d.numel() >= mx_weight_bytes(Cout, Cin, K, 1) and wsc_d.numel() >= mx_scale_bytes(Cout, Cin, K, 1),
          "mx dgrad weights")
    nb = (dy.numel() + dx.numel()) * 2
    fl = 2 * N * Cin * H * W * Cout * K * K
    _timed(f"mx_conv_dgrad[{N}x{Ho}x{Wo}x{Cout}->{Cin} k{K}p{pad}]", nb, fl,
           lambda: call("avd_mx_conv_dgrad", p(dy), p(wq_d), p(wsc_d), p(dx), N, Cin, H, W, Cout, K,
                        pad, stream()))


def mx_wgrad_chunks(N, Cin, H, Cout, K, pad):
    return lib.avd_mx_wgrad_chunks(N, Cin, H, Cout, K, pad)


def mx_conv_wgrad(x, dy, parts, N, Cin, H, W, Cout, K, pad):
    """Per-slab weight-gradient partials [chunks][Cout][Cin][K][K] on the MX MFMA (sum: sum_rows)."""
    Ho, Wo = H + 2 * pad - K + 1, W + 2 * pad - K + 1
    nch = mx_wgrad_chunks(N, Cin, H, Cout, K, pad)
    _need(H == W and nch > 0, f"mx wgrad: no kernel for {Cin}->{Cout} @{H}")
    _need(x.dtype == dy.dtype == torch.bfloat16, "mx wgrad dtypes (bf16 maps)")
    _need(x.numel() == N * H * W * Cin and dy.numel() == N * Ho * Wo * Cout, "mx wgrad sizes")
    _need(parts.dtype == torch.float32 and parts.numel() >= nch * Cout * Cin * K * K, "mx wgrad parts")
    nb = (x.numel() + dy.numel()) * 2 + nch * Cout * Cin * K * K * 4
    fl = 2 * N * Ho * Wo * Cout * Cin * K * K
    _timed(f"mx_conv_wgrad[{N}x{H}x{W}x{Cin}->{Cout} k{K}p{pad}]", nb, fl,
           lambda: call("avd_mx_conv_wgrad", p(x), p(dy), p(parts), N, Cin, H, W, Cout, K, pad, stream()))


def cl_stat_pivot(Ho, Wo, B, K, Cin, Cout, dtype):
    return bool(lib.avd_cl_stat_pivot(Ho, Wo, B, K, Cin, Cout, _DT[dtype]))


def cl_conv_fwd(x, wk, bias, y, stats, N, B, Cin, H, W, Cout, K, pad, pivot=None):
    """NHWC conv (+bias) with fused BN partial sums: stats [Cout][N/B][R][2]; with ``pivot``
    [Cout] (where cl_stat_pivot) sums about it (avd_cl_conv_fwd_pv)."""
    Ho, Wo = H + 2 * pad - K + 1, W + 2 * pad - K + 1
    _need(x.numel() == N * H * W * Cin and y.numel() == N * Ho * Wo * Cout, "cl conv sizes")
    _need(x.dtype == y.dtype == wk.dtype, "cl conv dtypes")
    _need(wk.numel() >= cl_weight_elems(Cout, Cin, K, 0), "cl conv wk")
    if stats is not None:
        R = cl_stat_rows(Ho, Wo, B, K, Cin, Cout, x.dtype)
        _need(R > 0 and stats.numel() >= Cout * (N // B) * R * 2, "cl conv stats size")
    if pivot is not None:
        _need(stats is not None and pivot.numel() >= Cout and pivot.dtype == torch.float32 and
              cl_stat_pivot(Ho, Wo, B, K, Cin, Cout, x.dtype), "cl conv pivot")
    nb = x.numel() * x.element_size() + y.numel() * y.element_size()
    fl = 2 * N * Cout * Ho * Wo * Cin * K * K
    _timed(f"cl_conv_fwd[{N}x{H}x{W}x{Cin}->{Cout} k{K}p{pad} {x.dtype}]", nb, fl,
           lambda: call("avd_cl_conv_fwd_pv", p(x), p(wk), p(bias), p(pivot), p(y), p(stats), dtcode(x),
                        N, B, Cin, H, W, Cout, K, pad, stream()))


def cl_conv_dgrad(dy, wk_d, dx, N, Cin, H, W, Cout, K, pad):
    Ho, Wo = H + 2 * pad - K + 1, W + 2 * pad - K + 1
    _need(dy.numel() == N * Ho * Wo * Cout and dx.numel() == N * H * W * Cin, "cl dgrad sizes")
    _need(dy.dtype == dx.dtype == wk_d.dtype, "cl dgrad dtypes")
    _need(wk_d.numel() >= cl_weight_elems(Cout, Cin, K, 1), "cl dgrad wk")
    nb = (dy.numel() + dx.numel()) * dy.element_size()
    fl = 2 * N * Cin * H * W * Cout * K * K
    _timed(f"cl_conv_dgrad[{N}x{Ho}x{Wo}x{Cout}->{Cin} k{K}p{pad} {dy.dtype}]", nb, fl,
           lambda: call("avd_cl_conv_dgrad", p(dy), p(wk_d), p(dx), dtcode(dy), N, Cin, H, W, Cout,
                        K, pad, stream()))


def cl_wgrad_chunks(N, Cout, Cin, K):
    return lib.avd_cl_wgrad_chunks(N, Cout, Cin, K)


def cl_conv_wgrad(x, dy, parts, N, Cin, H, W, Cout, K, pad):
    """Per-sample-chunk weight-gradient slabs [chunks][Cout][Cin][K][K] (reduce: sum_rows)."""
    Ho, Wo = H + 2 * pad - K + 1, W + 2 * pad - K + 1
    _need(x.numel() == N * H * W * Cin and dy.numel() == N * Ho * Wo * Cout, "cl wgrad sizes")
    _need(x.dtype == dy.dtype, "cl wgrad dtypes")
    _need(parts.numel() >= cl_wgrad_chunks(N, Cout, Cin, K) * Cout * Cin * K * K, "cl wgrad parts")
    nb = x.numel() * x.element_size() + dy.numel() * dy.element_size()
    fl = 2 * dy.numel() * Cin * K * K
    _timed(f"cl_conv_wgrad[{N}x{H}x{W}x{Cin}->{Cout} k{K}p{pad} {x.dtype}]", nb, fl,
           lambda: call("avd_cl_conv_wgrad", p(x), p(dy), dtcode(x), p(parts), N, Cin, H, W, Cout,
                        K, pad, stream()))


def cl_bn_relu_pool(y, scale, shift, out, mode, N, B, C, H, W):
    """mode 0: NHWC pooled (y dtype); 1: GAP f32 [N,C]; 2: f32 (c,h,w)-flattened pooled map."""
    _need(y.numel() == N * H * W * C, "cl pool y")
    want = {0: N * (H // 2) * (W // 2) * C, 1: N * C, 2: N * C * (H // 2) * (W // 2)}[mode]
    _need(out.numel() == want and (out.dtype == y.dtype if mode == 0 else out.dtype == torch.float32),
          "cl pool out")
    nb = y.numel() * y.element_size() + out.numel() * out.element_size()
    _timed(f"cl_bn_relu_pool[{N}x{H}x{W}x{C} m{mode} {y.dtype}]", nb, 0,
           lambda: call("avd_cl_bn_relu_pool", p(y), dtcode(y), p(scale), p(shift), p(out), mode, N,
                        B, C, H, W, stream()))


def cl_bn_bwd_rows(B, C, H, W, dtype):
    return lib.avd_cl_bn_bwd_rows(B, C, H, W, _DT[dtype])


def cl_bn_bwd_reduce(y, gout, mode, scale, shift, mean, invstd, parts, N, B, C, H, W):
    R = cl_bn_bwd_rows(B, C, H, W, y.dtype)
    _need(parts.numel() >= C * (N // B) * R * 2, "cl bwd parts")
    nb = y.numel() * y.element_size() + gout.numel() * gout.element_size()
    _timed(f"cl_bn_bwd_reduce[{N}x{H}x{W}x{C} m{mode} {y.dtype}]", nb, 0,
           lambda: call("avd_cl_bn_bwd_reduce", p(y), dtcode(y), p(gout), mode, p(scale), p(shift),
                        p(mean), p(invstd), p(parts), N, B, C, H, W, stream()))


def cl_bn_bwd_reduce_pooled(y, pooled, gout, mode, gamma, beta, mean, invstd, parts, N, B, C, H, W):
    """cl_bn_bwd_reduce's partial rows from the pooled output (xhat = (p - beta)/gamma at the
    argmax): reads pooled + gout instead of y + gout."""
    R = cl_bn_bwd_rows(B, C, H, W, y.dtype)
    _need(parts.numel() >= C * (N // B) * R * 2, "cl bwd parts")
    _need(mode in (0, 2) and pooled.numel() == gout.numel() and pooled.dtype == gout.dtype,
          "pooled bwd reduce layout")
    nb = pooled.numel() * pooled.element_size() + gout.numel() * gout.element_size()
    _timed(f"cl_bn_bwd_reduce_pooled[{N}x{H}x{W}x{C} m{mode} {y.dtype}]", nb, 0,
           lambda: call("avd_cl_bn_bwd_reduce_pooled", p(y), dtcode(y), p(pooled), p(gout), mode,
                        p(gamma), p(beta), p(mean), p(invstd), p(parts), N, B, C, H, W, stream()))


def counters_add(arena, idx, val):
    """arena[idx[i]] += val[i] (int64, distinct indices): avd_counters_add."""
    _need(arena.dtype == idx.dtype == val.dtype == torch.int64 and idx.numel() == val.numel(),
          "counters_add operands")
    call("avd_counters_add", p(arena), p(idx), p(val), idx.numel(), stream())


def cl_bn_bwd_apply(y, gout, mode, scale, shift, coef, dy, N, B, C, H, W):
    _need(dy.numel() == y.numel() and dy.dtype == y.dtype, "cl bwd dy")
    nb = 2 * y.numel() * y.element_size() + gout.numel() * gout.element_size()
    _timed(f"cl_bn_bwd_apply[{N}x{H}x{W}x{C} m{mode} {y.dtype}]", nb, 0,
           lambda: call("avd_cl_bn_bwd_apply", p(y), dtcode(y), p(gout), mode, p(scale), p(shift),
                        p(coef), p(dy), N, B, C, H, W, stream()))


def cl_apply_wgrad_slabs(dtype, N, Cin, H, W, Cout, K, pad):
    """Slabs of the fused BN-apply + wgrad first-layer kernel, 0 if the shape is not served."""
    return lib.avd_cl_apply_wgrad_slabs(1 if dtype == torch.bfloat16 else 0, N, Cin, H, W, Cout, K, pad)


def cl_bn_bwd_apply_wgrad(y, gout, scale, shift, coef, x, parts, N, B, Cin, H, W, Cout, K, pad):
    ns = cl_apply_wgrad_slabs(y.dtype, N, Cin, H, W, Cout, K, pad)
    _need(ns > 0 and parts.numel() >= ns * Cout * Cin * K * K, "apply+wgrad shape / slabs")
    _need(y.numel() == N * H * W * Cout and x.numel() == N * H * W * Cin, "apply+wgrad sizes")
    _need(gout.numel() == N * (H // 2) * (W // 2) * Cout and gout.dtype == y.dtype, "apply+wgrad gout")
    nb = (y.numel() + x.numel() + gout.numel()) * y.element_size()
    _timed(f"cl_bn_bwd_apply_wgrad[{N}x{H}x{W}x{Cin}->{Cout} k{K} {y.dtype}]", nb,
           2 * N * H * W * Cout * K * K,
           lambda: call("avd_cl_bn_bwd_apply_wgrad", p(y), p(gout), p(scale), p(shift), p(coef), p(x),
                        p(parts), dtcode(y), N, B, Cin, H, W, Cout, K, pad, stream()))


APPLY_GMAX = 8          # BN groups a fused BN-backward apply serves (csrc/bnapply.h)


def cl_layer_bwd_slabs(dtype, N, Cin, H, W, Cout, K, pad):
    """Slabs (= grid) of the fused layer backward (avd_cl_layer_bwd), 0 if the shape is not
    served (the audio conv2: 56^2, 8 -> 16, 5x5 pad 2, bf16)."""
    return lib.avd_cl_layer_bwd_slabs(_DT[dtype], N, Cin, H, W, Cout, K, pad)


def cl_layer_bwd(y, gout, scale, shift, coef, dy, x, wk_d, dx, parts, slabs, N, B, Cin, H, W, Cout,
                 K, pad):
    """The whole backward of one conv layer in one launch (lbwd.hip): dY formed from y and the
    pooled gradient (or taken from ``dy`` when y is None) in LDS only, dX (bit-identical to
    cl_conv_dgrad) and the weight-gradient slabs parts[slabs][Cout*Cin*K*K] (sum_rows)."""
    Ho = H + 2 * pad - K + 1
    _need(slabs > 0 and parts.dtype == torch.float32 and parts.numel() >= slabs * Cout * Cin * K * K,
          "layer bwd slabs / parts")
    _need(x.dtype == dx.dtype == torch.bfloat16 and x.numel() == N * H * W * Cin and dx.numel() == x.numel(),
          "layer bwd x / dx")
    _need(wk_d.numel() >= cl_weight_elems(Cout, Cin, K, 1), "layer bwd dgrad weights")
    if y is not None:
        _need(y.dtype == torch.bfloat16 and y.numel() == N * Ho * Ho * Cout, "layer bwd y")
        _need(gout.dtype == torch.bfloat16 and gout.numel() == N * (Ho // 2) * (Ho // 2) * Cout, "layer bwd gout")
        _need(N % B == 0 and N // B <= APPLY_GMAX, "layer bwd groups")
        nb = (y.numel() + gout.numel() + x.numel() + dx.numel()) * 2
    else:
        _need(dy is not None and dy.dtype == torch.bfloat16 and dy.numel() == N * Ho * Ho * Cout, "layer bwd dy")
        nb = (dy.numel() + x.numel() + dx.numel()) * 2
    nb += slabs * Cout * Cin * K * K * 4
    fl = 2 * 2 * N * Ho * Ho * Cout * Cin * K * K
    _timed(f"cl_layer_bwd[{N}x{H}x{W}x{Cin}->{Cout} k{K} {'apply' if y is not None else 'dy'}]", nb, fl,
           lambda: call("avd_cl_layer_bwd", p(y), p(gout), p(scale), p(shift), p(coef), p(dy), p(x),
                        p(wk_d), p(dx), p(parts), int(slabs), 1, N, B, Cin, H, W, Cout, K, pad, stream()))


C1_STATS, C1_APPLY, C1_REDUCE, C1_WGRAD, C1_REDUCE_MOMENTS = 0, 1, 2, 3, 4


def c1_moment_cols(Cout, K):
    """Columns of one pass-4 moment row (avd_cl_c1_moment_cols): Cout 16/32/64 sum dz xk
    [Cout][KK] + Gram rows [KK][KK+1]; the 5x5 audio conv1 (Cout 8) sum dz x25 [8][25] + Gram
    [25][25] + sum x25 [25]."""
    n = lib.avd_cl_c1_moment_cols(Cout, K)
    _need(n > 0, f"no pass-4 moments for Cout {Cout}")
    return n


def cl_c1_recompute_rows(pas, dtype, N, B, Cin, H, W, Cout, K, pad):
    return lib.avd_cl_c1_recompute_rows(pas, 1 if dtype == torch.bfloat16 else 0, N, B, Cin, H, W,
                                        Cout, K, pad)


def cl_c1_recompute(pas, x, wk, bias, N, B, Cin, H, W, Cout, K, pad, scale=None, shift=None,
                    mean=None, invstd=None, coef=None, gz=None, z=None, out=None):
    """Recompute-y passes of the audio first layer (include/avdino.h avd_cl_c1_recompute)."""
    rows = cl_c1_recompute_rows(pas, x.dtype, N, B, Cin, H, W, Cout, K, pad)
    _need(rows > 0 and x.numel() == N * H * W * Cin, "c1 recompute shape")
    G = N // B
    if pas in (C1_STATS, C1_REDUCE):
        _need(out is not None and out.numel() >= Cout * G * rows * 2, "c1 recompute rows")
    if pas == C1_REDUCE_MOMENTS:
        _need(out is not None and out.numel() >= G * rows * (Cout * 2 + c1_moment_cols(Cout, K)),
              "c1 recompute rows + moments")
        _need(mean is not None and invstd is not None, "c1 recompute mean/invstd")
    if pas == C1_WGRAD:
        _need(out is not None and out.numel() >= rows * Cout * Cin * K * K, "c1 recompute slabs")
    npool = N * (H // 2) * (W // 2) * Cout
    if pas == C1_APPLY:
        _need(z is not None and z.numel() == npool and z.dtype == x.dtype, "c1 recompute z")
    if pas in (C1_REDUCE, C1_WGRAD, C1_REDUCE_MOMENTS):
        _need(gz is not None and gz.numel() == npool and gz.dtype == x.dtype, "c1 recompute gz")
    nb = x.numel() * x.element_size() + (npool * 2 if pas != C1_STATS else 0)
    name = ["stats", "apply", "reduce", "wgrad", "reduce_moments"][pas]
    # MFMA work: the y recompute; the weight-gradient passes also dY x (or dz x), and pass 4 the
    # patch Gram matrix (KK x (KK + 1) per output pixel, the ones column included)
    KK = K * K
    fl = 2 * N * H * W * (Cout * KK * (2 if pas in (C1_WGRAD, C1_REDUCE_MOMENTS) else 1) +
                          (KK * (KK + 1) if pas == C1_REDUCE_MOMENTS else 0))
    _timed(f"cl_c1_recompute_{name}[{N}x{H}x{W}x{Cin}->{Cout} k{K}]", nb, fl,
           lambda: call("avd_cl_c1_recompute", pas, p(x), p(wk), p(bias), p(scale), p(shift), p(mean),
                        p(invstd), p(coef), p(gz), p(z), p(out), dtcode(x), N, B, Cin, H, W, Cout, K,
                        pad, stream()))


def cl_c1_recompute_combine(moments, coef, wk, bias, dw, G, Cout, K=None):
    """dW of a first layer from pass 4's row-summed moments (avd_cl_c1_recompute_combine): the
    3x3 / 5x5 layers (Cout 16/32/64) and the 5x5 audio conv1 (Cout 8)."""
    K = (5 if Cout == 8 else 3) if K is None else K
    _need(moments.numel() >= G * c1_moment_cols(Cout, K) and coef.numel() >= G * Cout * 3 and
          dw.numel() >= Cout * K * K, "c1 recompute combine shape")
    call("avd_cl_c1_recompute_combine", p(moments), p(coef), p(wk), p(bias), p(dw), G, Cout, K, stream())


# ---- the audio conv1 backward routed by forward codes (include/avdino.h avd_cl_c1_*codes*)
def c1_codes_rows(N, B, H, W):
    """Rows per BN group of avd_cl_c1_moments_codes (0 = shape not served)."""
    return lib.avd_cl_c1_codes_rows(N, B, H, W)


def c1_codes_cols():
    return lib.avd_cl_c1_codes_cols()


def c1_apply_codes(x, wk, bias, scale, shift, z, codes, N, B, H, W):
    """BN -> ReLU -> 2x2 max-pool of the recomputed conv1 output (avd_cl_c1_recompute pass 1)
    plus the routing codes [N, H/2, W/2] (int32 storage of the u32 nibble words)."""
    npool = N * (H // 2) * (W // 2)
    _need(c1_codes_rows(N, B, H, W) > 0 and x.numel() == N * H * W and x.dtype == torch.bfloat16,
          "c1 codes shape")
    _need(z.numel() == npool * 8 and z.dtype == x.dtype, "c1 codes z")
    _need(codes.numel() >= npool and codes.element_size() == 4, "c1 codes buffer")
    _timed(f"c1_apply_codes[{N}x{H}x{W}x1->8 k5]", x.numel() * 2 + npool * 20, 2 * N * H * W * 8 * 25,
           lambda: call("avd_cl_c1_apply_codes", p(x), p(wk), p(bias), p(scale), p(shift), p(z),
                        p(codes), N, B, H, W, stream()))


def c1_moments_codes(x, gz, codes, out, N, B, H, W):
    """One pass over x, the pooled gradient and the codes -> moment rows [R][G][MOMC]."""
    R = c1_codes_rows(N, B, H, W)
    npool = N * (H // 2) * (W // 2)
    _need(R > 0 and x.numel() == N * H * W and x.dtype == torch.bfloat16, "c1 moments codes shape")
    _need(gz.numel() == npool * 8 and gz.dtype == x.dtype and codes.numel() >= npool, "c1 moments gz/codes")
    _need(out.numel() >= R * (N // B) * c1_codes_cols(), "c1 moments rows")
    # algorithmic work: dz x (8 x 25 per pixel pair, dense over the routed tile) + the patch Gram
    fl = 2 * N * H * W * (8 * 25 + 25 * 26)
    _timed(f"c1_moments_codes[{N}x{H}x{W}x1->8 k5]", x.numel() * 2 + npool * 20, fl,
           lambda: call("avd_cl_c1_moments_codes", p(x), p(gz), p(codes), p(out), N, B, H, W, stream()))


def c1_codes_combine(moments, wk, bias, gamma, mean, invstd, count, dw, dgamma, dbeta, dbias, coef, G):
    """bn1 backward + conv1 bias / weight gradients from the row-summed moments [G][MOMC]."""
    _need(moments.numel() >= G * c1_codes_cols() and dw.numel() >= 200, "c1 codes combine")
    call("avd_cl_c1_codes_combine", p(moments), p(wk), p(bias), p(gamma), p(mean), p(invstd), int(count),
         p(dw), p(dgamma), p(dbeta), p(dbias), p(coef), G, stream())


# ---- the audio conv1's statistics from its patch Gram (include/avdino.h avd_cl_c1_gram*)
def c1_gram_cols():
    return lib.avd_cl_c1_gram_cols()


def c1_gram(x, out, N, B, H, W):
    """Patch Gram + sums rows [R][G][650] of the audio conv1 input (R = c1_codes_rows)."""
    R = c1_codes_rows(N, B, H, W)
    _need(R > 0 and x.numel() == N * H * W and x.dtype == torch.bfloat16, "c1 gram shape")
    _need(out.numel() >= R * (N // B) * c1_gram_cols(), "c1 gram rows")
    _timed(f"c1_gram[{N}x{H}x{W}x1 k5]", x.numel() * 2, 2 * N * H * W * 26 * 26,
           lambda: call("avd_cl_c1_gram", p(x), p(out), N, B, H, W, stream()))


def c1_gram_finalize(gram, wk, bias, gamma, beta, count, mean, invstd, scale, shift, rm=None, rv=None,
                     G=1, eps=1e-5, momentum=0.1):
    _need(gram.numel() >= G * c1_gram_cols(), "c1 gram finalize")
    call("avd_cl_c1_gram_finalize", p(gram), p(wk), p(bias), p(gamma), p(beta), int(count), eps, momentum,
         p(mean), p(invstd), p(scale), p(shift), p(rm), p(rv), G, stream())


def c1_moments_codes_ng(x, gz, codes, out, N, B, H, W):
    """The routed backward's M and sum dz only (MOMC rows, Gram / S slots zero)."""
    R = c1_codes_rows(N, B, H, W)
    npool = N * (H // 2) * (W // 2)
    _need(R > 0 and x.numel() == N * H * W and x.dtype == torch.bfloat16, "c1 moments ng shape")
    _need(gz.numel() == npool * 8 and gz.dtype == x.dtype and codes.numel() >= npool, "c1 moments ng gz/codes")
    _need(out.numel() >= R * (N // B) * c1_codes_cols(), "c1 moments ng rows")
    _timed(f"c1_moments_codes_ng[{N}x{H}x{W}x1->8 k5]", x.numel() * 2 + npool * 20, 2 * N * H * W * 8 * 26,
           lambda: call("avd_cl_c1_moments_codes_ng", p(x), p(gz), p(codes), p(out), N, B, H, W, stream()))


def c1_codes_combine_gram(moments, gram, wk, bias, gamma, mean, invstd, count, dw, dgamma, dbeta, dbias,
                          coef, G):
    _need(moments.numel() >= G * c1_codes_cols() and gram.numel() >= G * c1_gram_cols() and dw.numel() >= 200,
          "c1 codes combine gram")
    call("avd_cl_c1_codes_combine_gram", p(moments), p(gram), p(wk), p(bias), p(gamma), p(mean), p(invstd),
         int(count), p(dw), p(dgamma), p(dbeta), p(dbias), p(coef), G, stream())


# ---- the routed 3x3 first layer (include/avdino.h avd_cl_c1r3_*: SimCLR / unimodal conv1)
def c1r3_codes_rows(N, B, H, W, Cout=32):
    """Rows per BN group of avd_cl_c1r3_moments_codes (0 = shape not served)."""
    return lib.avd_cl_c1r3_codes_rows(N, B, H, W, Cout)


def c1r3_codes_cols(Cout=32):
    return lib.avd_cl_c1r3_codes_cols(Cout)


def c1r3_apply_codes(x, wk, bias, scale, shift, z, codes, N, B, H, W, Cout=32):
    """BN -> ReLU -> 2x2 max-pool of the recomputed 3x3 conv1 output (c1r3 pass 1, same pooled
    map) plus the routing codes [N, H/2, W/2, Cout/4] (int16 storage of the u16 nibble words)."""
    npool = N * (H // 2) * (W // 2)
    _need(c1r3_codes_rows(N, B, H, W, Cout) > 0 and x.numel() == N * H * W and x.dtype == torch.bfloat16,
          "c1r3 codes shape")
    _need(z.numel() == npool * Cout and z.dtype == x.dtype, "c1r3 codes z")
    _need(codes.numel() >= npool * Cout // 4 and codes.element_size() == 2, "c1r3 codes buffer")
    _timed(f"c1r3_apply_codes[{N}x{H}x{W}x1->{Cout} k3]", x.numel() * 2 + npool * Cout * 2 + npool * Cout // 2,
           2 * N * H * W * Cout * 9,
           lambda: call("avd_cl_c1r3_apply_codes", p(x), p(wk), p(bias), p(scale), p(shift), p(z),
                        p(codes), N, B, H, W, Cout, stream()))


def c1r3_moments_codes(x, wk, gz, codes, out, N, B, H, W, Cout=32):
    """One pass over x, the pooled gradient and the codes -> moment rows [R][G][cols]."""
    R = c1r3_codes_rows(N, B, H, W, Cout)
    npool = N * (H // 2) * (W // 2)
    _need(R > 0 and x.numel() == N * H * W and x.dtype == torch.bfloat16, "c1r3 moments codes shape")
    _need(gz.numel() == npool * Cout and gz.dtype == x.dtype and codes.numel() >= npool * Cout // 4,
          "c1r3 moments gz/codes")
    _need(out.numel() >= R * (N // B) * c1r3_codes_cols(Cout), "c1r3 moments rows")
    fl = 2 * N * H * W * (Cout * 10 + 10 * 10)
    _timed(f"c1r3_moments_codes[{N}x{H}x{W}x1->{Cout} k3]",
           x.numel() * 2 + npool * Cout * 2 + npool * Cout // 2, fl,
           lambda: call("avd_cl_c1r3_moments_codes", p(x), p(wk), p(gz), p(codes), p(out), N, B, H, W,
                        Cout, stream()))


def c1r3_codes_combine(moments, wk, bias, gamma, mean, invstd, count, dw, dgamma, dbeta, dbias, coef, G,
                       Cout=32):
    _need(moments.numel() >= G * c1r3_codes_cols(Cout) and dw.numel() >= Cout * 9 and G <= 32,
          "c1r3 codes combine")
    call("avd_cl_c1r3_codes_combine", p(moments), p(wk), p(bias), p(gamma), p(mean), p(invstd),
         int(count), p(dw), p(dgamma), p(dbeta), p(dbias), p(coef), G, Cout, stream())


# ---- the image conv1 backward routed by forward codes (include/avdino.h avd_cl_c1r5_*)
def c1r5_codes_rows(N, B, H, W):
    """Rows per BN group of avd_cl_c1r5_moments_codes (0 = shape not served)."""
    return lib.avd_cl_c1r5_codes_rows(N, B, H, W)


def c1r5_codes_cols():
    return lib.avd_cl_c1r5_codes_cols()


def c1r5_serves(N, B, H, W):
    """The pixel-major image conv1 passes (avd_cl_c1r5_stats / _apply_codes) serve this shape."""
    return lib.avd_cl_c1r5_stats_rows(N, B, H, W) > 0


def c1r5_stats_rows(N, B, H, W):
    return lib.avd_cl_c1r5_stats_rows(N, B, H, W)


def c1r5_stats(x, wk, bias, out, N, B, H, W):
    """BN partial sums [32][G][R][2] of the recomputed image conv1 output (bf16 y)."""
    R = c1r5_stats_rows(N, B, H, W)
    _need(R > 0 and x.numel() == N * H * W and x.dtype == torch.bfloat16, "c1r5 stats shape")
    _need(out.numel() >= 32 * (N // B) * R * 2, "c1r5 stats rows")
    _timed(f"c1r5_stats[{N}x{H}x{W}x1->32 k5]", x.numel() * 2, 2 * N * H * W * 32 * 25,
           lambda: call("avd_cl_c1r5_stats", p(x), p(wk), p(bias), p(out), N, B, H, W, stream()))


def c1r5_apply_codes(x, wk, bias, scale, shift, z, codes, N, B, H, W):
    """BN -> ReLU -> 2x2 max-pool of the recomputed image conv1 output (bit-identical to c1r3
    pass 1) plus, when ``codes`` is given, the routing codes [N, H/2, W/2, 8] (int16 storage of
    the u16 nibble words)."""
    npool = N * (H // 2) * (W // 2)
    _need(c1r5_serves(N, B, H, W) and x.numel() == N * H * W and x.dtype == torch.bfloat16,
          "c1r5 apply shape")
    _need(z.numel() == npool * 32 and z.dtype == x.dtype, "c1r5 apply z")
    if codes is not None:
        _need(codes.numel() >= npool * 8 and codes.element_size() == 2, "c1r5 codes buffer")
    name = "c1r5_apply_codes" if codes is not None else "c1r5_apply"
    _timed(f"{name}[{N}x{H}x{W}x1->32 k5]", x.numel() * 2 + npool * (80 if codes is not None else 64),
           2 * N * H * W * 32 * 25,
           lambda: call("avd_cl_c1r5_apply_codes", p(x), p(wk), p(bias), p(scale), p(shift), p(z),
                        p(codes), N, B, H, W, stream()))


def c1r5_moments_codes(x, gz, codes, out, N, B, H, W):
    """One pass over x, the pooled gradient and the codes -> moment rows [R][G][cols]."""
    R = c1r5_codes_rows(N, B, H, W)
    npool = N * (H // 2) * (W // 2)
    _need(R > 0 and x.numel() == N * H * W and x.dtype == torch.bfloat16, "c1r5 moments codes shape")
    _need(gz.numel() == npool * 32 and gz.dtype == x.dtype and codes.numel() >= npool * 8,
          "c1r5 moments gz/codes")
    _need(out.numel() >= R * (N // B) * c1r5_codes_cols(), "c1r5 moments rows")
    # algorithmic work: dz x (32 x 26 per pixel, dense over the routed map) + the patch Gram
    fl = 2 * N * H * W * (32 * 26 + 26 * 26)
    _timed(f"c1r5_moments_codes[{N}x{H}x{W}x1->32 k5]", x.numel() * 2 + npool * 80, fl,
           lambda: call("avd_cl_c1r5_moments_codes", p(x), p(gz), p(codes), p(out), N, B, H, W, stream()))


def c1r5_codes_combine(moments, wk, bias, gamma, mean, invstd, count, dw, dgamma, dbeta, dbias, coef, G):
    """bn1 backward + image conv1 bias / weight gradients from the row-summed moments."""
    _need(moments.numel() >= G * c1r5_codes_cols() and dw.numel() >= 800 and G <= 32, "c1r5 codes combine")
    call("avd_cl_c1r5_codes_combine", p(moments), p(wk), p(bias), p(gamma), p(mean), p(invstd),
         int(count), p(dw), p(dgamma), p(dbeta), p(dbias), p(coef), G, stream())


_SUM_WS = {}
_SUM_SPLIT = True      # row chunks in parallel (False: one pass)


def sum_rows(x, rows, cols, out, accumulate=0, ld=None, off=0):
    """out[c] (+)= sum_r x[off + r*ld + c]: avd_sum_rows_split (row chunks in parallel, then
    the chunk partials in fixed order) with a per-(device, stream) scratch."""
    ld = cols if ld is None else ld
    _need(off + (rows - 1) * ld + cols <= x.numel() and out.numel() >= cols, "sum_rows bounds")
    if not _SUM_SPLIT:
        call("avd_sum_rows", x.data_ptr() + 4 * off, rows, cols, ld, p(out), accumulate, stream())
        return
    n = lib.avd_sum_rows_chunks(rows, cols) * cols
    key = (x.device, torch.cuda.current_stream(x.device).cuda_stream)
    w = _SUM_WS.get(key)
    if w is None or w.numel() < n:
        w = _SUM_WS[key] = torch.empty(max(n, 1 << 16), device=x.device, dtype=torch.float32)
        bump_alloc_epoch()
    call("avd_sum_rows_split", x.data_ptr() + 4 * off, rows, cols, ld, p(out), accumulate, p(w),
         w.numel(), stream())


def colstats_parts(rows_per_group):
    return lib.avd_colstats_parts(rows_per_group)


def colstats(x, rows, G, C, parts, pivot=None):
    call("avd_colstats", p(x), rows, G, C, p(parts), p(pivot), stream())


def act_fwd(x, out, act, scale, shift, rows, G, C, drop_p, seed, seed_off=None):
    """seed_off: optional device u64 [1] added to seed (the engine's StepState.seed_off)."""
    if seed_off is None:
        call("avd_act_fwd", p(x), p(out), act, p(scale), p(shift), rows, G, C, drop_p, seed, stream())
    else:
        call("avd_act_fwd_dev", p(x), p(out), act, p(scale), p(shift), rows, G, C, drop_p, seed,
             p(seed_off), stream())


def act_bwd(x, dout, dx, act, scale, shift, rows, G, C, drop_p, seed, seed_off=None):
    if seed_off is not None:
        call("avd_act_bwd_dev", p(x), p(dout), p(dx), act, p(scale), p(shift), rows, G, C, drop_p,
             seed, p(seed_off), stream())
        return
    call("avd_act_bwd", p(x), p(dout), p(dx), act, p(scale), p(shift), rows, G, C, drop_p, seed,
         stream())


def bn1d_act_bwd_reduce(x, dout, dz, scale, shift, mean, invstd, rows, G, C, drop_p, seed, parts,
                        seed_off=None):
    """act_bwd(act=1) + bn1d_bwd_reduce in one launch (avd_bn1d_act_bwd_reduce; bit-identical)."""
    call("avd_bn1d_act_bwd_reduce", p(x), p(dout), p(dz), p(scale), p(shift), p(mean), p(invstd),
         rows, G, C, drop_p, seed, p(seed_off) if seed_off is not None else None, p(parts), stream())


def bn1d_bwd_reduce(x, dz, mean, invstd, rows, G, C, parts):
    call("avd_bn1d_bwd_reduce", p(x), p(dz), p(mean), p(invstd), rows, G, C, p(parts), stream())


def bn1d_bwd_apply(x, dz, coef, dx, rows, G, C):
    call("avd_bn1d_bwd_apply", p(x), p(dz), p(coef), p(dx), rows, G, C, stream())


# ---------------------------------------------------------------- losses
def dino_loss(s, t_raw, center, V, T, B, P, tau_s, tau_t, center_m, center_teacher, loss_parts,
              ds, center_new, work):
    _need(work.numel() >= (B + T * B) * P, "dino work")
    call("avd_dino_loss", p(s), p(t_raw), p(center), V, T, B, P, tau_s, tau_t, center_m,
         int(center_teacher), p(loss_parts), p(ds), p(center_new), p(work), stream())


def mse_loss(a, b, B, P, loss_parts, da, db):
    call("avd_mse_loss", p(a), p(b), B, P, p(loss_parts), p(da), p(db), stream())


def l2norm_fwd(x, y, norms, rows, P):
    call("avd_l2norm_fwd", p(x), p(y), p(norms), rows, P, stream())


def l2norm_bwd(y, norms, dy, dx, rows, P):
    call("avd_l2norm_bwd", p(y), p(norms), p(dy), p(dx), rows, P, stream())


def softmax_xent(logits, ld, R, C, targets, target_mode, col_major, mask_diag, gscale, loss_parts,
                 dlogits, ldd, accumulate, tgt_off=0, mask_off=None):
    """mask_diag masks column r (+ mask_off when given); tgt_off shifts target_mode 1."""
    if mask_off is None:
        mask_off = 0 if mask_diag else -1
    call("avd_softmax_xent", p(logits), ld, R, C, p(targets), target_mode, int(tgt_off),
         int(col_major), int(mask_off), gscale, p(loss_parts), p(dlogits), ldd, int(accumulate),
         stream())


def lds_poison():
    """Test hook (avd_lds_poison): fill the LDS of every CU with NaN bit patterns, so a kernel
    launched after it that reads LDS it never wrote sees NaN instead of a benign leftover
    (tools/lds_poison.py)."""
    call("avd_lds_poison", stream())


def xent_fused_ws(R, C, P):
    n = lib.avd_xent_fused_ws(R, C, P)
    _need(n > 0, f"fused softmax-CE: P must be 128 or 256 (got {P})")
    return n


def xent_fused(q, k, R, C, P, Bh, tgt, msk, inv_t, gscale, loss, dq, dk, ws):
    """Softmax cross-entropy over S = inv_t q k^T with per-half targets / masks, loss rows and
    both gradients, without materialising S (avd_xent_fused, xent.hip; bf16 MFMA)."""
    for t, n in ((q, R * P), (k, C * P), (dq, R * P), (dk, C * P), (loss, R)):
        _need(t.dtype == torch.float32 and t.is_contiguous() and t.numel() >= n, "xent operand")
    _need(ws.dtype == torch.float32 and ws.numel() >= xent_fused_ws(R, C, P), "xent workspace")
    fl = 4 * 2 * R * C * P
    _timed(f"xent_fused[{R}x{C}x{P}]", 4 * (2 * R * P + 2 * C * P + R), fl,
           lambda: call("avd_xent_fused", p(q), p(k), R, C, P, Bh, int(tgt[0]), int(tgt[1]), int(msk[0]),
                        int(msk[1]), inv_t, gscale, p(loss), p(dq), p(dk), p(ws), ws.numel(), stream()))


def cosine_consistency(emb, V, B, D, alpha, loss_parts, demb):
    _need(emb.numel() >= V * B * D and (demb is None or demb.numel() >= V * B * D)
          and (loss_parts is None or loss_parts.numel() >= B), "cosine consistency shapes")
    call("avd_cosine_consistency", p(emb), V, B, D, alpha, p(loss_parts), p(demb), stream())


# ---------------------------------------------------------------- optimiser / misc
def ema(teacher, student, n, m):
    call("avd_ema", p(teacher), p(student), n, m, stream())


def adam(p_, g, m, v, n, lr, b1, b2, eps, wd, bc1, bc2):
    call("avd_adam", p(p_), p(g), p(m), p(v), n, lr, b1, b2, eps, wd, bc1, bc2, stream())


def step_begin(t, hyp, seed_off, b1, b2, seed_stride):
    """Device step state: seed_off = t * stride; t += 1; hyp[1:3] = bias corrections of t."""
    _need(t.dtype == torch.int64 and hyp.dtype == torch.float32 and hyp.numel() >= 3, "step state")
    call("avd_step_begin", p(t), p(hyp), p(seed_off), float(b1), float(b2), seed_stride, stream())


def adam_dev(p_, g, m, v, n, hyp, b1, b2, eps, wd, decoupled=False):
    """Adam / AdamW reading lr and the bias corrections from the device step state hyp."""
    _need(p_.numel() >= n and g.numel() >= n and hyp.numel() >= 3, "adam_dev sizes")
    call("avd_adamw_dev" if decoupled else "avd_adam_dev", p(p_), p(g), p(m), p(v), n, p(hyp), b1, b2,
         eps, wd, stream())


def adamw(p_, g, m, v, n, lr, b1, b2, eps, wd, bc1, bc2):
    call("avd_adamw", p(p_), p(g), p(m), p(v), n, lr, b1, b2, eps, wd, bc1, bc2, stream())


def bn_eval_coef(gamma, beta, rm, rv, scale, shift, eps=1e-5):
    C = gamma.numel()
    _need(all(t.numel() >= C for t in (beta, rm, rv, scale, shift)), "bn eval coef")
    call("avd_bn_eval_coef", p(gamma), p(beta), p(rm), p(rv), eps, C, p(scale), p(shift), stream())


def argmax_correct(logits, ld, R, C, targets, correct):
    _need(logits.numel() >= (R - 1) * ld + C and targets.numel() >= R and correct.numel() >= R,
          "argmax shapes")
    call("avd_argmax_correct", p(logits), ld, R, C, p(targets), p(correct), stream())


def argmax_rows(logits, ld, R, C, idx):
    _need(logits.numel() >= (R - 1) * ld + C and idx.numel() >= R and idx.dtype == torch.int64,
          "argmax_rows shapes")
    call("avd_argmax_rows", p(logits), ld, R, C, p(idx), stream())


def row_sqnorm(x, N, D, out):
    _need(x.dtype == torch.float32 and x.numel() >= N * D and out.numel() >= N, "row_sqnorm shapes")
    call("avd_row_sqnorm", p(x), N, D, p(out), stream())


def knn_select(S, ldS, xnorm, M, N, K, labels, C, nbr, pred, Q=None, X=None, D=0):
    """S [M, ldS] = -2 Q X^T (f32), xnorm [N], labels [N] int64 -> pred [M] int64 (+ nbr [M, K]);
    Q [M, D] / X [N, D]: re-rank the best 16 candidates by direct distance."""
    _need(Q is None or (Q.numel() >= M * D and X is not None and X.numel() >= N * D), "knn Q/X")
    _need(S.dtype == torch.float32 and S.numel() >= (M - 1) * ldS + N and xnorm.numel() >= N, "knn S")
    _need(labels.dtype == torch.int64 and labels.numel() >= N, "knn labels")
    _need(pred.dtype == torch.int64 and pred.numel() >= M, "knn pred")
    _need(nbr is None or (nbr.dtype == torch.int64 and nbr.numel() >= M * K), "knn nbr")
    _need(1 <= K <= 16 and K <= N and 1 <= C <= 64, "knn K <= 16, C <= 64")
    call("avd_knn_select", p(S), ldS, p(xnorm), M, N, K, p(Q), p(X), D, p(labels), C, p(nbr), p(pred),
         stream())


def axpy(y, x, a=1.0):
    """y += a*x (contiguous f32, same numel)."""
    _need(y.numel() == x.numel() and y.dtype == x.dtype == torch.float32, "axpy operands")
    call("avd_axpy", p(y), p(x), y.numel(), a, stream())


def sum_to(x, n, scale, out):
    call("avd_sum", p(x), n, scale, p(out), stream())


def stage_views(g, G, l, L, orig, B, HW, out):
    _need(g.numel() == B * G * HW and (l is None or l.numel() == B * L * HW), "stage views")
    _need(orig is None or orig.numel() == B * HW, "stage orig")
    _need(out.numel() == (G + L + (orig is not None)) * B * HW, "stage out")
    call("avd_stage_views", p(g), G, p(l), L, p(orig), B, HW, p(out), dtcode(out), stream())


AUG_REC = 28  # floats per (sample, view) record, include/avdino.h AVD_AUG_REC


def augment_views(src_u8, idx, lut, rec, gm, group, seed, V, H, W, out, order=0, kinds=None):
    """Device view augmentation (avd_augment_views_dt; with ``kinds``, the chain's stage kinds in
    application order, avd_augment_views_seq): src_u8 [N, H*W] u8, idx [B] int64, lut
    [256] f32, rec [B*V, AUG_REC] f32, gm [R, words] int32/uint32 or None, out f32 or bf16
    [B,V,H,W] (order 0) or [V,B,H,W] (order 1; a bf16 out may be a row range of the engine's
    staged view-major input).  Sample ids and bitmask rows are range-checked by the caller
    (avdino.augment.ViewAugmenter)."""
    B = idx.numel()
    _need(src_u8.dtype == torch.uint8 and src_u8.dim() == 2 and src_u8.shape[1] == H * W, "aug src")
    _need(idx.dtype == torch.int64 and lut.numel() == 256 and lut.dtype == torch.float32, "aug idx/lut")
    _need(rec.dtype == torch.float32 and rec.shape == (B * V, AUG_REC), "aug records")
    _need(out.dtype in (torch.float32, torch.bfloat16) and out.numel() == B * V * H * W, "aug out")
    for t in (src_u8, idx, lut, rec, out) + ((gm,) if gm is not None else ()):
        _need(t.is_contiguous() and t.device == out.device, "aug operands contiguous, one device")
    words = gm.shape[1] if gm is not None else 0
    if kinds is None:
        call("avd_augment_views_dt", p(src_u8), p(idx), src_u8.shape[0], B, V, H, W, p(lut), p(rec),
             p(gm), words, group, seed & (2**64 - 1), order, p(out), dtcode(out), stream())
        return
    import numpy as _np
    ks = _np.ascontiguousarray(kinds, _np.int32)
    _need(ks.ndim == 1 and ks.shape[0] <= AUG_MAX_STAGES, "aug stage kinds")
    call("avd_augment_views_seq", p(src_u8), p(idx), src_u8.shape[0], B, V, H, W, p(lut), p(rec),
         p(gm), words, group, seed & (2**64 - 1), order, ks.ctypes.data, ks.shape[0], p(out),
         dtcode(out), stream())


AUG_STAGE_F = 8       # floats per chain stage of avd_augment_records
AUG_MAX_STAGES = 9


def augment_records(stages, n, H, W, group, seed, rec, gm):
    """Device parameter draws (avd_augment_records): stages float32 numpy [S, 8] (host),
    rec f32 [n, AUG_REC] and gm int32 [n, words] (or None without grouped masking) on the
    device."""
    import numpy as _np
    st = _np.ascontiguousarray(stages, _np.float32)
    _need(st.ndim == 2 and st.shape[1] == AUG_STAGE_F and st.shape[0] <= AUG_MAX_STAGES, "aug stages")
    _need(rec.dtype == torch.float32 and rec.shape == (n, AUG_REC) and rec.is_contiguous(), "aug rec out")
    words = 0
    if gm is not None:
        _need(gm.dim() == 2 and gm.shape[0] == n and gm.is_contiguous(), "aug gm out")
        words = gm.shape[1]
    call("avd_augment_records", st.ctypes.data, st.shape[0], n, H, W, group, seed & (2**64 - 1),
         p(rec), p(gm), words, stream())


# ---------------------------------------------------------------- timeline marks (tools)
class Marks:
    """Phase marks of a step (avd_mark): ``mark(name)`` records the device real-time counter
    when the current stream reaches it.  Enabled by engine code through the module-level
    MARKS (None = off, no launch).  ``read()`` -> [(name, stream id, t_us)] of the last pass."""

    def __init__(self, device, cap=512):
        self.buf = torch.zeros(cap, dtype=torch.int64, device=device)
        self.names = []

    def mark(self, name):
        s = torch.cuda.current_stream()
        i = len(self.names)
        if i >= self.buf.numel():
            return
        self.names.append((name, s.cuda_stream))
        call("avd_mark", p(self.buf), i, s.cuda_stream)

    def reset(self):
        self.names = []

    def read(self):
        torch.cuda.synchronize()
        t = self.buf[:len(self.names)].cpu().tolist()
        t0 = min(t) if t else 0
        return [(n, s, (v - t0) / 100.0) for (n, s), v in zip(self.names, t)]


MARKS = None


def mark(name):
    if MARKS is not None:
        MARKS.mark(name)


def mark_reset():
    """Start of a (captured or eager) step: the marks are re-numbered from 0."""
    if MARKS is not None:
        MARKS.reset()
