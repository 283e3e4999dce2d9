"""The training-step engine: explicit forward and backward of the reference's multimodal-DINO
step over libavdino kernels (no autograd, no per-view Python loop, no per-parameter loops).

Reference step, multi_central with training_mode mse:
  MultiModalDINOWithMSELightning.training_step (dino.py:1214-1238)
    MultiModalDINO.forward (dino.py:655-727): student over 2 global + 4 local views, teacher
      over the global views (no grad, train mode), projections, centring, update_center
    + image/audio projection heads on the original image/audio (dino.py:1163-1171)
    dino_loss (822-854) + alpha * mse_loss (1193-1211)
    update_teacher (635-646)  <- before backward / Adam, so the EMA sees the pre-step student
  Lightning: zero_grad -> backward -> Adam.step (configure_optimizers 953-962)

MI355X-native restructuring (results identical up to fp32 rounding):
  * all views of a step go through each conv layer in ONE launch (N = views*B samples) with
    BatchNorm statistics kept per (view, channel): same math as the reference's per-view
    calls, one launch instead of V;
  * the student's original-image/audio pass of the MSE / InfoNCE / supervised heads shares
    those launches (one more BN group), and its gradient accumulates in the same wgrad;
  * cat() of image/audio features is a strided GEMM write; slices are pointer offsets;
  * EMA / Adam / grad all-reduce run on flat arenas (params.py).
"""

import torch

from . import contrastive, ops
from .capture import GraphedStep, host_point, new_event  # noqa: F401  (GraphedStep re-exported)
from .spec import HEAD_NAMES, MULTI_ENCODERS, PROJ_HIDDEN, UNI_ALIASES, UNI_ENCODERS

F32 = torch.float32
# early gradient buckets at a host point inside the step (False: one all-reduce after the step)
BUCKETS = True


class Workspace:
    """Named device scratch buffers, grown on demand and reused across steps.  Every
    (re)allocation bumps this workspace's own ``epoch``, so graphs captured over its old
    buffers are retired (GraphedStep ``deps``) -- and only those: a probe's or a loss helper's
    workspace growing does not retire an engine's graphs.

    Cross-stream safety.  A workspace buffer is used by several streams (main,
    side, weight-gradient, data), but the caching allocator hands out memory in the order of
    the ALLOCATING stream only: a new buffer may be a block that stream freed while kernels
    still queued on it use the block, and the buffer a regrowth drops may still be read by
    another stream.  So every (re)allocation outside a graph capture synchronises the device
    once the new buffer exists and before the old one is dropped; allocations happen only in
    warm-up steps and at shape changes, never in a steady-state step.  (Without this, the
    real-data prefetch's second staging set -- allocated on the main stream under step 0 and
    written on the data stream -- could land on a block step 0 was still using.)"""

    # bytes of canary after every buffer (tests / tools/dbg_guard.py: check_guards() names any
    # buffer whose writer ran past its end); 0 in production
    GUARD = 0
    CANARY = 0xA5

    def __init__(self, device):
        self.device = device
        self.bufs = {}
        self.guards = {}
        self.epoch = 0

    def get(self, name, numel, dtype=F32):
        b = self.bufs.get(name)
        if b is None or b.numel() < numel or b.dtype != dtype:
            n = max(numel, 1)
            es = torch.empty(0, dtype=dtype).element_size()
            g = -(-self.GUARD // es)
            full = torch.empty(n + g, dtype=dtype, device=self.device)
            nb = full[:n]
            if g:
                full.view(torch.uint8)[n * es:].fill_(self.CANARY)
                self.guards[name] = (full, n * es)
            if nb.is_cuda and not torch.cuda.is_current_stream_capturing():
                torch.cuda.synchronize(self.device)
            self.bufs[name] = b = nb
            self.epoch += 1
        return b[:numel]

    def check_guards(self):
        """[(buffer name, first clobbered byte past its end, clobbered bytes)] (GUARD > 0)."""
        bad = []
        for name, (full, nb) in self.guards.items():
            gz = full.view(torch.uint8)[nb:]
            hit = (gz != self.CANARY).nonzero()
            if hit.numel():
                bad.append((name, int(hit[0]), int(hit.numel())))
        return bad

    def nbytes(self):
        return sum(b.numel() * b.element_size() for b in self.bufs.values())


# ============================================================================ conv stacks
def launch_layouts(batch, mxb):
    """Every bf16 conv weight layout in one launch (16 per launch) and every MX one in another."""
    for j in range(0, len(batch), 16):
        ops.cl_weight_layout_batch(batch[j:j + 16])
    for j in range(0, len(mxb), 16):
        ops.mx_weight_layout_batch(mxb[j:j + 16])


class ConvBranch:
    """[conv -> BN(train, per group) -> ReLU -> maxpool2] x L (+ (c,h,w) flatten or GAP) over
    channels-last maps, forward and backward (CentralUnimodalImage/Audio.forward,
    unimodal.py:127-221; the 3x3 CNNs, dino.py:18-73).  Same kernels for f32 (parity, f32
    MFMA) and bf16 (bench) storage; the final features are f32 [N, F] in the reference's
    flatten order, or -- ``hwc`` (bf16, flatten tails) -- the last pooled map itself, bf16 NHWC,
    for the encoder Linear's (h, w, c)-ordered kernels (avd_linear_*_hwc)."""

    def __init__(self, stack, act_dtype, fp8=False, hwc=False):
        self.stack = stack
        self.act = act_dtype
        self.dims = stack.layer_dims()
        self.hwc = bool(hwc) and act_dtype == torch.bfloat16 and not stack.gap
        # fp8: the layers after the first run their forward, input gradient AND weight gradient
        # on the block-scaled e4m3 MFMA (config 5's "fp8 MFMA conv path", avd_mx_conv_*: both
        # operands quantised to e4m3 while staged, one E8M0 scale per strip / 32-k block); the
        # stored maps stay bf16, statistics and accumulators f32.  A layer whose strip size does
        # not divide the batch (an odd last batch) runs on the bf16 kernels.
        self.fp8 = bool(fp8) and act_dtype == torch.bfloat16

    # fp8 (config 5): a layer the fused bf16 layer backward serves (the audio conv2, 56^2) keeps
    # its input and weight gradient in bf16 through that one launch; its forward stays MX
    # (16.7-17.0 vs 17.4-17.8 ms per B = 4096 step, profiles/r6_ab_fp8_fused_bwd.txt)
    FP8_FUSED_BWD = True

    def _fused_bwd(self, i, N):
        ci, co, k, p = self.stack.convs[i]
        H = self.dims[i][0]
        return (self.FP8_FUSED_BWD and self.LAYER_BWD and i > 0
                and ops.cl_layer_bwd_slabs(self.act, N, ci, H, H, co, k, p) > 0)

    def _mx_ok(self, i, N, B=None, dgrad=False):
        """MX kernel for layer i's forward (B: the BN group size when it writes partials) or
        input gradient over N samples."""
        ci, co, k, p = self.stack.convs[i]
        return (self.fp8 and i > 0 and not (dgrad and self._fused_bwd(i, N))
                and ops.mx_conv_serves(ci, self.dims[i][0], co, k, p, dgrad, N, None if dgrad else B))

    def prepare(self, ws, store, tag, need_dgrad, N, B=None, launch=True):
        """MFMA weight layouts for this step (the weights change every step), per layer:
        (bf16 forward rows, bf16 dgrad rows, MX forward (e4m3 rows, scales), MX dgrad).
        B: BN group size of a training forward (None: eval, no partials).  launch=False: returns
        (layouts, bf16 batch entries, MX batch entries) for the caller to launch together with
        other branches' (``launch_layouts``)."""
        wts, batch, mxb = [], [], []
        for i, (ci, co, k, _p) in enumerate(self.stack.convs):
            w = store[self.stack.conv_keys[i] + ".weight"]
            wk = wd = q = qd = None
            if self._mx_ok(i, N, B):
                q = (ws.get(f"{tag}.wq{i}", ops.mx_weight_bytes(co, ci, k, 0), torch.uint8),
                     ws.get(f"{tag}.wqs{i}", ops.mx_scale_bytes(co, ci, k, 0), torch.uint8))
                mxb.append((w, q[0], q[1], 0))
            else:
                wk = ws.get(f"{tag}.wk{i}", ops.cl_weight_elems(co, ci, k, 0), self.act)
                batch.append((w, wk, 0))
            if need_dgrad and i > 0:
                if self._mx_ok(i, N, dgrad=True):
                    qd = (ws.get(f"{tag}.wqd{i}", ops.mx_weight_bytes(co, ci, k, 1), torch.uint8),
                          ws.get(f"{tag}.wqds{i}", ops.mx_scale_bytes(co, ci, k, 1), torch.uint8))
                    mxb.append((w, qd[0], qd[1], 1))
                else:
                    wd = ws.get(f"{tag}.wd{i}", ops.cl_weight_elems(co, ci, k, 1), self.act)
                    batch.append((w, wd, 1))
            wts.append((wk, wd, q, qd))
        if not launch:
            return wts, batch, mxb
        launch_layouts(batch, mxb)
        return wts

    def _conv_fwd(self, i, h, wt, bias, y, parts, N, B, pivot=None):
        ci, co, k, pad = self.stack.convs[i]
        H = self.dims[i][0]
        if wt[2] is not None:
            ops.mx_conv_fwd(h, wt[2][0], wt[2][1], bias, y, parts, N, B, ci, H, H, co, k, pad, pivot=pivot)
        else:
            ops.cl_conv_fwd(h, wt[0], bias, y, parts, N, B, ci, H, H, co, k, pad, pivot=pivot)

    def _conv_dgrad(self, i, dy, wt, dx, N):
        ci, co, k, pad = self.stack.convs[i]
        H = self.dims[i][0]
        if wt[3] is not None:
            ops.mx_conv_dgrad(dy, wt[3][0], wt[3][1], dx, N, ci, H, H, co, k, pad)
        else:
            ops.cl_conv_dgrad(dy, wt[1], dx, N, ci, H, H, co, k, pad)

    def _mx_wgrad(self, i, N):
        ci, co, k, p = self.stack.convs[i]
        return (self.fp8 and i > 0 and not self._fused_bwd(i, N)
                and ops.mx_wgrad_chunks(N, ci, self.dims[i][0], co, k, p) > 0)

    def _wgrad_chunks(self, i, N):
        ci, co, k, p = self.stack.convs[i]
        if self._mx_wgrad(i, N):
            return ops.mx_wgrad_chunks(N, ci, self.dims[i][0], co, k, p)
        return ops.cl_wgrad_chunks(N, co, ci, k)

    def _conv_wgrad(self, i, x, dy, wparts, N):
        ci, co, k, pad = self.stack.convs[i]
        H = self.dims[i][0]
        if self._mx_wgrad(i, N):
            ops.mx_conv_wgrad(x, dy, wparts, N, ci, H, H, co, k, pad)
        else:
            ops.cl_conv_wgrad(x, dy, wparts, N, ci, H, H, co, k, pad)

    def _stat_pivot(self, store, i, N, B):
        """The BN running mean as the statistics pivot where the producer takes one (the
        persistent mid layers: avd_cl_stat_pivot, and the MX kernels) -- None elsewhere."""
        ci, co, k, _p = self.stack.convs[i]
        Ho = self.dims[i][1]
        if not (self._mx_ok(i, N, B) or ops.cl_stat_pivot(Ho, Ho, B, k, ci, co, self.act)):
            return None
        return store[self.stack.bn_keys[i] + ".running_mean"]

    def _stat_rows(self, i, N, B):
        ci, co, k, p = self.stack.convs[i]
        H, Ho = self.dims[i][0], self.dims[i][1]
        if self._mx_ok(i, N, B):
            return ops.mx_stat_rows(H, B, k, ci, co, p)
        return ops.cl_stat_rows(Ho, Ho, B, k, ci, co, self.act)

    def _tail_mode(self):
        """Layout of the last block's pooled output: 1 = GAP f32, 2 = (c,h,w) flatten f32,
        0 = NHWC in the activation dtype (hwc)."""
        return 1 if self.stack.gap else (0 if self.hwc else 2)

    def feat_shape(self):
        """(channels, pooled pixels) of the last block: the hwc Linear's C and HW."""
        return self.stack.convs[-1][1], self.dims[-1][2] ** 2

    def forward(self, ws, store, tag, x, N, G, update_running=True, need_dgrad=False, wts=None):
        """x: staged input [N,H,W,1] (act dtype).  Returns (features [N, F], ctx): f32 in the
        reference's flatten order, or the NHWC pooled map (hwc).  wts: this call's layouts
        from prepare(..., launch=False), already launched."""
        B = N // G
        if wts is None:
            wts = self.prepare(ws, store, tag, need_dgrad, N, B)
        ctx = {"x": [x], "y": [], "stats": [], "wts": wts, "N": N, "G": G}
        h = x
        nl = len(self.stack.convs)
        for i, (ci, co, k, pad) in enumerate(self.stack.convs):
            H, Ho, Hp = self.dims[i]
            if i == 0 and nl > 1 and self._recompute_ok(N, B, ci, H, co, k, pad, need_dgrad):
                h = self._first_layer_recompute_fwd(ws, store, tag, ctx, h, N, G, B, update_running,
                                                    need_dgrad)
                ops.mark(f"{tag}.f{i}")
                continue
            R = self._stat_rows(i, N, B)
            y = ws.get(f"{tag}.y{i}", N * Ho * Ho * co, self.act)
            parts = ws.get("stat_parts", co * G * R * 2)
            pv = self._stat_pivot(store, i, N, B)
            self._conv_fwd(i, h, wts[i], store[self.stack.conv_keys[i] + ".bias"], y, parts, N, B, pv)
            st = ws.get(f"{tag}.bn{i}", 4 * G * co).view(4, G * co)
            bk = self.stack.bn_keys[i]
            ops.bn_finalize(parts, G, R, co, B * Ho * Ho, store[bk + ".weight"], store[bk + ".bias"],
                            st[0], st[1], st[2], st[3],
                            store[bk + ".running_mean"] if update_running else None,
                            store[bk + ".running_var"] if update_running else None,
                            pivot=pv, pivot_gs=0)
            if update_running:
                store.bump_nbt(bk + ".num_batches_tracked", G)
            ctx["y"].append(y)
            ctx["stats"].append(st)
            if i == nl - 1:
                mode = self._tail_mode()
                out = ws.get(f"{tag}.feat", N * co * (1 if mode == 1 else Hp * Hp), F32 if mode else self.act)
            else:
                mode = 0
                out = ws.get(f"{tag}.x{i + 1}", N * Hp * Hp * co, self.act)
            if (i == 0 and mode == 0 and self.RC_APPLY and self.act == torch.bfloat16 and
                    ops.cl_c1_recompute_rows(ops.C1_APPLY, self.act, N, B, ci, H, H, co, k, pad) > 0):
                # BN -> ReLU -> pool from the conv recomputed out of x (bit-identical y)
                ops.cl_c1_recompute(ops.C1_APPLY, h, wts[0][0], store[self.stack.conv_keys[0] + ".bias"],
                                    N, B, ci, H, H, co, k, pad, scale=st[2], shift=st[3], z=out)
            else:
                ops.cl_bn_relu_pool(y, st[2], st[3], out, mode, N, B, co, Ho, Ho)
            if i < nl - 1:
                ctx["x"].append(out)
            else:
                ctx["feat"] = out     # the tail's pooled output (the backward's BN reduce reads it)
            h = out
            ops.mark(f"{tag}.f{i}")
        return h.view(N, -1), ctx

    def forward_eval(self, ws, store, tag, x, N):
        """Eval-mode forward (nn.Module.eval(): BatchNorm from the running statistics, no
        statistics pass, nothing saved) -> features f32 [N, F]."""
        wts = self.prepare(ws, store, tag, False, N)
        h = x
        nl = len(self.stack.convs)
        for i, (ci, co, k, pad) in enumerate(self.stack.convs):
            H, Ho, Hp = self.dims[i]
            y = ws.get(f"{tag}.y{i}", N * Ho * Ho * co, self.act)
            self._conv_fwd(i, h, wts[i], store[self.stack.conv_keys[i] + ".bias"], y, None, N, N)
            bk = self.stack.bn_keys[i]
            coef = ws.get(f"{tag}.ev{i}", 2 * co).view(2, co)
            ops.bn_eval_coef(store[bk + ".weight"], store[bk + ".bias"], store[bk + ".running_mean"],
                             store[bk + ".running_var"], coef[0], coef[1])
            if i == nl - 1:
                mode = self._tail_mode()
                out = ws.get(f"{tag}.feat", N * co * (1 if mode == 1 else Hp * Hp), F32 if mode else self.act)
            else:
                mode = 0
                out = ws.get(f"{tag}.x{i + 1}", N * Hp * Hp * co, self.act)
            ops.cl_bn_relu_pool(y, coef[0], coef[1], out, mode, N, N, co, Ho, Ho)
            h = out
        return h.view(N, -1)

    # ---- first layer without a stored conv output (avd_cl_c1_recompute).  The route switches
    # below are plain class attributes (tests flip them to compare routes; nothing reads the
    # environment).
    # forwards without a backward (the teacher): y is never needed, so never stored -- stats
    # and apply passes recompute it from the 8x smaller input (r1_34: +1.5 % step rate)
    RC_NOGRAD = True
    # stored-y forward whose BN -> ReLU -> pool recomputes y from x instead of reading the
    # 1.44 GB it just wrote (bit-identical y; r1_34: +0.5 %)
    RC_APPLY = True
    # 3x3 first layers (the SimCLR / unimodal encoders): recompute passes c1r3_kernel, whose y
    # is one MFMA per 16 channels x 16 pixels from the staged input tile
    RECOMPUTE3 = True
    # their backward as one pass (avd_cl_c1_recompute pass 4) + a tiny combine: dW is linear in
    # dy = k1 dz + kx y + k0, so the pass accumulates sum dz x9 and the Gram matrix of x9
    RC_MOMENTS = True
    # the 5x5 audio conv1 in training: no stored y either -- its backward is the one moments
    # pass (x and the pooled gradient in, BN-backward sums + dW moments out) and a combine
    MOMENTS5 = True

    def _recompute_ok(self, N, B, ci, H, co, k, pad, need_dgrad=True):
        rc = (self.RECOMPUTE3 and k == 3) or (self.RC_NOGRAD and not need_dgrad)
        if not rc and self.MOMENTS5 and self.RC_MOMENTS and k == 5 and self.act == torch.bfloat16:
            rc = ops.cl_c1_recompute_rows(ops.C1_REDUCE_MOMENTS, self.act, N, B, ci, H, H, co, k, pad) > 0
        return (rc and self.act == torch.bfloat16 and
                ops.cl_c1_recompute_rows(ops.C1_STATS, self.act, N, B, ci, H, H, co, k, pad) > 0)

    # the 5x5 conv1 backwards from the forward's routing codes: the audio conv1 (1->8 at 112^2,
    # avd_cl_c1_moments_codes) and the image conv1 (1->32 at 28^2, avd_cl_c1r5_moments_codes);
    # False keeps the recomputing moments pass (pass 4) for both
    CODES = True

    # the image conv1's forward passes (statistics; BN -> ReLU -> pool [+ codes]) on the
    # pixel-major MFMA kernels of c1r5.hip (one pooling window per lane); False runs them on
    # c1r3 passes 0 / 1 instead (same pooled map; statistics summed in another order)
    PIXEL_MAJOR = True

    def _pixel_major(self, N, B):
        ci, co, k, pad = self.stack.convs[0]
        H = self.dims[0][0]
        return (self.PIXEL_MAJOR and (ci, co, k, pad) == (1, 32, 5, 2) and self.act == torch.bfloat16
                and ops.c1r5_serves(N, B, H, H))

    def _codes_ok(self, N, B, need_dgrad):
        """"audio" / "image" when the first layer's training backward is the routed moments pass,
        else None."""
        ci, co, k, pad = self.stack.convs[0]
        H = self.dims[0][0]
        if not (self.CODES and need_dgrad and self.act == torch.bfloat16):
            return None
        if (ci, co, k, pad) == (1, 8, 5, 2) and ops.c1_codes_rows(N, B, H, H) > 0:
            return "audio"
        if (ci, co, k, pad) == (1, 32, 5, 2) and ops.c1r5_codes_rows(N, B, H, H) > 0:
            return "image"
        if (ci, co, k, pad) == (1, 32, 3, 1) and self.CODES3 and ops.c1r3_codes_rows(N, B, H, H) > 0:
            return "c3"
        return None

    # the 3x3 first layers (SimCLR / unimodal encoders) routed the same way (avd_cl_c1r3_*);
    # False keeps the recomputing moments pass (c1r3 pass 4)
    CODES3 = True

    # the audio conv1's BN statistics from its patch Gram matrix (avd_cl_c1_gram) instead of a
    # recomputing statistics pass; False restores the latter
    GRAM = True

    def _gram_ok(self, N, B):
        ci, co, k, pad = self.stack.convs[0]
        H = self.dims[0][0]
        return (self.GRAM and (ci, co, k, pad) == (1, 8, 5, 2) and self.act == torch.bfloat16
                and ops.c1_codes_rows(N, B, H, H) > 0)

    def _first_layer_recompute_fwd(self, ws, store, tag, ctx, x, N, G, B, update_running,
                                   need_dgrad=True):
        ci, co, k, pad = self.stack.convs[0]
        H, Ho, Hp = self.dims[0]
        wk = ctx["wts"][0][0]
        bias = store[self.stack.conv_keys[0] + ".bias"]
        pm = self._pixel_major(N, B)
        st = ws.get(f"{tag}.bn0", 4 * G * co).view(4, G * co)
        bk = self.stack.bn_keys[0]
        rm = store[bk + ".running_mean"] if update_running else None
        rv = store[bk + ".running_var"] if update_running else None
        if self._gram_ok(N, B):
            # statistics of y = w . x25 + b from the patch Gram (one MFMA pass over x, no y);
            # the routed backward reuses the Gram
            R, gc = ops.c1_codes_rows(N, B, H, H), ops.c1_gram_cols()
            gparts = ws.get("c1_gram_parts", R * G * gc)
            ops.c1_gram(x, gparts, N, B, H, H)
            gram = ws.get(f"{tag}.c1gram", G * gc)
            ops.sum_rows(gparts, R, G * gc, gram)
            ops.c1_gram_finalize(gram, wk, bias, store[bk + ".weight"], store[bk + ".bias"], B * Ho * Ho,
                                 st[0], st[1], st[2], st[3], rm, rv, G)
            ctx["gram"] = gram
        else:
            if pm:
                R = ops.c1r5_stats_rows(N, B, H, H)
                parts = ws.get("stat_parts", co * G * R * 2)
                ops.c1r5_stats(x, wk, bias, parts, N, B, H, H)
            else:
                R = ops.cl_c1_recompute_rows(ops.C1_STATS, self.act, N, B, ci, H, H, co, k, pad)
                parts = ws.get("stat_parts", co * G * R * 2)
                ops.cl_c1_recompute(ops.C1_STATS, x, wk, bias, N, B, ci, H, H, co, k, pad, out=parts)
            ops.bn_finalize(parts, G, R, co, B * Ho * Ho, store[bk + ".weight"], store[bk + ".bias"],
                            st[0], st[1], st[2], st[3], rm, rv)
        if update_running:
            store.bump_nbt(bk + ".num_batches_tracked", G)
        out = ws.get(f"{tag}.x1", N * Hp * Hp * co, self.act)
        route = self._codes_ok(N, B, need_dgrad)
        if route == "audio":
            # training forward: the pooling pass also records where each window's gradient goes
            # (routing codes), so the backward needs neither y nor a recompute of it
            codes = ws.get(f"{tag}.c1codes", N * Hp * Hp, torch.int32)
            ops.c1_apply_codes(x, wk, bias, st[2], st[3], out, codes, N, B, H, H)
            ctx["codes"] = (route, codes)
        elif route == "image":
            codes = ws.get(f"{tag}.c1codes", N * Hp * Hp * 8, torch.int16)
            ops.c1r5_apply_codes(x, wk, bias, st[2], st[3], out, codes, N, B, H, H)
            ctx["codes"] = (route, codes)
        elif route == "c3":
            codes = ws.get(f"{tag}.c1codes", N * Hp * Hp * co // 4, torch.int16)
            ops.c1r3_apply_codes(x, wk, bias, st[2], st[3], out, codes, N, B, H, H, co)
            ctx["codes"] = (route, codes)
        elif pm:
            ops.c1r5_apply_codes(x, wk, bias, st[2], st[3], out, None, N, B, H, H)
        else:
            ops.cl_c1_recompute(ops.C1_APPLY, x, wk, bias, N, B, ci, H, H, co, k, pad, scale=st[2],
                                shift=st[3], z=out)
        ctx["y"].append(None)          # never stored: the backward recomputes it
        ctx["stats"].append(st)
        ctx["x"].append(out)
        return out

    def _first_layer_recompute_bwd(self, ws, store, ctx, gout, N, G, B):
        ci, co, k, pad = self.stack.convs[0]
        H, Ho, Hp = self.dims[0]
        x, wk, st = ctx["x"][0], ctx["wts"][0][0], ctx["stats"][0]
        bk, ck = self.stack.bn_keys[0], self.stack.conv_keys[0]
        bias = store[ck + ".bias"]
        if ctx.get("codes") is not None:
            # one pass over x, the pooled gradient and the routing codes; a float64 combine forms
            # the BN backward and dW from the moments (avd_cl_c1_codes_combine / c1r5)
            route, codes = ctx["codes"]
            if route == "audio" and ctx.get("gram") is not None:
                # M and sum dz only; the Gram / S are the forward statistics pass's
                Rc, mc = ops.c1_codes_rows(N, B, H, H), ops.c1_codes_cols()
                parts = ws.get("c1_codes_parts", Rc * G * mc)
                ops.c1_moments_codes_ng(x, gout, codes, parts, N, B, H, H)
                mom = ws.get("c1_codes_mom", G * mc)
                ops.sum_rows(parts, Rc, G * mc, mom)
                ops.c1_codes_combine_gram(mom, ctx["gram"], wk, bias, store[bk + ".weight"], st[0], st[1],
                                          B * Ho * Ho, store.grad_of(ck + ".weight"),
                                          store.grad_of(bk + ".weight"), store.grad_of(bk + ".bias"),
                                          store.grad_of(ck + ".bias"), None, G)
                return
            if route == "c3":
                Rc, mc = ops.c1r3_codes_rows(N, B, H, H, co), ops.c1r3_codes_cols(co)
                parts = ws.get("c1_codes_parts", Rc * G * mc)
                ops.c1r3_moments_codes(x, wk, gout, codes, parts, N, B, H, H, co)
                mom = ws.get("c1_codes_mom", G * mc)
                ops.sum_rows(parts, Rc, G * mc, mom)
                ops.c1r3_codes_combine(mom, wk, bias, store[bk + ".weight"], st[0], st[1], B * Ho * Ho,
                                       store.grad_of(ck + ".weight"), store.grad_of(bk + ".weight"),
                                       store.grad_of(bk + ".bias"), store.grad_of(ck + ".bias"), None, G, co)
                return
            img = route == "image"
            Rc = (ops.c1r5_codes_rows if img else ops.c1_codes_rows)(N, B, H, H)
            mc = ops.c1r5_codes_cols() if img else ops.c1_codes_cols()
            parts = ws.get("c1_codes_parts", Rc * G * mc)
            (ops.c1r5_moments_codes if img else ops.c1_moments_codes)(x, gout, codes, parts, N, B, H, H)
            mom = ws.get("c1_codes_mom", G * mc)
            ops.sum_rows(parts, Rc, G * mc, mom)
            (ops.c1r5_codes_combine if img else ops.c1_codes_combine)(
                mom, wk, bias, store[bk + ".weight"], st[0], st[1], B * Ho * Ho,
                store.grad_of(ck + ".weight"), store.grad_of(bk + ".weight"),
                store.grad_of(bk + ".bias"), store.grad_of(ck + ".bias"), None, G)
            return
        R4 = ops.cl_c1_recompute_rows(ops.C1_REDUCE_MOMENTS, self.act, N, B, ci, H, H, co, k, pad)
        if self.RC_MOMENTS and R4 > 0:
            # one pass: BN-backward sums + the moments dW is linear in (3x3 layers)
            mc = ops.c1_moment_cols(co, k)
            parts = ws.get("bwd_parts_m", co * G * R4 * 2 + R4 * G * mc)
            ops.cl_c1_recompute(ops.C1_REDUCE_MOMENTS, x, wk, bias, N, B, ci, H, H, co, k, pad,
                                scale=st[2], shift=st[3], mean=st[0], invstd=st[1], gz=gout, out=parts)
            coef = ws.get("bwd_coef", G * co * 3)
            ops.bn_bwd_finalize(parts, G, R4, co, B * Ho * Ho, store[bk + ".weight"], st[0], st[1],
                                coef, store.grad_of(bk + ".weight"), store.grad_of(bk + ".bias"),
                                store.grad_of(ck + ".bias"))
            mom = ws.get("c1_moments", G * mc)
            ops.sum_rows(parts, R4, G * mc, mom, off=co * G * R4 * 2)
            ops.cl_c1_recompute_combine(mom, coef, wk, bias, store.grad_of(ck + ".weight"), G, co, k)
            return
        R = ops.cl_c1_recompute_rows(ops.C1_REDUCE, self.act, N, B, ci, H, H, co, k, pad)
        parts = ws.get("bwd_parts", co * G * R * 2)
        ops.cl_c1_recompute(ops.C1_REDUCE, x, wk, bias, N, B, ci, H, H, co, k, pad, scale=st[2],
                            shift=st[3], mean=st[0], invstd=st[1], gz=gout, out=parts)
        coef = ws.get("bwd_coef", G * co * 3)
        ops.bn_bwd_finalize(parts, G, R, co, B * Ho * Ho, store[bk + ".weight"], st[0], st[1],
                            coef, store.grad_of(bk + ".weight"), store.grad_of(bk + ".bias"),
                            store.grad_of(ck + ".bias"))
        nsl = ops.cl_c1_recompute_rows(ops.C1_WGRAD, self.act, N, B, ci, H, H, co, k, pad)
        wparts = ws.get("wgrad_parts", nsl * co * ci * k * k)
        ops.cl_c1_recompute(ops.C1_WGRAD, x, wk, bias, N, B, ci, H, H, co, k, pad, scale=st[2],
                            shift=st[3], coef=coef, gz=gout, out=wparts)
        ops.sum_rows(wparts, nsl, co * ci * k * k, store.grad_of(ck + ".weight"))

    # Measured and removed (round 5 pruning): the BN-backward apply fused into
    # the dgrad / wgrad staging (2.62 vs 2.17 ms for the four mid layers), the previous layer's
    # BN-backward reduce in the dgrad epilogue (146k vs 159k pairs/s), the dgrad storing dy
    # (160.2k vs 166.7k), weight gradients on the main stream or deferred after the input-gradient
    # chain (within noise).

    # layers whose weight gradient runs on the input-gradient (main) stream even when a
    # weight-gradient stream is given: the audio 14^2 layer (its launch ran 640-650 us in the
    # graph beside two other streams' kernels, 153 us alone).  Round 6, with the fused 56^2 layer
    # backward, three interleaved rounds (profiles/r6_ab_wgrad_main.txt): {3} 4.913-4.936 ms,
    # none 4.911-4.957, {2} 4.973-5.004, {2, 3} (round 5's choice) 4.991-5.031
    WGRAD_MAIN = frozenset({3})

    # the audio conv2 (56^2) backward as ONE launch (avd_cl_layer_bwd: BN-backward apply, input
    # and weight gradient from the same staged tiles, no dY in HBM); False: apply + dgrad + wgrad
    LAYER_BWD = True

    def backward(self, ws, store, ctx, dfeat, wstream=None):
        """dfeat: gradient of the features (f32 [N, F]; hwc: NHWC act dtype); writes conv/BN
        parameter grads.
        wstream: a second stream for the mid layers' weight gradients (they only read dy and
        the layer input, so they overlap the input-gradient chain); joined before returning."""
        N, G = ctx["N"], ctx["G"]
        B = N // G
        gout = dfeat
        nl = len(self.stack.convs)
        main = torch.cuda.current_stream(dfeat.device) if wstream is not None else None
        wdone = []
        for i in reversed(range(nl)):
            ci, co, k, pad = self.stack.convs[i]
            H, Ho, Hp = self.dims[i]
            y, st = ctx["y"][i], ctx["stats"][i]
            if y is None:              # recompute-path first layer
                self._first_layer_recompute_bwd(ws, store, ctx, gout, N, G, B)
                ops.mark(f"b{i}")
                continue
            mode = self._tail_mode() if i == nl - 1 else 0
            bk, ck = self.stack.bn_keys[i], self.stack.conv_keys[i]
            R = ops.cl_bn_bwd_rows(B, co, Ho, Ho, self.act)
            parts = ws.get("bwd_parts", co * G * R * 2)
            pooled = ctx["x"][i + 1] if i < nl - 1 else ctx.get("feat")
            if mode in (0, 2) and pooled is not None and Ho % 2 == 0:
                # from the pooled output (2/4 of y's bytes): xhat = (p - beta)/gamma at the argmax
                ops.cl_bn_bwd_reduce_pooled(y, pooled, gout, mode, store[bk + ".weight"],
                                            store[bk + ".bias"], st[0], st[1], parts, N, B, co, Ho, Ho)
            else:
                ops.cl_bn_bwd_reduce(y, gout, mode, st[2], st[3], st[0], st[1], parts, N, B, co, Ho, Ho)
            coef = ws.get("bwd_coef", G * co * 3)
            ops.bn_bwd_finalize(parts, G, R, co, B * Ho * Ho, store[bk + ".weight"], st[0], st[1],
                                coef, store.grad_of(bk + ".weight"), store.grad_of(bk + ".bias"),
                                store.grad_of(ck + ".bias"))
            x = ctx["x"][i]
            wt = ctx["wts"][i]
            # (the fused layer's BN-backward apply holds at most ops.APPLY_GMAX groups' coefficients,
            # e.g. not 2 + 7 views)
            lbs = (ops.cl_layer_bwd_slabs(self.act, N, ci, H, H, co, k, pad)
                   if (self.LAYER_BWD and i > 0 and mode == 0 and wt[1] is not None and wt[3] is None
                       and N // B <= ops.APPLY_GMAX and not self._mx_wgrad(i, N)) else 0)
            if lbs:
                # the whole layer backward in one launch: dY formed in LDS from y and the pooled
                # gradient, dX and the dW slabs from the same tiles (lbwd.hip); its own dX
                # buffer, since gout is the previous dgrad's "bwd_dx"
                wparts = ws.get(f"lb_parts{i}", lbs * co * ci * k * k)
                dx = ws.get("bwd_dx_lb", N * H * H * ci, self.act)
                ops.mark(f"w{i}.begin")
                ops.cl_layer_bwd(y, gout, st[2], st[3], coef, None, x, wt[1], dx, wparts, lbs, N, B, ci,
                                 H, H, co, k, pad)
                ops.sum_rows(wparts, lbs, co * ci * k * k, store.grad_of(ck + ".weight"))
                ops.mark(f"w{i}.end")
                gout = dx
                ops.mark(f"b{i}")
                continue
            nsl = ops.cl_apply_wgrad_slabs(self.act, N, ci, H, H, co, k, pad) if (i == 0 and mode == 0) else 0
            if nsl:   # first layer: BN-backward apply fused with the weight gradient (no dy)
                wparts = ws.get("wgrad_parts", nsl * co * ci * k * k)
                ops.cl_bn_bwd_apply_wgrad(y, gout, st[2], st[3], coef, x, wparts, N, B, ci, H, H, co,
                                          k, pad)
                ops.sum_rows(wparts, nsl, co * ci * k * k, store.grad_of(ck + ".weight"))
                ops.mark(f"b{i}")
                continue
            nch = self._wgrad_chunks(i, N)
            dy = ws.get(f"bwd_dy{i}" if wstream is not None else "bwd_dy", N * Ho * Ho * co, self.act)
            ops.cl_bn_bwd_apply(y, gout, mode, st[2], st[3], coef, dy, N, B, co, Ho, Ho)
            if wstream is not None and i > 0 and i not in self.WGRAD_MAIN:
                wparts = ws.get(f"wgrad_parts{i}", nch * co * ci * k * k)
                wstream.wait_stream(main)
                with torch.cuda.stream(wstream):
                    ops.mark(f"w{i}.begin")
                    self._conv_wgrad(i, x, dy, wparts, N)
                    ops.sum_rows(wparts, nch, co * ci * k * k, store.grad_of(ck + ".weight"))
                    ops.mark(f"w{i}.end")
                    ev = new_event()
                    ev.record(wstream)
                wdone.append(ev)
            else:
                wparts = ws.get("wgrad_parts", nch * co * ci * k * k)
                ops.mark(f"w{i}.begin")
                self._conv_wgrad(i, x, dy, wparts, N)
                ops.sum_rows(wparts, nch, co * ci * k * k, store.grad_of(ck + ".weight"))
                ops.mark(f"w{i}.end")
            if i > 0:
                dx = ws.get("bwd_dx", N * H * H * ci, self.act)
                self._conv_dgrad(i, dy, ctx["wts"][i], dx, N)
                gout = dx
            ops.mark(f"b{i}")
        for ev in wdone:
            main.wait_event(ev)


# ============================================================================ dense heads
class ProjHead:
    """ProjectionHead (dino.py:1240-1254): Linear -> BN1d(train) -> GELU -> Dropout -> Linear."""

    def __init__(self, prefix, in_dim, out_dim, hidden=PROJ_HIDDEN, gemm_mode=ops.GEMM_F32_MFMA):
        self.p = prefix
        self.i, self.o, self.h = in_dim, out_dim, hidden
        self.gm = gemm_mode

    def forward(self, ws, store, tag, x, rows, out, drop_p=0.0, seed=0, x_ld=None, x_off=0,
                update_running=True, G=1, seed_off=None):
        """G > 1: the rows are G separate calls of the head (BatchNorm1d statistics and running
        updates per call, in order), e.g. SimCLR's image-image mode."""
        p, Hd = self.p, self.h
        rpg = rows // G
        h = ws.get(f"{tag}.h", rows * Hd)
        ops.linear_fwd(x, store[p + ".mlp.0.weight"], store[p + ".mlp.0.bias"], h, rows,
                       x_ld=x_ld, x_off=x_off, mode=self.gm)
        R = ops.colstats_parts(rpg)
        parts = ws.get("stat_parts", Hd * G * R * 2)
        pivot = ws.get(f"{tag}.pivot", G * Hd)
        ops.colstats(h, rows, G, Hd, parts, pivot)
        st = ws.get(f"{tag}.bn", 4 * G * Hd).view(4, G * Hd)
        ops.bn_finalize(parts, G, R, Hd, rpg, store[p + ".mlp.1.weight"], store[p + ".mlp.1.bias"],
                        st[0], st[1], st[2], st[3],
                        store[p + ".mlp.1.running_mean"] if update_running else None,
                        store[p + ".mlp.1.running_var"] if update_running else None, pivot=pivot)
        if update_running:
            store.bump_nbt(p + ".mlp.1.num_batches_tracked", G)
        a = ws.get(f"{tag}.a", rows * Hd)
        ops.act_fwd(h, a, 1, st[2], st[3], rows, G, Hd, drop_p, seed, seed_off)
        ops.linear_fwd(a, store[p + ".mlp.4.weight"], store[p + ".mlp.4.bias"], out, rows, mode=self.gm)
        return {"x": x, "x_ld": x_ld if x_ld is not None else self.i, "x_off": x_off, "h": h,
                "a": a, "st": st, "rows": rows, "G": G, "drop_p": drop_p, "seed": seed,
                "seed_off": seed_off}

    def backward(self, ws, store, ctx, dout, dx, dx_ld=None, dx_off=0):
        for _ in self.backward_steps(ws, store, ctx, dout, dx, dx_ld, dx_off):
            pass

    def backward_steps(self, ws, store, ctx, dout, dx, dx_ld=None, dx_off=0):
        """backward() as a generator that yields between its launch groups (so two heads'
        backward passes on two streams can be queued interleaved)."""
        p, Hd, rows, G = self.p, self.h, ctx["rows"], ctx["G"]
        rpg = rows // G
        da = ws.get("head_da", rows * Hd)
        ops.linear_bwd(dout, ctx["a"], store[p + ".mlp.4.weight"], store.grad_of(p + ".mlp.4.weight"),
                       store.grad_of(p + ".mlp.4.bias"), da, rows, mode=self.gm)
        yield
        st = ctx["st"]
        dz = ws.get("head_dz", rows * Hd)
        R = ops.colstats_parts(rpg)
        parts = ws.get("bwd_parts", Hd * G * R * 2)
        # GELU / dropout backward and the BatchNorm1d partials in one launch
        ops.bn1d_act_bwd_reduce(ctx["h"], da, dz, st[2], st[3], st[0], st[1], rows, G, Hd,
                                ctx["drop_p"], ctx["seed"], parts, ctx.get("seed_off"))
        yield
        coef = ws.get("bwd_coef", G * Hd * 3)
        ops.bn_bwd_finalize(parts, G, R, Hd, rpg, store[p + ".mlp.1.weight"], st[0], st[1], coef,
                            store.grad_of(p + ".mlp.1.weight"), store.grad_of(p + ".mlp.1.bias"), None)
        dh = ws.get("head_dh", rows * Hd)
        ops.bn1d_bwd_apply(ctx["h"], dz, coef, dh, rows, G, Hd)
        yield
        ops.linear_bwd(dh, ctx["x"], store[p + ".mlp.0.weight"], store.grad_of(p + ".mlp.0.weight"),
                       store.grad_of(p + ".mlp.0.bias"), dx, rows, x_ld=ctx["x_ld"],
                       x_off=ctx["x_off"], dx_ld=dx_ld, dx_off=dx_off, mode=self.gm)


class Hyper:
    def __init__(self, lr=1e-4, weight_decay=1e-6, momentum=0.996, center_momentum=0.9,
                 student_temperature=0.1, teacher_temperature=0.04, dropout=0.3,
                 fusion_dropout=0.3, alpha=1.0, betas=(0.9, 0.999), eps=1e-8):
        self.lr, self.wd = lr, weight_decay
        self.momentum, self.center_momentum = momentum, center_momentum
        self.tau_s, self.tau_t = student_temperature, teacher_temperature
        self.dropout, self.fusion_dropout = dropout, fusion_dropout
        self.alpha = alpha
        self.betas, self.eps = betas, eps


SEED_MASK = 0xFFFFFFFFFFFF


class StepState:
    """The per-step scalars of a training step in device memory (avd_step_begin): the optimizer
    step count, lr and Adam bias corrections, and the dropout counter offset.  Kernels read them
    from there, so a step captured once as a hipGraph replays every later step exactly as the
    eager step would run it (fresh dropout masks, the right bias corrections).  The host keeps
    no copy that can drift: ``t`` and ``seed_off`` advance only on the device."""

    SEED_STRIDE = 16

    def __init__(self, device, lr, betas=(0.9, 0.999)):
        self.t = torch.zeros(1, dtype=torch.int64, device=device)
        self.seed_off = torch.zeros(1, dtype=torch.int64, device=device)
        self.hyp = torch.zeros(4, dtype=torch.float32, device=device)
        self.b1, self.b2 = betas
        self.lr = None
        self.set_lr(lr)

    def set_lr(self, lr):
        """Host-side schedule change (eager, outside any captured graph)."""
        if lr != self.lr:
            self.hyp[0:1].fill_(lr)
            self.lr = lr

    def begin(self, seed=True):
        """seed_off = t * 16; t += 1; hyp[1:3] = 1 - beta^t."""
        ops.step_begin(self.t, self.hyp, self.seed_off if seed else None, self.b1, self.b2,
                       self.SEED_STRIDE)


def adam_step_dev(store, hp, sstate, lo=0, n=None):
    """adam_step with lr / bias corrections from the device StepState (graph-replayable)."""
    n = store.n_live - lo if n is None else n
    b1, b2 = hp.betas
    ops.adam_dev(store.student[lo:lo + n], store.grad[lo:lo + n], store.adam_m[lo:lo + n],
                 store.adam_v[lo:lo + n], n, sstate.hyp, b1, b2, hp.eps, hp.wd)


def adam_step(store, hp):
    """torch.optim.Adam over the live arena (params with grad=None are outside it)."""
    store.adam_step += 1
    t = store.adam_step
    b1, b2 = hp.betas
    ops.adam(store.student, store.grad, store.adam_m, store.adam_v, store.n_live, hp.lr, b1, b2,
             hp.eps, hp.wd, 1 - b1 ** t, 1 - b2 ** t)


def ema_step(store, m):
    ops.ema(store.teacher, store.student[store.n_heads:], store.n_ema, m)


def _exchange_in_step(hook):
    """A bucket-capable gradient hook (dist.GradAllReduce) at world > 1: the step's final
    exchange runs at a host point inside the step body (eager, or between captured segments),
    followed by the 1/world scale and the optimizer in the same (last) graph segment."""
    from . import dist as avdist
    return (hasattr(hook, "finish") and BUCKETS
            and avdist.distributed(getattr(hook, "group", None)))


def _exchange_begin(hook):
    """Start of a step's gradient exchange (eager, before any replayed segment)."""
    if hasattr(hook, "begin"):
        hook.begin()


def _exchange_finish(hook, grad, ranges=None):
    """Inside a step body, every forked stream joined: the rest of the all-reduce and the wait
    at a host point, then x 1/world as device work of the current segment."""
    host_point(lambda: hook.finish(grad, ranges))
    hook.scale(grad)


# ============================================================================ multimodal DINO
class MultiCentralEngine:
    """Training step of MultiModalDINO{,WithMSE,WithINFONCE,SemiSupervised} over
    CentralMultiModalEncoder (``--model multi_central``, dino.py:454-468) or
    SimpleMultiModalEncoder (``--model multi_simple``, dino.py:214-234: the 3x3 image_encoder /
    audio_encoder with global average pooling), ``--training_mode {default,mse,infonce,
    semi_supervised}``.  Both encoders are the same dataflow -- two conv branches, each a
    Linear to E, cat, fusion -- so only the stacks and the Linear keys differ."""

    def __init__(self, store, mode, E, D, P, hp, act_dtype=F32, grad_hook=None, seed=0,
                 buffer_hook=None, negatives="global", group=None, concurrent=True, conv_fp8=False,
                 encoder="multi_central"):
        self.store, self.mode, self.E, self.D, self.P, self.hp = store, mode, E, D, P, hp
        self.act = act_dtype
        # Linear layers: bf16 MFMA in the bf16 mode (like the reference's fp16 autocast),
        # exact-f32 MFMA in the fp32 (parity) mode
        self.gm = ops.GEMM_BF16_MFMA if act_dtype == torch.bfloat16 else ops.GEMM_F32_MFMA
        self.ws = Workspace(store.device)
        # conv_fp8: block-scaled e4m3 MFMA forward + input gradient for the mid-layer convs
        # (bf16 mode only; config 5)
        self.conv_fp8 = bool(conv_fp8) and act_dtype == torch.bfloat16
        self.encoder = encoder
        istack, self.img_lin, astack, self.aud_lin, _sd = MULTI_ENCODERS[encoder]
        # bf16: the flatten tails stay NHWC bf16 and the encoder Linears run on the (h, w, c)
        # ordered kernels (avd_linear_*_hwc) with a per-step bf16 copy of their weights
        hwc = self.HWC and act_dtype == torch.bfloat16
        self.img = ConvBranch(istack("student"), act_dtype, conv_fp8, hwc)
        self.aud = ConvBranch(astack("student"), act_dtype, conv_fp8, hwc)
        self.t_img = ConvBranch(istack("teacher"), act_dtype, conv_fp8, hwc)
        self.t_aud = ConvBranch(astack("teacher"), act_dtype, conv_fp8, hwc)
        self.sproj = ProjHead("student_projection", D, P, gemm_mode=self.gm)
        self.tproj = ProjHead("teacher_projection", D, P, gemm_mode=self.gm)
        self.heads = None
        if mode in HEAD_NAMES:
            hi, ha = HEAD_NAMES[mode]
            out = 10 if mode == "semi_supervised" else P
            self.heads = (ProjHead(hi, E, out, gemm_mode=self.gm), ProjHead(ha, E, out, gemm_mode=self.gm))
        # teacher forward and the image-branch backward run on a side stream with their own
        # scratch (Workspace, split-K GEMM buffer), joined by events; concurrent=False keeps
        # everything on the caller's stream
        # (one stream: 146.7k vs 162.6k pairs/s in round 2)
        self.side = torch.cuda.Stream(store.device) if (concurrent and store.device.type == "cuda") else None
        # the audio branch's mid-layer weight gradients on a third stream
        self.wside = torch.cuda.Stream(store.device) if self.side is not None else None
        self.tws = Workspace(store.device) if self.side is not None else self.ws
        self.iws = Workspace(store.device) if self.side is not None else self.ws
        self.grad_hook = grad_hook      # e.g. DDP all-reduce of store.grad (avdino.dist)
        self.buffer_hook = buffer_hook  # e.g. rank-0 buffer broadcast before each forward
        # InfoNCE negatives under DDP: "global" = all-gathered (single-device loss over the
        # global batch), "local" = this rank's batch only (the reference's DDP)
        self.negatives, self.group = negatives, group
        self.seed = seed
        self.step_idx = 0
        self.fwd_count = 0     # forwards so far (a backward belongs to the latest one)
        self.last = {}
        self.sstate = StepState(store.device, hp.lr, hp.betas)
        self.use_graph = False     # step(): capture the device work once, replay it (bench)
        self.graph = GraphedStep(deps=self._graph_deps)
        # pipeline=True: step(batch, next_batch) runs the teacher forward of next_batch on a
        # fourth stream under this step's backward (it only needs the EMA'd teacher and the next
        # batch's global views), so the next step's loss finds the teacher output ready.  Same
        # losses and parameters as the sequential step; the teacher's BN running statistics and
        # counters run one batch ahead between steps (train-mode BN normalises with the batch's
        # own statistics, so no output depends on them; under DDP the rank-0 buffer broadcast
        # of the next step then carries rank 0's already-updated teacher statistics).  Measured
        # no faster on the config-2 step (profiles/r2f_ab.txt: the chip is already shared by
        # three streams), so off by default.
        self.pipeline = False
        self.tside = None
        # real-data input prefetch (prefetch()): data stream, the staging buffer set in use (0/1),
        # the pending prefetch (batch, set, done event, staged)
        self.dstream = None
        self._par = 0
        self._pf = None
        self._t_ready = None       # (batch, B, G) of the teacher output waiting in t_proj
        self.tin_pending = None    # the next batch's teacher inputs while its forward is queued
        self._tseed = None

    def _graph_deps(self):
        """What a captured step's buffer addresses depend on: the shared GEMM / row-sum scratch
        (ops.alloc_epoch) and this engine's own workspaces."""
        return (ops.alloc_epoch(), self.ws.epoch, self.tws.epoch, self.iws.epoch)

    # encoder Linears over the NHWC bf16 pooled maps in the bf16 step (False: f32 (c,h,w)
    # features through avd_gemm / avd_linear_bwd, as in the fp32 parity mode)
    HWC = True

    def _wp(self, prefix, branch):
        """The per-step bf16 (h, w, c)-column copy of ``prefix``'s image / audio encoder Linear."""
        lin = self.img_lin if branch == "img" else self.aud_lin
        w = self.store[f"{prefix}.{lin}.weight"]
        return self.ws.get(f"wp.{prefix}.{branch}", w.numel(), torch.bfloat16)

    def _prepare_hwc(self, prefixes):
        """Refresh the bf16 (h, w, c) weight copies of these prefixes' encoder Linears (one
        launch), after Adam / EMA changed the weights."""
        ent = []
        for prefix in prefixes:
            for branch, cb in (("img", self.img), ("aud", self.aud)):
                if not cb.hwc:
                    continue
                lin = self.img_lin if branch == "img" else self.aud_lin
                C, HW = cb.feat_shape()
                ent.append((self.store[f"{prefix}.{lin}.weight"], self._wp(prefix, branch), C, HW))
        if ent:
            ops.linear_weight_hwc(ent)

    def _layouts(self, jobs):
        """The conv weight layouts of several branch passes in one launch (per kind): jobs =
        [(branch, ws, tag, need_dgrad, N, B)] -> each pass's layouts for ``forward(wts=...)``."""
        out, batch, mxb = [], [], []
        for cb, ws, tag, need_dgrad, N, B in jobs:
            w, b, m = cb.prepare(ws, self.store, tag, need_dgrad, N, B, launch=False)
            out.append(w)
            batch += b
            mxb += m
        launch_layouts(batch, mxb)
        return out

    def _linear_fwd(self, prefix, branch, cb, feat, cat, N, off):
        E = self.E
        lin = f"{prefix}.{self.img_lin if branch == 'img' else self.aud_lin}"
        if cb.hwc:
            C, HW = cb.feat_shape()
            ops.linear_fwd_hwc(feat, self._wp(prefix, branch), self.store[lin + ".bias"], cat, N, E, C, HW,
                               out_ld=2 * E, out_off=off)
        else:
            ops.linear_fwd(feat, self.store[lin + ".weight"], self.store[lin + ".bias"], cat, N,
                           out_ld=2 * E, out_off=off, mode=self.gm)

    # the heads' backward queued interleaved with the main chain's (else after it); the
    # originals' heads forward queued after the fusion / projection (else before)
    INTERLEAVE = True
    FHEADS_LATE = True

    # -------------------------------------------------------------- streams
    def _on_side(self, fn, after=None):
        """Run fn() on the side stream after everything queued so far on the current stream (or
        after the event ``after`` recorded on it earlier); returns (fn's result, completion
        event), or runs inline without a side stream."""
        if self.side is None:
            return fn(), None
        main = torch.cuda.current_stream(self.store.device)
        if after is not None:
            self.side.wait_event(after)
        else:
            self.side.wait_stream(main)
        with torch.cuda.stream(self.side):
            out = fn()
            done = new_event()
            done.record(self.side)
        return out, done

    def _join(self, done):
        if done is not None:
            torch.cuda.current_stream(self.store.device).wait_event(done)


    # -------------------------------------------------------------- pieces
    def _encoder_fwd(self, prefix, ib, ab, x_img, x_aud, N, G, tag, need_dgrad, update_running=True,
                     ws=None, wts=(None, None)):
        """Image + audio conv stacks and their Linear(., E) into one [N, 2E] buffer (= the cat).
        wts: the two branches' conv layouts when already launched (``_layouts``)."""
        ws, st, E = ws or self.ws, self.store, self.E
        cat = ws.get(tag + ".cat", N * 2 * E)

        # (the student's image branch on the side stream beside its audio branch measured slower:
        # 149.7k vs 152.4k pairs/s, r1_39 -- both fill the chip)
        fi, ci = ib.forward(ws, st, tag + ".img", x_img, N, G, update_running, need_dgrad, wts=wts[0])
        self._linear_fwd(prefix, "img", ib, fi, cat, N, 0)
        fa, ca = ab.forward(ws, st, tag + ".aud", x_aud, N, G, update_running, need_dgrad, wts=wts[1])
        self._linear_fwd(prefix, "aud", ab, fa, cat, N, E)
        return cat, (fi, ci, fa, ca)

    def _fusion_fwd(self, prefix, cat, rows, tag, seed, ws=None, seed_off=None):
        """fusion: Linear(2E,E) -> ReLU -> Dropout(0.3, hard-coded dino.py:204/215) -> Linear(E,D)."""
        ws, st, E, D = ws or self.ws, self.store, self.E, self.D
        seed_off = self.sstate.seed_off if seed_off is None else seed_off
        h = ws.get(tag + ".fh", rows * E)
        ops.linear_fwd(cat, st[prefix + ".fusion.0.weight"], st[prefix + ".fusion.0.bias"], h, rows,
                       x_ld=2 * E, mode=self.gm)
        r = ws.get(tag + ".fr", rows * E)
        ops.act_fwd(h, r, 0, None, None, rows, 1, E, self.hp.fusion_dropout, seed, seed_off)
        out = ws.get(tag + ".fout", rows * D)
        ops.linear_fwd(r, st[prefix + ".fusion.3.weight"], st[prefix + ".fusion.3.bias"], out, rows,
                       mode=self.gm)
        return out, (h, r)

    # the next real-data batch's device augmentation queued on a data stream under the current
    # step (prefetch); False stages every batch synchronously
    PREFETCH = True

    def _aug_bufs(self, batch, with_orig, par):
        """Staged-input buffers of set ``par`` (0/1) for a {"aug", "idx"} batch:
        (x_img, x_aud, B, G, L)."""
        aug, idx = batch["aug"], batch["idx"]
        B, G, L = len(idx), aug.n_global_views, aug.n_local_views
        nv = G + L + (1 if with_orig else 0)
        sfx = "" if par == 0 else ".1"
        return (self.ws.get("in.img" + sfx, nv * B * 784, self.act),
                self.ws.get("in.aud" + sfx, nv * B * 12544, self.act), B, G, L)

    def prefetch(self, batch):
        """Queue the augmentation of the NEXT step's real-data batch ({"aug", "idx", ...}) on the
        data stream, into the staging buffers the current step does not read: its host work
        (parameter draws, id transfers, launches) is done while the current step runs, and the
        next stage() of that same batch object waits for it and takes those buffers.  Returns
        False when not applicable (synthetic views, no GPU, prefetch off).

        The data stream starts after the whole step just queued: an augmentation
        kernel running on the data stream BESIDE a replayed multi-stream step graph returns
        wrong pixels in about one run of three (a few lanes of a wave -- always lanes 48-63 --
        read zeros; its records, sample ids, staged LDS row and output buffer were all verified,
        the same kernel without LDS fails the same way, and eager multi-stream steps or
        single-stream graphs beside it never do), so the GPU work is not overlapped."""
        if not self.PREFETCH or "aug" not in batch or self.store.device.type != "cuda":
            return False
        if self._pf is not None:
            raise RuntimeError("prefetch: the previously prefetched batch was never consumed")
        par = 1 - self._par
        if self.dstream is None:
            self.dstream = torch.cuda.Stream(self.store.device)
        # the set's buffers are taken from the workspace here, on the main stream: a first
        # allocation (or a regrowth for a larger batch) synchronises the device inside
        # Workspace.get, so the block cannot be one that kernels of the current step still use
        main = torch.cuda.current_stream(self.store.device)
        self.dstream.wait_stream(main)
        with_orig = self.heads is not None
        staged = self._aug_bufs(batch, with_orig, par)
        with torch.cuda.stream(self.dstream):
            batch["aug"].stage(batch["idx"], staged[0], staged[1], with_orig)
            done = new_event()
            done.record(self.dstream)
        self._pf = (batch, par, done, staged)
        return True

    def stage(self, batch, with_orig, training=True):
        """Device batch dict -> view-major staged image/audio inputs (act dtype) and the labels,
        in fixed workspace buffers (what a captured step reads).

        A pending prefetch (prefetch()) of THIS batch is consumed: wait for the data stream, use
        its buffer set.  Any other staging first waits for that prefetch's data stream (it may
        still be writing its buffer set) and stages into the set in use, so nothing races it;
        an eval staging (``training=False``) leaves the prefetch pending for the step it was
        made for, a training staging of another batch drops it (that batch is augmented again
        when its own step comes)."""
        ws = self.ws
        main = torch.cuda.current_stream(self.store.device) if self.store.device.type == "cuda" else None
        pf = self._pf
        if pf is not None and pf[0] is batch:
            # prefetched under the previous step: wait for the data stream, use its buffers
            self._pf = None
            main.wait_event(pf[2])
            self._par = pf[1]
            x_img, x_aud, B, G, L = pf[3]
        else:
            if pf is not None:
                main.wait_event(pf[2])
                if training:
                    self._pf = None
            # the set the prefetch does not own (every set is free once no prefetch is pending)
            par = self._par if self._pf is not None else (self._par if "aug" in batch else 0)
            if "aug" in batch:
                # real-data path: the device augmentation writes the views straight into the
                # staged inputs ({"aug": MultiModalAugmentation, "idx": sample ids, "label": ...})
                x_img, x_aud, B, G, L = self._aug_bufs(batch, with_orig, par)
                batch["aug"].stage(batch["idx"], x_img, x_aud, with_orig)
            else:
                g_img, l_img = batch["g_img"], batch["l_img"]
                B, G = g_img.shape[:2]
                L = l_img.shape[1]
                nv = G + L + (1 if with_orig else 0)
                sfx = "" if par == 0 else ".1"
                x_img = ws.get("in.img" + sfx, nv * B * 784, self.act)
                x_aud = ws.get("in.aud" + sfx, nv * B * 12544, self.act)
                ops.stage_views(g_img.contiguous(), G, l_img.contiguous() if L else None, L,
                                batch["image"].contiguous() if with_orig else None, B, 784, x_img)
                ops.stage_views(batch["g_aud"].contiguous(), G, batch["l_aud"].contiguous() if L else None, L,
                                batch["audio"].contiguous() if with_orig else None, B, 12544, x_aud)
            self._par = par
        labels = None
        if self.mode == "semi_supervised":
            labels = ws.get("in.label" + ("" if self._par == 0 else ".1"), B, torch.int64)
            labels.copy_(batch["label"].reshape(-1))
        return x_img, x_aud, B, G, L, labels

    def reset_pipeline(self):
        """Forget a pipelined teacher output and a pending prefetch (e.g. at an epoch boundary,
        on resume, or before switching batches): the next step computes its own teacher forward
        and stages its batch itself.  Waits for the prefetch's data stream, so its buffers are
        free afterwards."""
        if self._pf is not None and self.store.device.type == "cuda":
            torch.cuda.current_stream(self.store.device).wait_event(self._pf[2])
        self._pf = None
        self._t_ready = None

    def stage_teacher(self, batch):
        """The global views of a (pre-augmented) batch into the teacher's own staged inputs
        (pipelined step: the student of the current step still reads its staged buffers)."""
        if "aug" in batch:
            raise ValueError("pipelined teacher: needs the batch's views ({'g_img', 'g_aud', ...})")
        g_img, g_aud = batch["g_img"], batch["g_aud"]
        B, G = g_img.shape[:2]
        x_img = self.ws.get("tin.img", G * B * 784, self.act)
        x_aud = self.ws.get("tin.aud", G * B * 12544, self.act)
        ops.stage_views(g_img.contiguous(), G, None, 0, None, B, 784, x_img)
        ops.stage_views(g_aud.contiguous(), G, None, 0, None, B, 12544, x_aud)
        return x_img, x_aud, B, G

    def _teacher_fwd(self, x_img, x_aud, B, G, seed_off=None, wts=(None, None)):
        """Teacher: global views, train-mode BN, no grad, into t_proj [G*B, P] (its workspace)."""
        tws, st = self.tws, self.store
        base = (self.seed * 1000003) & SEED_MASK
        ops.mark("t.begin")
        tcat, _ = self._encoder_fwd("teacher", self.t_img, self.t_aud, x_img[:G * B * 784],
                                    x_aud[:G * B * 12544], G * B, G, "t", need_dgrad=False, ws=tws,
                                    wts=wts)
        tout, _ = self._fusion_fwd("teacher", tcat, G * B, "t", base + 2, ws=tws, seed_off=seed_off)
        t_proj = tws.get("t_proj", G * B * self.P)
        self.tproj.forward(tws, st, "tp", tout, G * B, t_proj, 0.0, 0)
        ops.mark("t.end")
        return t_proj

    def _teacher_next(self, tin):
        """Pipelined step: the teacher forward of the next batch on the fourth stream, after
        everything queued so far on this one (the EMA'd teacher, the loss that read t_proj);
        its fusion dropout uses the next step's counter offset.  Returns the completion event."""
        main = torch.cuda.current_stream(self.store.device)
        if self.tside is None:
            self.tside = torch.cuda.Stream(self.store.device)
            self._tseed = torch.zeros_like(self.sstate.seed_off)
        self.tside.wait_stream(main)
        with torch.cuda.stream(self.tside):
            torch.add(self.sstate.seed_off, StepState.SEED_STRIDE, out=self._tseed)
            x_img, x_aud, B, G = tin
            self._prepare_hwc(("teacher",))           # the EMA'd teacher's Linear copies
            self._teacher_fwd(x_img, x_aud, B, G, seed_off=self._tseed)
            done = new_event()
            done.record(self.tside)
        return done

    # -------------------------------------------------------------- the step
    def forward(self, batch, training=True):
        # training=False skips the input-grad weight layouts (forward-only use of the API)
        """Forward of the whole step; fills self.last with everything backward needs.
        Returns the loss (a device scalar in the workspace)."""
        return self._forward_staged(self.stage(batch, self.heads is not None, training), training)

    def _forward_staged(self, staged, training=True, teacher_ready=False):
        hp, ws, st = self.hp, self.ws, self.store
        E, D, P = self.E, self.D, self.P
        with_orig = self.heads is not None
        x_img, x_aud, B, G, L, labels = staged
        V = G + L
        NG = V + (1 if with_orig else 0)   # BN groups of the student pass
        N = NG * B
        if training:
            self.sstate.begin()        # dropout offset of this step, optimizer step count
        ops.mark("fwd.begin")
        base = (self.seed * 1000003) & SEED_MASK
        # this step's bf16 (h, w, c) copies of the encoder Linears (student; teacher unless its
        # forward already ran under the previous step)
        self._prepare_hwc(("student",) if teacher_ready else ("student", "teacher"))
        # and the student's (and teacher's) conv weight layouts, all in one launch
        jobs = [(self.img, ws, "s.img", training, N, B), (self.aud, ws, "s.aud", training, N, B)]
        if not teacher_ready:
            jobs += [(self.t_img, self.tws, "t.img", False, G * B, B),
                     (self.t_aud, self.tws, "t.aud", False, G * B, B)]
        lw = self._layouts(jobs)

        # teacher: global views (prefix of the staged buffers), train-mode BN, no grad -- on a
        # side stream, concurrently with the student (independent until the loss); pipelined
        # steps find it computed under the previous step's backward
        if teacher_ready:
            t_proj, t_done = self.tws.get("t_proj", G * B * P), None
        else:
            t_proj, t_done = self._on_side(lambda: self._teacher_fwd(x_img, x_aud, B, G,
                                                                     wts=(lw[2], lw[3])))
        # student: all views (+ originals) in one pass per conv layer
        cat, senc = self._encoder_fwd("student", self.img, self.aud, x_img, x_aud, N, NG, "s",
                                      need_dgrad=training, wts=(lw[0], lw[1]))
        loss_parts = ws.get("loss_parts", V * B + B)
        head_out = None
        hctx = None
        h_done = None
        n_parts = V * B
        if with_orig:
            # the originals' heads and their loss depend only on the cat rows [V*B, N): on the
            # side stream (its own scratch), concurrently with fusion, projection and DINO loss.
            # InfoNCE stays on this stream (its collectives keep one order per rank).
            def heads():
                hws = self.iws if self.mode != "infonce" else ws
                hi, ha = self.heads
                no = hi.o
                zi = hws.get("zi", B * no)
                za = hws.get("za", B * no)
                off = V * B * 2 * E
                ci = hi.forward(hws, st, "hi", cat, B, zi, 0.0, 0, x_ld=2 * E, x_off=off)
                ca = ha.forward(hws, st, "ha", cat, B, za, 0.0, 0, x_ld=2 * E, x_off=off + E)
                dzi = hws.get("dzi", B * no)
                dza = hws.get("dza", B * no)
                aux = loss_parts[V * B:V * B + B]
                if self.mode == "mse":
                    ops.mse_loss(zi, za, B, no, aux, dzi, dza)
                    # mse parts are already divided by B*P; loss = sum
                elif self.mode == "infonce":
                    self._infonce(zi, za, B, no, aux, dzi, dza)
                else:
                    self._supervised(zi, za, labels, B, no, aux, dzi, dza, hws)
                if hp.alpha != 1.0:
                    aux.mul_(hp.alpha)
                    dzi.mul_(hp.alpha)
                    dza.mul_(hp.alpha)
                ops.mark("heads.fwd")
                return (zi, za), (ci, ca, dzi, dza)

            f_after = None
            if self.mode == "infonce":
                if self._global_negatives():
                    # its all-gather is a host point: no forked stream may be in flight there
                    self._join(t_done)
                    t_done = None
                head_out, hctx = heads()
            elif self.FHEADS_LATE and self.side is not None:
                # queued (captured) after the fusion / projection below, depending only on
                # what is queued so far (the cat)
                f_after = new_event()
                f_after.record(torch.cuda.current_stream(st.device))
            else:
                (head_out, hctx), h_done = self._on_side(heads)
            n_parts = V * B + B
        ops.mark("s.enc")
        fout, sfus = self._fusion_fwd("student", cat, V * B, "s", base + 1)
        s_proj = ws.get("s_proj", V * B * P)
        spc = self.sproj.forward(ws, st, "sp", fout, V * B, s_proj, hp.dropout, base + 3,
                                 seed_off=self.sstate.seed_off)
        ops.mark("s.proj")
        if with_orig and f_after is not None:
            (head_out, hctx), h_done = self._on_side(heads, after=f_after)
        self._join(t_done)

        # DINO loss (+ centring and centre EMA) -- forward and d/ds in one pass
        ds = ws.get("ds", V * B * P)
        center_new = ws.get("center_new", P)
        work = ws.get("dino_work", (B + G * B) * P)
        center = st["center"]
        ops.dino_loss(s_proj, t_proj, center, V, G, B, P, hp.tau_s, hp.tau_t, hp.center_momentum,
                      False, loss_parts[:V * B], ds, center_new, work)
        t_out = ws.get("t_out", G * B * P)  # centred teacher output (API only; the loss used t_raw)
        ops.mark("dino")
        self._join(h_done)
        loss = ws.get("loss", 1)
        ops.sum_to(loss_parts, n_parts, 1.0, loss)
        ops.mark("loss")
        self.fwd_count += 1
        self.last = dict(B=B, G=G, L=L, V=V, NG=NG, N=N, cat=cat, senc=senc, sfus=sfus, spc=spc,
                         ds=ds, hctx=hctx, center_new=center_new, loss=loss, s_proj=s_proj,
                         t_proj=t_proj, training=training, head_out=head_out)
        st.flush_nbt()
        return loss

    def _infonce(self, zi, za, B, P, aux, dzi, dza, temperature=0.07):
        """infoNCE_loss (dino.py:1091-1128): symmetric CE over S = n(i) n(a)^T / tau, with the
        other ranks' rows as extra negatives when negatives == "global" (contrastive.py)."""
        parts = self.ws.get("nce.parts", 2 * B)
        scale = contrastive.infonce(self.ws, zi, za, B, P, dzi, dza, parts, temperature, self.gm,
                                    self.group, local=self.negatives == "local")
        ops.sum_to(parts, 2 * B, scale, aux[:1])
        aux[1:].zero_()

    def _supervised(self, zi, za, labels, B, C, aux, dzi, dza, ws=None):
        """supervised_loss (dino.py:1001-1025): CE(image) + CE(audio), mean over the batch."""
        ws = ws or self.ws
        parts = ws.get("sup.parts", 2 * B)
        ops.softmax_xent(zi, C, B, C, labels, 0, False, False, 1.0 / B, parts[:B], dzi, C, False)
        ops.softmax_xent(za, C, B, C, labels, 0, False, False, 1.0 / B, parts[B:], dza, C, False)
        ops.sum_to(parts, 2 * B, 1.0 / B, aux[:1])
        aux[1:].zero_()

    def update_center(self):
        self.store["center"].copy_(self.last["center_new"].view(1, -1))

    def backward(self, ds=None, dheads=None):
        """Backward of the last forward into the gradient arena (overwritten, not accumulated).
        Seeds: the fused losses' own d/ds and d/d(head outputs) by default; ``ds`` [V*B*P]
        and ``dheads`` = (d image head, d audio head) [B*out] replace them when the loss was
        computed outside the engine (the differentiable ``MultiModalDINO.forward`` path)."""
        ws, st, E, D, P = self.ws, self.store, self.E, self.D, self.P
        c = self.last
        B, V, N = c["B"], c["V"], c["N"]
        if ds is not None:
            c["ds"] = ds
        # d cat buffer [N, 2E]: rows [0, V*B) from the fusion, rows [V*B, N) from the heads
        dcat = ws.get("dcat", N * 2 * E)
        h_done = None

        # the heads' backward (disjoint dcat rows and parameters) on the side stream, beside
        # the projection / fusion backward on this one; both chains are generators yielding
        # between launch groups and are queued interleaved (INTERLEAVE), so a replayed graph
        # -- whose launches go out in capture order -- runs them side by side
        def heads_steps():
            ci, ca, dzi, dza = c["hctx"]
            if dheads is not None:
                dzi, dza = dheads
            hi, ha = self.heads
            off = V * B * 2 * E
            hws = self.iws
            yield from hi.backward_steps(hws, st, ci, dzi, dcat, dx_ld=2 * E, dx_off=off)
            yield from ha.backward_steps(hws, st, ca, dza, dcat, dx_ld=2 * E, dx_off=off + E)

        # (the main chain's Linear weight gradients beside it on the weight-gradient stream, the
        # chain running the input gradients only: measured no faster, round 5 -- bwd.main_heads
        # 246.9 vs 245.2 us, and the conv weight gradients queued behind them start later)
        def main_steps():
            dfout = ws.get("dfout", V * B * D)
            yield from self.sproj.backward_steps(ws, st, c["spc"], c["ds"], dfout)
            h, r = c["sfus"]
            dr = ws.get("fus_dr", V * B * E)
            ops.linear_bwd(dfout, r, st["student.fusion.3.weight"], st.grad_of("student.fusion.3.weight"),
                           st.grad_of("student.fusion.3.bias"), dr, V * B, mode=self.gm)
            yield
            dh = ws.get("fus_dh", V * B * E)
            ops.act_bwd(h, dr, dh, 0, None, None, V * B, 1, E, self.hp.fusion_dropout,
                        ((self.seed * 1000003) & SEED_MASK) + 1, self.sstate.seed_off)
            yield
            ops.linear_bwd(dh, c["cat"], st["student.fusion.0.weight"], st.grad_of("student.fusion.0.weight"),
                           st.grad_of("student.fusion.0.bias"), dcat, V * B, x_ld=2 * E, dx_ld=2 * E,
                           mode=self.gm)

        def drain(gen):
            for _ in gen:
                pass

        if c["hctx"] is None:
            drain(main_steps())
        elif self.side is None:
            drain(heads_steps())
            drain(main_steps())
        elif self.INTERLEAVE:
            main = torch.cuda.current_stream(self.store.device)
            self.side.wait_stream(main)
            gens = [(main_steps(), main), (heads_steps(), self.side)]
            while gens:
                for g in list(gens):
                    with torch.cuda.stream(g[1]):
                        if next(g[0], StopIteration) is StopIteration:
                            gens.remove(g)
            h_done = new_event()
            h_done.record(self.side)
        else:
            h_after = new_event()
            h_after.record(torch.cuda.current_stream(self.store.device))
            drain(main_steps())
            _, h_done = self._on_side(lambda: drain(heads_steps()), after=h_after)
        ops.mark("bwd.main_heads")
        self._join(h_done)
        ops.mark("bwd.heads_joined")
        # every stream is joined here and the heads / fusion / projection gradients are final:
        # their all-reduce goes out now (a host point), overlapping the conv-branch backward
        if self._bucketed():
            g = self.store.grad
            host_point(lambda: self.grad_hook.bucket(g, self._early_ranges))
        fi, cimg, fa, caud = c["senc"]
        iws = self.iws
        dfi = iws.get("dfeat_img", fi.numel(), fi.dtype)
        ilin, alin = "student." + self.img_lin, "student." + self.aud_lin

        def image_linear():
            if self.img.hwc:
                C, HW = self.img.feat_shape()
                ops.linear_bwd_hwc(dcat, fi, self._wp("student", "img"), st.grad_of(ilin + ".weight"),
                                   st.grad_of(ilin + ".bias"), dfi, N, E, C, HW, dout_ld=2 * E)
                return
            ops.linear_bwd(dcat, fi, st[ilin + ".weight"], st.grad_of(ilin + ".weight"),
                           st.grad_of(ilin + ".bias"), dfi, N, dout_ld=2 * E, mode=self.gm)

        def image_convs():
            self.img.backward(iws, st, cimg, dfi)
            ops.mark("img.bwd.end")

        def image_branch():      # independent of the audio branch: side stream
            ops.mark("img.bwd.begin")
            image_linear()
            image_convs()

        dfa = ws.get("dfeat_aud", fa.numel(), fa.dtype)

        def audio_linear():
            if self.aud.hwc:
                C, HW = self.aud.feat_shape()
                ops.linear_bwd_hwc(dcat, fa, self._wp("student", "aud"), st.grad_of(alin + ".weight"),
                                   st.grad_of(alin + ".bias"), dfa, N, E, C, HW, dout_ld=2 * E, dout_off=E)
                return
            ops.linear_bwd(dcat, fa, st[alin + ".weight"], st.grad_of(alin + ".weight"),
                           st.grad_of(alin + ".bias"), dfa, N, dout_ld=2 * E, dout_off=E,
                           mode=self.gm)

        if self._bucketed():
            # data parallel: both encoder Linears (1.2 M of the 2.1 M live gradients) first, on
            # this stream, then their bucket goes out under the conv branches' backward
            image_linear()
            audio_linear()
            g = self.store.grad
            host_point(lambda: self.grad_hook.bucket(g, self._linear_ranges))
            _, i_done = self._on_side(image_convs)
        else:
            _, i_done = self._on_side(image_branch)
            audio_linear()
        self.aud.backward(ws, st, caud, dfa, wstream=self.wside)
        ops.mark("aud.bwd.end")
        self._join(i_done)

    def _global_negatives(self):
        from . import dist as avdist
        return self.negatives != "local" and avdist.distributed(self.group)

    def _bucketed(self):
        """Early gradient bucket: a bucket-capable hook, world > 1, and no pipelined teacher
        forward in flight on its own stream at the bucket's host point."""
        from . import dist as avdist
        return (hasattr(self.grad_hook, "bucket") and self.tin_pending is None and BUCKETS
                and avdist.distributed(getattr(self.grad_hook, "group", None)))

    @property
    def _early_ranges(self):
        """Gradient-arena ranges final once the heads / fusion / projection backward is done:
        every live parameter outside the two conv branches (whose Linear to E included)."""
        st = self.store
        br = ("student." + self.img_lin.split(".")[0] + ".", "student." + self.aud_lin.split(".")[0] + ".")
        from .dist import merge_ranges
        from .params import ALIGN
        live = set(st.live_keys)
        return merge_ranges([(o, o + -(-n // ALIGN) * ALIGN) for k, (o, n) in st.s_offs.items()
                             if k in live and not k.startswith(br)])

    @property
    def _linear_ranges(self):
        """Gradient-arena ranges of the two encoder Linears (the second bucket)."""
        st = self.store
        from .dist import merge_ranges
        from .params import ALIGN
        keys = [f"student.{lin}.{p}" for lin in (self.img_lin, self.aud_lin) for p in ("weight", "bias")]
        return merge_ranges([(st.s_offs[k][0], st.s_offs[k][0] + -(-st.s_offs[k][1] // ALIGN) * ALIGN)
                             for k in keys])

    def _exchange_in_step(self):
        """The final gradient exchange inside the step body (a host point after every stream is
        joined), so the 1/world scale and Adam run in the step's last captured graph segment: a
        GradAllReduce hook at world > 1.  Else the hook runs after the step."""
        return _exchange_in_step(self.grad_hook)

    def step(self, batch, next_batch=None):
        """One full training step; returns the loss as a device tensor (no host sync).
        With ``use_graph`` everything after the input staging (and around the data-parallel
        collectives) is a captured hipGraph replayed per step.  With ``pipeline`` and the next
        step's batch, that batch's teacher forward runs under this step's backward."""
        if self.buffer_hook is not None:
            self.buffer_hook(self.store)
        self.sstate.set_lr(self.hp.lr)
        staged = self.stage(batch, self.heads is not None)
        B, G = staged[2], staged[3]
        # the previous step ran this batch's teacher (the reference held in _t_ready keeps the
        # object alive, so identity cannot be a recycled id).  Contract of the pipelined step:
        # ``batch`` IS the previous call's ``next_batch``, not mutated since -- that teacher
        # forward already updated the teacher's BN running statistics, so a different batch
        # here cannot be served without drifting from the sequential run: refuse it.
        if self._t_ready is not None and not (self._t_ready[0] is batch and self._t_ready[1:] == (B, G)):
            raise ValueError("pipelined step: batch must be the previous step's next_batch (its "
                             "teacher forward already ran); call reset_pipeline() (or set "
                             "pipeline=False) to change batches")
        ready = self._t_ready is not None
        tin = None
        if self.pipeline and next_batch is not None and self.side is not None and "aug" not in next_batch:
            tin = self.stage_teacher(next_batch)

        in_step = self._exchange_in_step()
        _exchange_begin(self.grad_hook)

        def body():
            ops.mark_reset()
            self._forward_staged(staged, training=True, teacher_ready=ready)
            self.update_center()
            ema_step(self.store, self.hp.momentum)     # update_teacher: pre-step student
            ops.mark("ema")
            t_done = self._teacher_next(tin) if tin is not None else None
            self.backward()
            self._join(t_done)
            if self.grad_hook is None:
                adam_step_dev(self.store, self.hp, self.sstate)
            elif in_step:
                _exchange_finish(self.grad_hook, self.store.grad)
                adam_step_dev(self.store, self.hp, self.sstate)
            self.store.flush_nbt()
            ops.mark("end")

        self._t_ready = (next_batch,) + tin[2:4] if tin is not None else None
        self.tin_pending = tin
        if self.use_graph:
            self.graph.run(staged[2:5] + (ready, tin is not None, self._par), body)
        else:
            body()
        self.tin_pending = None
        if next_batch is not None and "aug" in next_batch:
            self.prefetch(next_batch)
        if self.grad_hook is not None and not in_step:
            self.grad_hook(self.store.grad)
            adam_step_dev(self.store, self.hp, self.sstate)
        self.store.adam_step += 1
        self.step_idx += 1
        return self.last["loss"]

    def last_head_outputs(self):
        """(image head output, audio head output) [B, P or classes] of the last forward."""
        c = self.last
        zi, za = c["head_out"]
        return zi.view(c["B"], -1), za.view(c["B"], -1)

    def outputs(self):
        """(s_out [V,B,P], t_out [G,B,P] centred with the pre-update centre) of the last
        forward, as MultiModalDINO.forward returns them (dino.py:719-727).  Call before
        update_center()."""
        c = self.last
        B, V, G, P = c["B"], c["V"], c["G"], self.P
        s = c["s_proj"].view(V, B, P)
        t = c["t_proj"].view(G, B, P) - self.store["center"].view(1, 1, P)
        return s, t


# ============================================================================ unimodal DINO
class UniEncoder:
    """An UNIMODAL_MODEL_MAP encoder (run_dino.py:542-550) on channels-last maps: conv stack
    (ConvBranch) then its Linear chain -- ImageEncoder: GAP -> Linear(128,512) -> Linear(512,D)
    (dino.py:483-499); SpectrogramEncoder: GAP -> Linear(256,D) (502-513);
    SpectrogramEncoderCentral: CentralUnimodalAudio flatten -> Linear(3136,D) (515-523)."""

    def __init__(self, kind, prefix, act_dtype, gemm_mode):
        modality, stack, lins, _sd = UNI_ENCODERS[UNI_ALIASES.get(kind, kind)]
        self.modality = modality
        self.hw = 28 if modality == "image" else 112
        self.branch = ConvBranch(stack(prefix), act_dtype)
        self.lins = [f"{prefix}.{k}" for k in lins]
        self.gm = gemm_mode

    def forward(self, ws, store, tag, x, N, G, need_dgrad):
        feat, ctx = self.branch.forward(ws, store, tag, x, N, G, True, need_dgrad)
        acts = [feat]
        h = feat
        for i, k in enumerate(self.lins):
            w = store[k + ".weight"]
            out = ws.get(f"{tag}.lin{i}", N * w.shape[0])
            ops.linear_fwd(h, w, store[k + ".bias"], out, N, mode=self.gm)
            acts.append(out)
            h = out
        return h.view(N, -1), (ctx, acts)

    def forward_eval(self, ws, store, tag, x, N):
        h = self.branch.forward_eval(ws, store, tag, x, N)
        for i, k in enumerate(self.lins):
            w = store[k + ".weight"]
            out = ws.get(f"{tag}.lin{i}", N * w.shape[0])
            ops.linear_fwd(h, w, store[k + ".bias"], out, N, mode=self.gm)
            h = out
        return h.view(N, -1)

    def backward(self, ws, store, ctx, dout):
        bctx, acts = ctx
        N = bctx["N"]
        g = dout
        for i in reversed(range(len(self.lins))):
            k = self.lins[i]
            w = store[k + ".weight"]
            dx = ws.get(f"uni.dlin{i}", N * w.shape[1])
            ops.linear_bwd(g, acts[i], w, store.grad_of(k + ".weight"), store.grad_of(k + ".bias"),
                           dx, N, mode=self.gm)
            g = dx
        self.branch.backward(ws, store, bctx, g)


class UniModalEngine:
    """Training step of UniModalDINO + UniModalDINOLightning (dino.py:1257-1398, 1575-1668):
    student over G global + L local views of one modality (one launch per layer, BN per view),
    teacher over the global views (train-mode BN, no grad), projection heads, the unimodal DINO
    loss (teacher centred by ``center`` AND by its per-view batch mean, dino.py:1613-1614), the
    cosine-consistency term over the student embeddings when cosine_loss_alpha > 0, centre EMA,
    teacher EMA (before backward, dino.py:1661), backward, Adam with L2 weight decay."""

    def __init__(self, store, kind, D, P, hp, act_dtype=F32, cos_alpha=0.0, grad_hook=None,
                 buffer_hook=None, seed=0, step_order="lightning"):
        """step_order "lightning": UniModalDINOLightning.training_step + Adam(L2) (EMA before
        backward); "pretrain": training_structures.pretrain_dino (dino_train.py:137-166):
        AdamW (weight_decay 0.01) and the EMA AFTER the optimizer step, loss = the unimodal
        DINO loss only."""
        if step_order not in ("lightning", "pretrain"):
            raise ValueError(step_order)
        if step_order == "pretrain" and float(cos_alpha) > 0:
            # pretrain_dino (dino_train.py:137-166) optimises the unimodal DINO loss alone
            raise ValueError("step_order='pretrain' runs pretrain_dino's loss, which has no "
                             "cosine-consistency term: cos_alpha must be 0")
        self.step_order = step_order
        self.store, self.D, self.P, self.hp = store, D, P, hp
        self.kind = UNI_ALIASES.get(kind, kind)
        self.act = act_dtype
        self.gm = ops.GEMM_BF16_MFMA if act_dtype == torch.bfloat16 else ops.GEMM_F32_MFMA
        self.cos_alpha = float(cos_alpha)
        self.ws = Workspace(store.device)
        self.enc = UniEncoder(self.kind, "student", act_dtype, self.gm)
        self.t_enc = UniEncoder(self.kind, "teacher", act_dtype, self.gm)
        self.modality = self.enc.modality
        self.sproj = ProjHead("student_projection", D, P, gemm_mode=self.gm)
        self.tproj = ProjHead("teacher_projection", D, P, gemm_mode=self.gm)
        self.grad_hook, self.buffer_hook = grad_hook, buffer_hook
        self.seed, self.step_idx = seed, 0
        self.fwd_count = 0
        self.last = {}
        self.sstate = StepState(store.device, hp.lr, hp.betas)
        self.use_graph = False
        self.graph = GraphedStep(deps=lambda: (ops.alloc_epoch(), self.ws.epoch))

    def stage(self, batch):
        key = "img" if self.modality == "image" else "aud"
        g = batch["g_" + key]
        l = batch.get("l_" + key)
        B, G = g.shape[:2]
        L = 0 if l is None else l.shape[1]
        HW = self.enc.hw * self.enc.hw
        x = self.ws.get("in.x", (G + L) * B * HW, self.act)
        ops.stage_views(g.contiguous(), G, l.contiguous() if L else None, L, None, B, HW, x)
        return x, B, G, L

    def forward(self, batch, training=True):
        return self._forward_staged(self.stage(batch), training)

    def _forward_staged(self, staged, training=True):
        hp, ws, st, D, P = self.hp, self.ws, self.store, self.D, self.P
        x, B, G, L = staged
        V = G + L
        HW = self.enc.hw * self.enc.hw
        if training:
            self.sstate.begin()
        base = (self.seed * 1000003) & SEED_MASK
        emb, sctx = self.enc.forward(ws, st, "s", x, V * B, V, need_dgrad=training)
        temb, _ = self.t_enc.forward(ws, st, "t", x[:G * B * HW], G * B, G, need_dgrad=False)
        s_proj = ws.get("s_proj", V * B * P)
        spc = self.sproj.forward(ws, st, "sp", emb, V * B, s_proj, hp.dropout, base + 3,
                                 seed_off=self.sstate.seed_off)
        t_proj = ws.get("t_proj", G * B * P)
        self.tproj.forward(ws, st, "tp", temb, G * B, t_proj, 0.0, 0)
        cos = self.cos_alpha > 0 and V >= 2
        loss_parts = ws.get("loss_parts", V * B + (B if cos else 0))
        ds = ws.get("ds", V * B * P)
        center_new = ws.get("center_new", P)
        work = ws.get("dino_work", (B + G * B) * P)
        ops.dino_loss(s_proj, t_proj, st["center"], V, G, B, P, hp.tau_s, hp.tau_t,
                      hp.center_momentum, True, loss_parts[:V * B], ds, center_new, work)
        if cos:
            ops.cosine_consistency(emb, V, B, D, self.cos_alpha, loss_parts[V * B:], None)
        loss = ws.get("loss", 1)
        ops.sum_to(loss_parts, loss_parts.numel(), 1.0, loss)
        self.fwd_count += 1
        self.last = dict(B=B, G=G, L=L, V=V, emb=emb, sctx=sctx, spc=spc, ds=ds, cos=cos,
                         center_new=center_new, s_proj=s_proj, t_proj=t_proj, loss=loss)
        st.flush_nbt()
        return loss

    def update_center(self):
        self.store["center"].copy_(self.last["center_new"].view(1, -1))

    def backward(self, ds=None, demb=None):
        """Backward into the gradient arena.  ``ds`` [V*B*P] replaces the fused DINO loss's
        d/ds and ``demb`` [V*B*D] the cosine term's d/d(embeddings) (then added to the
        projection's input gradient) when the losses were computed outside the engine."""
        ws, st, c = self.ws, self.store, self.last
        B, V, D = c["B"], c["V"], self.D
        g = ws.get("demb", V * B * D)
        self.sproj.backward(ws, st, c["spc"], c["ds"] if ds is None else ds, g)
        if demb is not None:
            g.add_(demb.reshape(-1))
        elif ds is None and c["cos"]:
            ops.cosine_consistency(c["emb"], V, B, D, self.cos_alpha, None, g)
        self.enc.backward(ws, st, c["sctx"], g)

    def step(self, batch):
        if self.buffer_hook is not None:
            self.buffer_hook(self.store)
        self.sstate.set_lr(self.hp.lr)
        staged = self.stage(batch)

        pre = self.step_order == "pretrain"

        def opt_and_ema():
            if pre:     # AdamW, then the EMA sees the post-step student
                b1, b2 = self.hp.betas
                st = self.store
                ops.adam_dev(st.student, st.grad, st.adam_m, st.adam_v, st.n_live, self.sstate.hyp,
                             b1, b2, self.hp.eps, 0.01, decoupled=True)
                ema_step(st, self.hp.momentum)
            else:
                adam_step_dev(self.store, self.hp, self.sstate)

        in_step = _exchange_in_step(self.grad_hook)
        _exchange_begin(self.grad_hook)

        def body():
            self._forward_staged(staged, training=True)
            self.update_center()
            if not pre:
                ema_step(self.store, self.hp.momentum)
            self.backward()
            if self.grad_hook is None:
                opt_and_ema()
            elif in_step:
                _exchange_finish(self.grad_hook, self.store.grad)
                opt_and_ema()

        if self.use_graph:
            self.graph.run(staged[1:], body)
        else:
            body()
        if self.grad_hook is not None and not in_step:
            self.grad_hook(self.store.grad)
            opt_and_ema()
        self.store.adam_step += 1
        self.step_idx += 1
        return self.last["loss"]

    def outputs(self):
        """(s_out [V,B,P], t_out [G,B,P] centred with the pre-update centre, embeddings [V,B,D])
        as UniModalDINO.forward returns them (dino.py:1392-1398).  Call before update_center()."""
        c = self.last
        B, V, G, P = c["B"], c["V"], c["G"], self.P
        return (c["s_proj"].view(V, B, P), c["t_proj"].view(G, B, P) - self.store["center"].view(1, 1, P),
                c["emb"].view(V, B, -1))


# ============================================================================ multimodal SimCLR
class SimCLREngine:
    """Training step of MultiModalSimCLRLightning (other_ssl/multimodal_simclr/
    multimodal_simclr.py:22-112): a host-drawn modality pair per step (0 image/image,
    1 audio/audio, 2 image/audio, 3 audio/image; torch.randint(0, 4), line 34), the towers
    ImageEncoder / SpectrogramEncoder + ProjectionHead(D, P) (lines 12-20), NT-Xent over
    [z1; z2] (tau 0.07, lines 74-89) with local or all-gathered global negatives
    (contrastive.py), and Adam without weight decay (lines 103-112) stepped ONLY on the tower(s)
    used this step: torch.optim.Adam skips parameters whose grad is None, each keeping its own
    step count, so the image and audio arenas carry separate bias-correction counters.
    Same-tower modes run both views through one launch per layer with two BatchNorm groups
    (two separate module calls in the reference)."""

    GROUPS = ("image_", "audio_")

    def __init__(self, store, D, P, hp, act_dtype=F32, temperature=0.07, negatives="global",
                 group=None, grad_hook=None, seed=1234):
        self.store, self.D, self.P, self.hp = store, D, P, hp
        self.act = act_dtype
        self.gm = ops.GEMM_BF16_MFMA if act_dtype == torch.bfloat16 else ops.GEMM_F32_MFMA
        self.ws = Workspace(store.device)
        self.towers = (
            (UniEncoder("image_simple", "image_encoder", act_dtype, self.gm),
             ProjHead("image_projection_head", D, P, gemm_mode=self.gm)),
            (UniEncoder("spectrogram_simple", "audio_encoder", act_dtype, self.gm),
             ProjHead("audio_projection_head", D, P, gemm_mode=self.gm)))
        self.temperature, self.negatives, self.group = temperature, negatives, group
        self.grad_hook = grad_hook
        self.gen = torch.Generator().manual_seed(seed)
        self.adam_t = [0, 0]
        self.ranges = [store.group_range(i) for i in range(2)]
        self.fwd_count = 0
        self.last = {}
        # one optimizer step count per tower (torch.optim.Adam keeps per-parameter steps)
        self.sstates = [StepState(store.device, hp.lr, hp.betas) for _ in range(2)]
        self.use_graph = False
        self.graph = GraphedStep(deps=lambda: (ops.alloc_epoch(), self.ws.epoch))

    def draw_mode(self):
        return int(torch.randint(0, 4, (1,), generator=self.gen).item())

    def _stage(self, tag, views, tower):
        enc = self.towers[tower][0]
        HW = enc.hw * enc.hw
        B = views[0].shape[0]
        x = self.ws.get(tag, len(views) * B * HW, self.act)
        ops.stage_views(views[0].contiguous(), 1, views[1].contiguous() if len(views) > 1 else None,
                        len(views) - 1, None, B, HW, x)
        return x

    def stage(self, batch, mode):
        """The mode's input views into fixed workspace buffers."""
        if mode in (0, 1):
            k1, k2 = ("img1", "img2") if mode == 0 else ("spec1", "spec2")
            return (self._stage("in.x0", (batch[k1], batch[k2]), mode),)
        order = (0, 1) if mode == 2 else (1, 0)
        return tuple(self._stage(f"in.x{j}", (batch[("img" if t == 0 else "spec") + str(j + 1)],), t)
                     for j, t in enumerate(order))

    def forward(self, batch, mode=None):
        """batch: img1/spec1/img2/spec2 device tensors [B,1,H,W].  Returns the loss tensor."""
        mode = self.draw_mode() if mode is None else int(mode)
        return self._forward_staged(self.stage(batch, mode), mode, batch["img1"].shape[0])

    def _forward_staged(self, xs, mode, B):
        ws, st, P = self.ws, self.store, self.P
        reps = ws.get("reps", 2 * B * P)
        calls = []   # (tower, rows slice start, n rows, groups, encoder ctx, head ctx)
        if mode in (0, 1):
            t = mode
            x = xs[0]
            enc, head = self.towers[t]
            emb, ectx = enc.forward(ws, st, "e0", x, 2 * B, 2, need_dgrad=True)
            hctx = head.forward(ws, st, "h0", emb, 2 * B, reps, 0.0, 0, G=2)
            calls.append((t, 0, 2 * B, ectx, hctx))
        else:
            order = (0, 1) if mode == 2 else (1, 0)
            for j, t in enumerate(order):
                x = xs[j]
                enc, head = self.towers[t]
                emb, ectx = enc.forward(ws, st, f"e{j}", x, B, 1, need_dgrad=True)
                hctx = head.forward(ws, st, f"h{j}", emb, B, reps[j * B * P:(j + 1) * B * P], 0.0, 0)
                calls.append((t, j * B, B, ectx, hctx))
        parts = ws.get("ntx.parts", 2 * B)
        dreps = ws.get("dreps", 2 * B * P)
        scale = contrastive.nt_xent(ws, reps, B, P, dreps, parts, self.temperature, self.gm,
                                    self.group, local=self.negatives == "local")
        loss = ws.get("loss", 1)
        ops.sum_to(parts, 2 * B, scale, loss)
        self.fwd_count += 1
        self.last = dict(B=B, mode=mode, calls=calls, reps=reps, dreps=dreps, loss=loss)
        st.flush_nbt()
        return loss

    def backward(self, dreps=None):
        """Backward into the used towers' gradient ranges; ``dreps`` [2B*P] replaces the fused
        NT-Xent's d/d[z1; z2] when the loss was computed outside the engine."""
        ws, st, c = self.ws, self.store, self.last
        P, D = self.P, self.D
        dr = c["dreps"] if dreps is None else dreps.reshape(-1)
        calls = c["calls"]
        for i, (t, r0, n, ectx, hctx) in enumerate(calls):
            enc, head = self.towers[t]
            demb = ws.get("demb", n * D)
            head.backward(ws, st, hctx, dr[r0 * P:(r0 + n) * P], demb)
            enc.backward(ws, st, ectx, demb)
            if i + 1 < len(calls) and self._bucketed():
                # this tower's gradients are final (one stream): all-reduce them now, under
                # the other tower's backward
                o, m = self.ranges[t]
                g = st.grad
                host_point(lambda g=g, o=o, m=m: self.grad_hook.bucket(g, [(o, o + m)]))

    def used_towers(self):
        return sorted({t for t, *_ in self.last["calls"]})

    def adam(self):
        """Adam(lr), no weight decay, on the used towers with their own step counters (device
        step state per tower: graph-replayable)."""
        b1, b2 = self.hp.betas
        st = self.store
        for t in self.used_towers():
            ss = self.sstates[t]
            ss.begin(seed=False)
            o, n = self.ranges[t]
            ops.adam_dev(st.student[o:o + n], st.grad[o:o + n], st.adam_m[o:o + n], st.adam_v[o:o + n],
                         n, ss.hyp, b1, b2, self.hp.eps, 0.0)

    def _bucketed(self):
        from . import dist as avdist
        return (hasattr(self.grad_hook, "bucket") and BUCKETS
                and avdist.distributed(getattr(self.grad_hook, "group", None)))

    def step(self, batch, mode=None):
        mode = self.draw_mode() if mode is None else int(mode)
        for ss in self.sstates:
            ss.set_lr(self.hp.lr)
        B = batch["img1"].shape[0]
        xs = self.stage(batch, mode)

        in_step = _exchange_in_step(self.grad_hook)
        _exchange_begin(self.grad_hook)

        def body():
            self._forward_staged(xs, mode, B)
            self.backward()
            if self.grad_hook is None:
                self.adam()
            elif in_step:
                # only the used towers' ranges: every rank draws the same mode sequence (same
                # generator seed, as the reference's seed_everything), so the sizes agree
                _exchange_finish(self.grad_hook, self.store.grad,
                                 [(o, o + n) for o, n in (self.ranges[t] for t in self.used_towers())])
                self.adam()

        if self.use_graph:
            self.graph.run((mode, B), body)
        else:
            body()
        if self.grad_hook is not None and not in_step:
            if hasattr(self.grad_hook, "bucket"):
                # only the used towers' ranges: every rank draws the same mode sequence (same
                # generator seed, as the reference's seed_everything), so the sizes agree
                self.grad_hook(self.store.grad, ranges=[(o, o + n) for o, n in
                                                        (self.ranges[t] for t in self.used_towers())])
            else:
                self.grad_hook(self.store.grad)
            self.adam()
        for t in self.used_towers():
            self.adam_t[t] += 1
        return self.last["loss"]

    def outputs(self):
        c = self.last
        B, P = c["B"], self.P
        return c["reps"][:B * P].view(B, P), c["reps"][B * P:].view(B, P)
