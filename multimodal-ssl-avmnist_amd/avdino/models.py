"""Reference-shaped model API over the HIP training engine.

Class names, constructor arguments, forward() signatures/returns and state-dict keys follow
the reference (paths relative to its AVMNIST_Experiments/):

  CentralMultiModalEncoder          models/dino.py:454-468   (``--model multi_central``)
  SimpleMultiModalEncoder           models/dino.py:214-234   (``--model multi_simple``)
  ProjectionHead                    models/dino.py:1240-1254
  MultiModalDINO                    models/dino.py:588-727
  MultiModalDINOWithMSE             models/dino.py:1156-1171
  MultiModalDINOWithINFONCE         models/dino.py:1053-1068
  MultiModalDINOSemiSupervised      models/dino.py:964-980
  MultiModalDINO*Lightning          models/dino.py:730-962, 982-1051, 1070-1154, 1173-1238
  UniModalDINO(Lightning)           models/dino.py:1257-1398, 1490-1759
  MultiModalSimCLR(Model|Lightning) other_ssl/multimodal_simclr/multimodal_simclr.py:12-112

Every model is a ``torch.nn.Module`` (a ``LightningModule`` when ``lightning`` is installed)
whose parameters are the flat fp32 arenas of a :class:`~avdino.params.ParamStore` -- one
``nn.Parameter`` per independently stepped range, like FSDP's flat parameters -- while
``state_dict()`` / ``load_state_dict()`` speak the reference's per-layer keys.  Autograd is
wired through ``torch.autograd.Function``s whose backward runs the engine's hand-written
backward, so the reference's training loop shape works unchanged::

    loss = module.training_step(batch, i)       # forward + losses + centre + teacher EMA
    optimizer.zero_grad(); loss.backward()      # engine backward -> arena .grad
    optimizer.step()                            # FlatAdam: one kernel per arena

(Lightning's automatic optimisation runs exactly this inside ``optimizer.step(closure)``.)
``training_step`` uses the fused path (losses and their gradient seeds computed inside the
engine's forward); ``model(batch)`` is the general differentiable path whose outputs can feed
any loss -- both produce the same gradients (tests/test_gpu_boundary.py).
"""
import math
from collections import OrderedDict

import torch
import torch.nn as nn

from . import contrastive, ops
from .engine import Hyper, MultiCentralEngine, SimCLREngine, UniModalEngine, Workspace, ema_step
from .params import ParamStore
from .spec import MULTI_ENCODERS, multimodal_dino_sd, simclr_sd, unimodal_dino_sd

try:  # a real drop-in under Lightning's Trainer where Lightning is installed
    from lightning.pytorch import LightningModule as _LightningBase
    HAVE_LIGHTNING = True
except ImportError:  # this image: the module protocol is plain nn.Module + avdino.trainer
    _LightningBase = nn.Module
    HAVE_LIGHTNING = False

_DT = {"bf16": torch.bfloat16, "16-mixed": torch.bfloat16, "bf16-mixed": torch.bfloat16,
       "32": torch.float32, "fp32": torch.float32, "f32": torch.float32}


# ============================================================================ encoders
class BaseMultiModalEncoder:
    """models/dino.py:203-211 -- descriptor base (the compute is the engine's)."""

    arch = None

    def __init__(self, output_dim=256, encoder_output_dim=512, fusion_dropout=0.3):
        self.output_dim = output_dim
        self.encoder_output_dim = encoder_output_dim
        self.fusion_dropout = fusion_dropout


class SimpleMultiModalEncoder(BaseMultiModalEncoder):
    """image_encoder(E) (3x3 CNN 1->32->64->128, GAP, Linear(128,E)) and audio_encoder(E)
    (1->32->64->128->256, GAP, Linear(256,E)), concat fusion Linear(2E,E)-ReLU-
    Dropout(fusion_dropout)-Linear(E,D) (models/dino.py:18-73, 214-234)."""

    arch = "multi_simple"


class CentralMultiModalEncoder(BaseMultiModalEncoder):
    """CentralNet LeNet image (conv5x5 1->32->64) and audio (conv5x5 1->8->16->32->64)
    branches + Linear(., E) each, concat fusion Linear(2E,E)-ReLU-Dropout(0.3)-Linear(E,D)
    (models/dino.py:454-468, unimodal.py:105-221, fusion 214-234)."""

    arch = "multi_central"

    def __init__(self, output_dim=256, encoder_output_dim=512):
        super().__init__(output_dim, encoder_output_dim, fusion_dropout=0.3)


class ProjectionHead:
    """Linear(in, 512) -> BatchNorm1d -> GELU -> Dropout -> Linear(512, out) (dino.py:1240-1254)."""

    def __init__(self, input_dim, projection_dim=256, dropout_rate=0, hidden_dim=512):
        self.input_dim, self.projection_dim = input_dim, projection_dim
        self.dropout_rate, self.hidden_dim = dropout_rate, hidden_dim


class BaseUniModalEncoder:
    """models/dino.py:471-480 -- descriptor base (output_dim, modality)."""

    kind = None
    modality = None

    def __init__(self, output_dim=256):
        self.output_dim = output_dim


class ImageEncoder(BaseUniModalEncoder):
    """image_encoder(512) 3x3 CNN 1->32->64->128, GAP, Linear(128,512), projection
    Linear(512, output_dim) (models/dino.py:18-42, 483-499)."""
    kind, modality = "image_simple", "image"


class SpectrogramEncoder(BaseUniModalEncoder):
    """audio_encoder(output_dim) 3x3 CNN 1->32->64->128->256, GAP, Linear(256, output_dim)
    (models/dino.py:44-73, 502-513)."""
    kind, modality = "spectrogram_simple", "audio"


class SpectrogramEncoderCentral(SpectrogramEncoder):
    """CentralUnimodalAudio + Linear(3136, output_dim) (models/dino.py:515-523)."""
    kind = "spectrogram_central"


MODEL_MAP = {"multi_simple": SimpleMultiModalEncoder, "multi_central": CentralMultiModalEncoder}
UNIMODAL_MODEL_MAP = {"image_simple": ImageEncoder, "spectrogram_simple": SpectrogramEncoder,
                      "spectrogram_central": SpectrogramEncoderCentral}


def _device(device):
    if device is not None:
        return torch.device(device)
    return torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")


# ============================================================================ arena modules
class _ArenaModule(nn.Module):
    """An nn.Module backed by a ParamStore.

    Parameters: the trainable arena ranges (``arena`` or one per SimCLR tower), the frozen
    student tail (the CentralNet fc1/fc2 the reference builds but never runs: no gradient, like
    the reference's grad=None) and the teacher arena (requires_grad=False, as the reference's
    teacher).  Buffers: the running-stat/centre arena and the num_batches_tracked counters, so
    torch DDP's ``broadcast_buffers`` moves rank 0's in two collectives.  The arenas stay where
    they were built: moving the module to another device or dtype raises (rebuild instead)."""

    def _bind(self, store, ranges):
        self.store = store
        self._trainable = []
        for name, o, n in ranges:
            self.register_parameter(name, nn.Parameter(store.student[o:o + n]))
            self._trainable.append(name)
        hi = max(o + n for _, o, n in ranges)
        if store.student.numel() > hi:
            self.register_parameter("arena_frozen", nn.Parameter(store.student[hi:], requires_grad=False))
        if store.teacher is not None:
            self.register_parameter("teacher_arena", nn.Parameter(store.teacher, requires_grad=False))
        self.register_buffer("buffer_arena", store.buf_arena, persistent=False)
        self.register_buffer("counter_arena", store.nbt_arena, persistent=False)

    def trainable_arenas(self):
        return [getattr(self, n) for n in self._trainable]

    def _apply(self, fn, recurse=True):
        for t in list(self.parameters()) + list(self.buffers()):
            out = fn(t)
            if out.data_ptr() != t.data_ptr() or out.dtype != t.dtype:
                raise RuntimeError(f"{type(self).__name__} lives in its {t.device} arenas; build a new "
                                   f"model on the target device instead of moving it")
        return self

    # ---- reference state-dict keys (nn.Module's recursive save/load call these)
    def state_dict(self, *args, destination=None, prefix="", keep_vars=False):
        if destination is None:
            destination = OrderedDict()
        for k, v in self.store.state_dict().items():
            destination[prefix + k] = v if keep_vars else v.detach()
        return destination

    def _load_from_state_dict(self, state_dict, prefix, local_metadata, strict, missing_keys,
                              unexpected_keys, error_msgs):
        own = {}
        for k, v in state_dict.items():
            if k.startswith(prefix):
                key = k[len(prefix):]
                if key in self.store.spec:
                    own[key] = v
                elif strict:
                    unexpected_keys.append(k)
        for k in self.store.spec:
            if k not in own:
                missing_keys.append(prefix + k)
        try:
            self.store.load_state_dict(own, strict=False)
        except (ValueError, KeyError) as e:
            error_msgs.append(str(e))

    def load_state_dict(self, state_dict, strict=True, assign=False):
        return super().load_state_dict(state_dict, strict=strict)

    def reference_named_parameters(self):
        """(reference key, tensor view) for every parameter, as the reference's
        named_parameters() lists them (student, projections, heads, teacher)."""
        for k in self.store.spec:
            if k in self.store.s_offs or k in self.store.t_offs:
                yield k, self.store[k]

    @property
    def center(self):
        return self.store["center"]

    def _need_engine(self):
        if self.engine is None:
            raise RuntimeError("the HIP engine needs a ROCm device (no CPU fallback)")
        return self.engine


def _finish_backward(eng):
    """After an engine backward: the data-parallel gradient exchange (if any), then the dropout
    counter moves on (forward and backward of a step share its masks)."""
    if getattr(eng, "grad_hook", None) is not None:
        eng.grad_hook(eng.store.grad)
    eng.step_idx = getattr(eng, "step_idx", 0) + 1


def _begin_backward(eng):
    """Before an engine backward: a new gradient exchange (its early buckets fire inside)."""
    hook = getattr(eng, "grad_hook", None)
    if hasattr(hook, "begin"):
        hook.begin()


def _begin_forward(eng):
    """Before an engine forward: the data-parallel buffer broadcast (DDP broadcast_buffers)."""
    if getattr(eng, "buffer_hook", None) is not None:
        eng.buffer_hook(eng.store)


def _check_token(ctx):
    if ctx.eng.fwd_count != ctx.token:
        raise RuntimeError("backward of a stale forward: the engine keeps the saved state of its "
                           "latest forward only (call backward before the next forward)")


class _FusedStepFn(torch.autograd.Function):
    """training_step's fused path: engine forward with every loss and its gradient seed computed
    in-kernel -> scalar loss; backward = the engine backward -> gradient of each arena."""

    @staticmethod
    def forward(ctx, eng, batch, ranges, *arenas):
        _begin_forward(eng)
        loss = eng.forward(batch, training=True)
        ctx.eng, ctx.token, ctx.ranges = eng, eng.fwd_count, ranges
        return loss.clone().view(())   # a fresh tensor: the engine's slot is reused next step

    @staticmethod
    def backward(ctx, g):
        _check_token(ctx)
        eng = ctx.eng
        _begin_backward(eng)
        eng.backward()
        _finish_backward(eng)
        return (None, None, None) + _arena_grads(eng, ctx.ranges, g)


def _arena_grads(eng, ranges, g):
    used = getattr(eng, "used_towers", None)
    used = set(used()) if used is not None else None
    out = []
    for i, (o, n) in enumerate(ranges):
        if used is not None and i not in used:
            out.append(None)           # tower not run this step: grad stays None (Adam skips it)
        else:
            out.append(eng.store.grad[o:o + n] * g)
    return tuple(out)


# ============================================================================ multimodal DINO
class _MultiForwardFn(torch.autograd.Function):
    """MultiModalDINO*.forward with autograd: outputs (s [V,B,P], t [G,B,P] (no grad) [, image
    head, audio head]); backward feeds d s and d heads into the engine backward."""

    @staticmethod
    def forward(ctx, eng, batch, ranges, *arenas):
        _begin_forward(eng)
        eng.forward(batch, training=True)
        s, t = eng.outputs()
        outs = [s.clone(), t.clone()]
        if eng.heads is not None:
            zi, za = eng.last_head_outputs()
            outs += [zi.clone(), za.clone()]
        ctx.eng, ctx.token, ctx.ranges = eng, eng.fwd_count, ranges
        ctx.mark_non_differentiable(outs[1])
        return tuple(outs)

    @staticmethod
    def backward(ctx, ds, _dt, *dh):
        _check_token(ctx)
        eng = ctx.eng
        c = eng.last
        n = c["V"] * c["B"] * eng.P

        def seed(g, numel, dev):
            return torch.zeros(numel, device=dev) if g is None else g.float().contiguous().view(-1)

        dev = eng.store.device
        dheads = None
        if dh:
            no = eng.heads[0].o
            dheads = (seed(dh[0], c["B"] * no, dev), seed(dh[1], c["B"] * no, dev))
        _begin_backward(eng)
        eng.backward(ds=seed(ds, n, dev), dheads=dheads)
        _finish_backward(eng)
        return (None, None, None) + _arena_grads(eng, ctx.ranges, 1.0)


class _StudentView:
    """What the reference's downstream code reads off ``model.student``: output_dim (and
    modality for unimodal encoders) -- the weights stay in the owner's ParamStore."""

    def __init__(self, owner, kind, output_dim, encoder_output_dim=None, modality=None):
        self.owner, self.kind = owner, kind
        self.output_dim, self.encoder_output_dim = output_dim, encoder_output_dim
        if modality is not None:
            self.modality = modality

    def parameters(self):
        return iter(self.owner.trainable_arenas())


class MultiModalDINO(_ArenaModule):
    """Student/teacher multimodal DINO (models/dino.py:588-727) on the HIP engine."""

    mode = "default"

    def __init__(self, encoder_class=CentralMultiModalEncoder, encoder_kwargs=None, output_dim=256,
                 encoder_output_dim=512, projection_dim=128, momentum=0.996, center_momentum=0.9,
                 dropout=0.3, device=None, precision="bf16", seed=0, negatives="global", group=None):
        super().__init__()
        encoder_kwargs = dict(encoder_kwargs or {})
        encoder_kwargs["output_dim"] = output_dim
        encoder_kwargs["encoder_output_dim"] = encoder_output_dim
        enc = encoder_class(**encoder_kwargs)
        if getattr(enc, "arch", None) not in MULTI_ENCODERS:
            raise NotImplementedError(
                f"{encoder_class.__name__}: the MI355X engine runs {sorted(MULTI_ENCODERS)} "
                f"(SimpleMultiModalEncoder / CentralMultiModalEncoder)")
        self.student_spec = enc
        self.projection_dim, self.output_dim = projection_dim, output_dim
        self.encoder_output_dim = encoder_output_dim
        self.momentum, self.center_momentum, self.dropout = momentum, center_momentum, dropout
        self.device = _device(device)
        self.precision = precision
        store = ParamStore(multimodal_dino_sd(self.mode, encoder_output_dim, output_dim, projection_dim,
                                              encoder=enc.arch), self.device, seed=seed)
        self._bind(store, [("arena", 0, store.n_live)])
        self.hp = Hyper(momentum=momentum, center_momentum=center_momentum, dropout=dropout,
                        fusion_dropout=enc.fusion_dropout)
        self.engine = None
        if self.device.type == "cuda":
            self.engine = MultiCentralEngine(store, self.mode, encoder_output_dim, output_dim,
                                             projection_dim, self.hp, act_dtype=_DT[precision], seed=seed,
                                             negatives=negatives, group=group, encoder=enc.arch)
        self.student = _StudentView(self, enc.arch, output_dim, encoder_output_dim)

    def arena_ranges(self):
        return ((0, self.store.n_live),)

    # ---------------------------------------------------------------- reference methods
    @torch.no_grad()
    def update_teacher(self):
        """teacher <- m * teacher + (1-m) * student over ALL student params (dino.py:635-646)."""
        ema_step(self.store, self.momentum)

    @torch.no_grad()
    def update_center(self, teacher_output):
        """center <- 0.9 center + 0.1 mean_rows(teacher_output) (dino.py:648-653)."""
        c = self.store["center"]
        c.mul_(self.center_momentum).add_(teacher_output.reshape(-1, c.shape[1]).mean(0, keepdim=True)
                                          * (1 - self.center_momentum))

    @staticmethod
    def _views_dict(views):
        g_img, g_aud, l_img, l_aud = views
        return {"g_img": g_img, "g_aud": g_aud, "l_img": l_img, "l_aud": l_aud}

    def _batch(self, batch):
        return {k: v.to(self.device) for k, v in self._views_dict(batch).items()}

    def _run(self, b):
        if not self.training:
            raise NotImplementedError("eval-mode DINO forward: use FeatureExtractor / "
                                      "DownstreamClassifier (avdino.downstream) for frozen features")
        eng = self._need_engine()
        outs = _MultiForwardFn.apply(eng, b, self.arena_ranges(), *self.trainable_arenas())
        eng.update_center()                  # MultiModalDINO.forward updates the centre (717)
        return outs

    def forward(self, batch):
        """batch = (global_images, global_audios, local_images, local_audios), each
        [B, V, 1, H, W] -> (student_outputs [G+L,B,P], teacher_outputs [G,B,P] centred, None).
        Differentiable w.r.t. the student outputs; updates the centre, like the reference."""
        s, t = self._run(self._batch(batch))[:2]
        return s, t, None


class _WithHeads(MultiModalDINO):
    def _batch(self, batch):
        image, audio, views = batch[0], batch[1], batch[-1]
        b = self._views_dict(views)
        b.update(image=image, audio=audio)
        if self.mode == "semi_supervised":
            b["label"] = batch[2] if len(batch) == 4 else torch.zeros(image.shape[0], dtype=torch.long)
        return {k: v.to(self.device) for k, v in b.items()}

    def forward(self, batch):
        """batch = (image, audio, views) -> (image_out, audio_out, student_out, teacher_out);
        differentiable w.r.t. all but teacher_out."""
        s, t, zi, za = self._run(self._batch(batch))
        return zi, za, s, t


class MultiModalDINOWithMSE(_WithHeads):
    mode = "mse"


class MultiModalDINOWithINFONCE(_WithHeads):
    mode = "infonce"


class MultiModalDINOSemiSupervised(_WithHeads):
    mode = "semi_supervised"

    def __init__(self, *args, num_classes=10, **kwargs):
        if num_classes != 10:
            raise NotImplementedError("AVMNIST has 10 classes")
        self.num_classes = num_classes
        super().__init__(*args, **kwargs)


# ============================================================================ loss functions
class _DinoLossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, s, t, tau_s, tau_t, center_teacher):
        V, B, P = s.shape
        T = t.shape[0]
        s_ = s.detach().float().contiguous().view(V * B, P)
        t_ = t.detach().float().contiguous().view(T * B, P)
        zero = torch.zeros(P, device=s.device)
        parts = torch.empty(V * B, device=s.device)
        ds = torch.empty(V * B, P, device=s.device)
        cn = torch.empty(P, device=s.device)
        work = torch.empty((B + T * B) * P, device=s.device)
        ops.dino_loss(s_, t_, zero, V, T, B, P, tau_s, tau_t, 0.9, center_teacher, parts, ds, cn, work)
        loss = torch.empty(1, device=s.device)
        ops.sum_to(parts, V * B, 1.0, loss)
        ctx.save_for_backward(ds.view(V, B, P))
        return loss[0]

    @staticmethod
    def backward(ctx, g):
        (ds,) = ctx.saved_tensors
        return ds * g, None, None, None, None


class _MseLossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b):
        B, P = a.shape
        parts = torch.empty(B, device=a.device)
        da, db = torch.empty_like(a, dtype=torch.float32), torch.empty_like(b, dtype=torch.float32)
        ops.mse_loss(a.detach().float().contiguous(), b.detach().float().contiguous(), B, P, parts, da, db)
        loss = torch.empty(1, device=a.device)
        ops.sum_to(parts, B, 1.0, loss)
        ctx.save_for_backward(da, db)
        return loss[0]

    @staticmethod
    def backward(ctx, g):
        da, db = ctx.saved_tensors
        return da * g, db * g


class _InfoNCELossFn(torch.autograd.Function):
    """infoNCE_loss (dino.py:1091-1128) on one device: l2norm + MFMA GEMM + softmax-CE kernels."""

    @staticmethod
    def forward(ctx, zi, za, temperature):
        B, P = zi.shape
        ws = Workspace(zi.device)
        parts = torch.empty(2 * B, device=zi.device)
        dzi, dza = torch.empty(B * P, device=zi.device), torch.empty(B * P, device=zi.device)
        scale = contrastive.infonce(ws, zi.detach().float().contiguous().view(-1),
                                    za.detach().float().contiguous().view(-1), B, P, dzi, dza, parts,
                                    temperature, local=True)
        loss = torch.empty(1, device=zi.device)
        ops.sum_to(parts, 2 * B, scale, loss)
        ctx.save_for_backward(dzi.view(B, P), dza.view(B, P))
        return loss[0]

    @staticmethod
    def backward(ctx, g):
        dzi, dza = ctx.saved_tensors
        return dzi * g, dza * g, None


class _SupervisedLossFn(torch.autograd.Function):
    """supervised_loss (dino.py:1001-1025): CE(image logits) + CE(audio logits)."""

    @staticmethod
    def forward(ctx, li, la, labels):
        B, C = li.shape
        lab = labels.to(li.device).long().contiguous()
        parts = torch.empty(2 * B, device=li.device)
        di, da = torch.empty(B * C, device=li.device), torch.empty(B * C, device=li.device)
        ops.softmax_xent(li.detach().float().contiguous().view(-1), C, B, C, lab, 0, False, False,
                         1.0 / B, parts[:B], di, C, False)
        ops.softmax_xent(la.detach().float().contiguous().view(-1), C, B, C, lab, 0, False, False,
                         1.0 / B, parts[B:], da, C, False)
        loss = torch.empty(1, device=li.device)
        ops.sum_to(parts, 2 * B, 1.0 / B, loss)
        ctx.save_for_backward(di.view(B, C), da.view(B, C))
        return loss[0]

    @staticmethod
    def backward(ctx, g):
        di, da = ctx.saved_tensors
        return di * g, da * g, None


class _UniCosineLossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, emb):
        V, B, D = emb.shape
        e = emb.detach().float().contiguous()
        parts = torch.empty(B, device=emb.device)
        ops.cosine_consistency(e, V, B, D, 1.0, parts, None)
        d = torch.zeros(V * B * D, device=emb.device)
        ops.cosine_consistency(e, V, B, D, 1.0, None, d)
        loss = torch.empty(1, device=emb.device)
        ops.sum_to(parts, B, 1.0, loss)
        ctx.save_for_backward(d.view(V, B, D))
        return loss[0]

    @staticmethod
    def backward(ctx, g):
        (d,) = ctx.saved_tensors
        return d * g


class _NtXentFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, reps, temperature):
        N, P = reps.shape
        B = N // 2
        ws = Workspace(reps.device)
        parts = torch.empty(N, device=reps.device)
        d = torch.empty(N * P, device=reps.device)
        scale = contrastive.nt_xent(ws, reps.detach().float().contiguous().view(-1), B, P, d, parts,
                                    temperature, local=True)
        loss = torch.empty(1, device=reps.device)
        ops.sum_to(parts, N, scale, loss)
        ctx.save_for_backward(d.view(N, P))
        return loss[0]

    @staticmethod
    def backward(ctx, g):
        (d,) = ctx.saved_tensors
        return d * g, None


# ============================================================================ optimizer
class FlatAdam(torch.optim.Optimizer):
    """torch.optim.Adam (L2 added to the gradient) or AdamW (decoupled decay) over flat arena
    Parameters: one fused kernel per arena instead of one per tensor.  torch semantics kept:
    a parameter whose ``.grad`` is None is skipped and keeps its own step count (SimCLR's
    unused tower), ``step(closure)`` evaluates the closure first (Lightning's automatic
    optimisation runs training_step + zero_grad + backward inside it), and GradScaler's
    unscale_/step work on it like on any Optimizer."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0,
                 decoupled=False):
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay,
                                      decoupled=decoupled))

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for grp in self.param_groups:
            b1, b2 = grp["betas"]
            fn = ops.adamw if grp["decoupled"] else ops.adam
            for p in grp["params"]:
                if p.grad is None:
                    continue
                g = p.grad
                if g.dtype != torch.float32 or not g.is_contiguous():
                    raise RuntimeError("FlatAdam: expects contiguous fp32 arena gradients")
                st = self.state[p]
                if not st:
                    st["step"] = 0
                    st["exp_avg"] = torch.zeros_like(p)
                    st["exp_avg_sq"] = torch.zeros_like(p)
                st["step"] += 1
                t = st["step"]
                fn(p, g, st["exp_avg"], st["exp_avg_sq"], p.numel(), grp["lr"], b1, b2, grp["eps"],
                   grp["weight_decay"], 1 - b1 ** t, 1 - b2 ** t)
        return loss


def _cosine(opt, T_max):
    return torch.optim.lr_scheduler.CosineAnnealingLR(opt, T_max=T_max)


# ============================================================================ Lightning-shaped
class _LightningShaped(_LightningBase):
    """What the wrappers share: hparams, logging, the reference's forward/state-dict surface."""

    def _set_hparams(self, hp):
        if HAVE_LIGHTNING:
            self.save_hyperparameters(hp)
        else:
            self.hparams = hp

    if not HAVE_LIGHTNING:
        def log(self, name, value, **kw):
            """LightningModule.log stand-in: the last value and the running mean per key."""
            v = value.detach() if torch.is_tensor(value) else value
            self.logged[name] = v
            self.logged_history.setdefault(name, []).append(v)

    def forward(self, batch):
        return self.model(batch)

    @classmethod
    def load_from_checkpoint(cls, checkpoint_path, map_location=None, strict=True, **kwargs):
        """LightningModule.load_from_checkpoint (run_dino.py:386): rebuild from the
        checkpoint's hyper_parameters (kwargs override them, e.g. device=...), then load its
        state_dict (the reference's ``model.…`` keys)."""
        import inspect
        from .trainer import load_checkpoint
        ck = load_checkpoint(checkpoint_path)
        hp = dict(ck.get("hyper_parameters") or {})
        hp.update(kwargs)
        enc = hp.get("encoder_class")
        if isinstance(enc, str):
            known = {c.__name__: c for c in list(MODEL_MAP.values()) + list(UNIMODAL_MODEL_MAP.values())}
            hp["encoder_class"] = known[enc]
        params = inspect.signature(cls.__init__).parameters
        if not any(p.kind == p.VAR_KEYWORD for p in params.values()):
            hp = {k: v for k, v in hp.items() if k in params}
        m = cls(**hp)
        m.load_state_dict(ck["state_dict"], strict=strict)
        return m


class MultiModalDINOLightning(_LightningShaped):
    """Training wrapper (models/dino.py:730-962)."""

    model_class = MultiModalDINO

    def __init__(self, data_dir="data/avmnist", data_augmentation="burst_noise", dino_model=None,
                 encoder_class=CentralMultiModalEncoder, encoder_kwargs=None, projection_dim=256,
                 output_dim=256, encoder_output_dim=512, momentum=0.996, center_momentum=0.9,
                 student_temperature=0.1, teacher_temperature=0.04, learning_rate=0.0001,
                 use_mixed_precision=True, num_epochs=100, weight_decay=1e-6, dropout=0.3,
                 alpha=1, device=None, precision=None, seed=0, traindata=None, validdata=None,
                 negatives="global", group=None):
        super().__init__()
        self._set_hparams(dict(data_dir=data_dir, data_augmentation=data_augmentation,
                               encoder_class=encoder_class.__name__, encoder_kwargs=encoder_kwargs,
                               projection_dim=projection_dim, output_dim=output_dim,
                               encoder_output_dim=encoder_output_dim, momentum=momentum,
                               center_momentum=center_momentum,
                               student_temperature=student_temperature,
                               teacher_temperature=teacher_temperature, learning_rate=learning_rate,
                               use_mixed_precision=use_mixed_precision, num_epochs=num_epochs,
                               weight_decay=weight_decay, dropout=dropout, alpha=alpha))
        self.encoder_class, self.encoder_kwargs = encoder_class, encoder_kwargs
        self.output_dim, self.encoder_output_dim = output_dim, encoder_output_dim
        self.projection_dim = projection_dim
        self.momentum, self.center_momentum, self.dropout = momentum, center_momentum, dropout
        self.learning_rate, self.num_epochs = learning_rate, num_epochs
        self.student_temperature, self.teacher_temperature = student_temperature, teacher_temperature
        self.use_mixed_precision = use_mixed_precision
        self.weight_decay, self.alpha = weight_decay, alpha
        self.precision = precision or ("bf16" if use_mixed_precision else "32")
        self.logged, self.logged_history = {}, {}
        # the epoch-end probe's loaders (the reference builds AVMNISTDataModule(batch 128) here,
        # dino.py:795-802); None until set -- on_train_epoch_end is a no-op without them
        self.traindata, self.validdata = traindata, validdata
        if dino_model is None:
            dino_model = self.model_class(encoder_class=encoder_class, encoder_kwargs=encoder_kwargs,
                                          output_dim=output_dim, encoder_output_dim=encoder_output_dim,
                                          projection_dim=projection_dim, momentum=momentum,
                                          center_momentum=center_momentum, dropout=dropout,
                                          device=device, precision=self.precision, seed=seed,
                                          negatives=negatives, group=group)
        self.model = dino_model
        hp = self.model.hp
        hp.tau_s, hp.tau_t = student_temperature, teacher_temperature
        hp.lr, hp.wd, hp.alpha = learning_rate, weight_decay, float(alpha)

    # ---------------------------------------------------------------- losses (reference API)
    def dino_loss(self, student_outputs, teacher_outputs, alignment_loss=None):
        """dino.py:822-854 -- fused HIP kernel; differentiable w.r.t. student_outputs."""
        return _DinoLossFn.apply(student_outputs, teacher_outputs, self.student_temperature,
                                 self.teacher_temperature, False)

    def mse_loss(self, image_outputs, audio_outputs):
        """dino.py:1193-1211."""
        return _MseLossFn.apply(image_outputs, audio_outputs)

    def infoNCE_loss(self, image_outputs, audio_outputs, temperature=0.07):
        """dino.py:1091-1128 (this device's batch as negatives)."""
        return _InfoNCELossFn.apply(image_outputs, audio_outputs, temperature)

    def supervised_loss(self, image_logits, audio_logits, labels):
        """dino.py:1001-1025."""
        return _SupervisedLossFn.apply(image_logits, audio_logits, labels)

    # ---------------------------------------------------------------- step
    def _batch_dict(self, batch):
        if isinstance(batch, dict) and "aug" in batch:
            return batch       # AVMNISTDinoLoader(staged=True): the engine augments into its inputs
        if self.model.mode == "default":
            d = self.model._views_dict(batch)
        else:
            image, audio, labels, views = batch
            d = self.model._views_dict(views)
            d.update(image=image, audio=audio, label=labels)
        return {k: v.to(self.model.device, non_blocking=True) for k, v in d.items()}

    def prefetch(self, batch):
        """Trainer hook (after the optimizer step of the current batch): queue the NEXT batch's
        device augmentation under the step just issued (MultiCentralEngine.prefetch); only for
        staged real-data batches, a no-op otherwise."""
        eng = getattr(self.model, "engine", None)
        if isinstance(batch, dict) and "aug" in batch and hasattr(eng, "prefetch"):
            return eng.prefetch(batch)
        return False

    def training_step(self, batch, batch_idx):
        """Forward + losses (+ centre update) + teacher EMA before backward (dino.py:856-876,
        1027-1051, 1130-1154, 1214-1238) on the fused path.  Returns the differentiable loss."""
        m = self.model
        eng = m._need_engine()
        loss = _FusedStepFn.apply(eng, self._batch_dict(batch), m.arena_ranges(), *m.trainable_arenas())
        eng.update_center()
        m.update_teacher()
        self.log("train_loss", loss, on_step=True, on_epoch=True, prog_bar=True)
        return loss

    def reference_training_step(self, batch, batch_idx):
        """The reference's training_step composed literally: model(batch) -> loss methods ->
        update_teacher (same gradients as training_step, through the general path)."""
        if self.model.mode == "default":
            s, t, align = self.model(batch)
            loss = self.dino_loss(s, t, align)
        else:
            image, audio, labels, views = batch
            fi, fa, s, t = self.model((image, audio, labels, views))
            aux = {"mse": lambda: self.mse_loss(fi, fa), "infonce": lambda: self.infoNCE_loss(fi, fa),
                   "semi_supervised": lambda: self.supervised_loss(fi, fa, labels)}[self.model.mode]()
            loss = self.dino_loss(s, t) + self.alpha * aux
        self.model.update_teacher()
        self.log("train_loss", loss, on_step=True, on_epoch=True, prog_bar=True)
        return loss

    def configure_optimizers(self):
        """Adam(lr, weight_decay) + CosineAnnealingLR(T_max=num_epochs) (dino.py:953-962)."""
        opt = FlatAdam(self.model.trainable_arenas(), lr=self.learning_rate,
                       weight_decay=self.weight_decay)
        return {"optimizer": opt, "lr_scheduler": {"scheduler": _cosine(opt, self.num_epochs)}}

    def _probe_kind(self):
        enc = self.model.student_spec
        return getattr(enc, "kind", None) or enc.arch

    def on_train_epoch_end(self, traindata=None, validdata=None):
        """Linear probe (dino.py:878-951 / 1670-1735) over iterables of (images, audios,
        labels) batches (the reference's AVMNIST loaders, batch 128); logs val_loss and
        mlp_acc.  No data (none given and none set at construction): nothing to do."""
        traindata = traindata if traindata is not None else self.traindata
        validdata = validdata if validdata is not None else self.validdata
        if traindata is None or validdata is None:
            return None
        from .probe import LinearProbe
        m = self.model
        probe = LinearProbe(m.store, self._probe_kind(), m.output_dim,
                            getattr(m, "encoder_output_dim", None), lr=self.learning_rate,
                            act_dtype=_DT[self.precision],
                            fusion_dropout=getattr(m.hp, "fusion_dropout", 0.3))
        out = probe.run_epoch(traindata, validdata)
        self.log("val_loss", out["val_loss"])
        self.log("mlp_acc", out["mlp_acc"], on_epoch=True, prog_bar=True)
        return out

    def state_dict(self, *args, destination=None, prefix="", keep_vars=False):
        return self.model.state_dict(destination=destination, prefix=prefix + "model.",
                                     keep_vars=keep_vars)


class MultiModalDINOWithMSELightning(MultiModalDINOLightning):
    """dino.py:1173-1238 (reference ctor defaults encoder_output_dim=128)."""

    model_class = MultiModalDINOWithMSE

    def __init__(self, *args, output_dim=256, encoder_output_dim=128,
                 encoder_class=CentralMultiModalEncoder, alpha=1, **kwargs):
        super().__init__(*args, output_dim=output_dim, encoder_output_dim=encoder_output_dim,
                         encoder_class=encoder_class, alpha=alpha, **kwargs)


class MultiModalDINOWithINFONCELightning(MultiModalDINOLightning):
    """dino.py:1070-1154."""

    model_class = MultiModalDINOWithINFONCE

    def __init__(self, *args, output_dim=256, encoder_output_dim=128,
                 encoder_class=CentralMultiModalEncoder, alpha=1, **kwargs):
        super().__init__(*args, output_dim=output_dim, encoder_output_dim=encoder_output_dim,
                         encoder_class=encoder_class, alpha=alpha, **kwargs)


class MultiModalDINOSemiSupervisedLightning(MultiModalDINOLightning):
    """dino.py:982-1051."""

    model_class = MultiModalDINOSemiSupervised


MULTIMODAL_WRAPPERS = {
    "default": MultiModalDINOLightning,
    "semi_supervised": MultiModalDINOSemiSupervisedLightning,
    "mse": MultiModalDINOWithMSELightning,
    "infonce": MultiModalDINOWithINFONCELightning,
}


# ============================================================================ unimodal DINO
class _UniForwardFn(torch.autograd.Function):
    """UniModalDINO.forward with autograd: (s [V,B,P], t [G,B,P] (no grad), embeddings [V,B,D])."""

    @staticmethod
    def forward(ctx, eng, batch, ranges, *arenas):
        _begin_forward(eng)
        eng.forward(batch, training=True)
        s, t, e = eng.outputs()
        ctx.eng, ctx.token, ctx.ranges = eng, eng.fwd_count, ranges
        outs = (s.clone(), t.clone(), e.clone())
        ctx.mark_non_differentiable(outs[1])
        return outs

    @staticmethod
    def backward(ctx, ds, _dt, de):
        _check_token(ctx)
        eng = ctx.eng
        c = eng.last
        dev = eng.store.device
        ds = (torch.zeros(c["V"] * c["B"] * eng.P, device=dev) if ds is None
              else ds.float().contiguous().view(-1))
        de = None if de is None else de.float().contiguous().view(-1)
        if de is None:
            de = torch.zeros(c["V"] * c["B"] * eng.D, device=dev)
        _begin_backward(eng)
        eng.backward(ds=ds, demb=de)
        _finish_backward(eng)
        return (None, None, None) + _arena_grads(eng, ctx.ranges, 1.0)


class UniModalDINO(_ArenaModule):
    """Student/teacher unimodal DINO (models/dino.py:1257-1398) on the HIP engine."""

    def __init__(self, encoder_class=ImageEncoder, encoder_kwargs=None, output_dim=256,
                 projection_dim=128, momentum=0.996, center_momentum=0.9, dropout=0.3,
                 device=None, precision="bf16", seed=0, cosine_loss_alpha=0.0):
        super().__init__()
        encoder_kwargs = dict(encoder_kwargs or {})
        encoder_kwargs["output_dim"] = output_dim
        enc = encoder_class(**encoder_kwargs)
        if getattr(enc, "kind", None) is None:
            raise NotImplementedError(
                f"{encoder_class.__name__}: the MI355X engine runs ImageEncoder, SpectrogramEncoder "
                f"and SpectrogramEncoderCentral")
        self.student_spec = enc
        self.projection_dim, self.output_dim = projection_dim, output_dim
        self.momentum, self.center_momentum, self.dropout = momentum, center_momentum, dropout
        self.device = _device(device)
        self.precision = precision
        store = ParamStore(unimodal_dino_sd(enc.kind, output_dim, projection_dim), self.device,
                           seed=seed)
        self._bind(store, [("arena", 0, store.n_live)])
        self.hp = Hyper(momentum=momentum, center_momentum=center_momentum, dropout=dropout)
        self.engine = None
        if self.device.type == "cuda":
            self.engine = UniModalEngine(store, enc.kind, output_dim, projection_dim, self.hp,
                                         act_dtype=_DT[precision], cos_alpha=cosine_loss_alpha,
                                         seed=seed)
        self.student = _StudentView(self, enc.kind, output_dim, modality=enc.modality)

    arena_ranges = MultiModalDINO.arena_ranges
    update_teacher = MultiModalDINO.update_teacher
    update_center = MultiModalDINO.update_center

    def forward(self, batch):
        """batch = (global_images, global_audios, local_images, local_audios) -> (student_outputs
        [G+L,B,P], teacher_outputs [G,B,P] centred, embeddings [G+L,B,D]); updates the centre.
        Differentiable w.r.t. the student outputs and the embeddings."""
        if not self.training:
            raise NotImplementedError("eval-mode DINO forward: use avdino.downstream.FeatureExtractor")
        eng = self._need_engine()
        b = {k: v.to(self.device) for k, v in MultiModalDINO._views_dict(batch).items()}
        outs = _UniForwardFn.apply(eng, b, self.arena_ranges(), *self.trainable_arenas())
        eng.update_center()
        return outs


class UniModalDINOLightning(MultiModalDINOLightning):
    """models/dino.py:1490-1759: unimodal DINO loss (teacher centred per view) + optional
    cosine-consistency term (cosine_loss_alpha, default 0.3), EMA before backward, Adam(L2)."""

    model_class = UniModalDINO

    def __init__(self, data_dir="data/avmnist", dino_model=None, encoder_class=ImageEncoder,
                 encoder_kwargs=None, projection_dim=128, output_dim=256, momentum=0.996,
                 center_momentum=0.9, student_temperature=0.1, teacher_temperature=0.04,
                 learning_rate=0.0001, use_mixed_precision=True, weight_decay=1e-6,
                 cosine_loss_alpha=0.3, dropout=0.3, num_epochs=10, data_augmentation="burst_noise",
                 use_original_model=True, device=None, precision=None, seed=0, traindata=None,
                 validdata=None):
        _LightningShaped.__init__(self)
        self._set_hparams(dict(data_dir=data_dir, encoder_class=encoder_class.__name__,
                               encoder_kwargs=encoder_kwargs, projection_dim=projection_dim,
                               output_dim=output_dim, momentum=momentum,
                               center_momentum=center_momentum,
                               student_temperature=student_temperature,
                               teacher_temperature=teacher_temperature, learning_rate=learning_rate,
                               use_mixed_precision=use_mixed_precision, weight_decay=weight_decay,
                               cosine_loss_alpha=cosine_loss_alpha, dropout=dropout,
                               num_epochs=num_epochs, data_augmentation=data_augmentation))
        if not use_original_model:
            raise NotImplementedError("UniModalDINOV2 is not on the MI355X hot path")
        self.learning_rate, self.num_epochs = learning_rate, num_epochs
        self.student_temperature, self.teacher_temperature = student_temperature, teacher_temperature
        self.weight_decay, self.cosine_loss_alpha = weight_decay, cosine_loss_alpha
        self.output_dim, self.projection_dim = output_dim, projection_dim
        self.precision = precision or ("bf16" if use_mixed_precision else "32")
        self.logged, self.logged_history = {}, {}
        self.traindata, self.validdata = traindata, validdata
        if dino_model is None:
            dino_model = UniModalDINO(encoder_class=encoder_class, encoder_kwargs=encoder_kwargs,
                                      output_dim=output_dim, projection_dim=projection_dim,
                                      momentum=momentum, center_momentum=center_momentum,
                                      dropout=dropout, device=device, precision=self.precision,
                                      seed=seed, cosine_loss_alpha=cosine_loss_alpha)
        self.model = dino_model
        hp = self.model.hp
        hp.tau_s, hp.tau_t = student_temperature, teacher_temperature
        hp.lr, hp.wd = learning_rate, weight_decay

    def dino_loss(self, student_outputs, teacher_outputs):
        """dino.py:1596-1635 (teacher additionally centred by its per-view batch mean)."""
        return _DinoLossFn.apply(student_outputs, teacher_outputs, self.student_temperature,
                                 self.teacher_temperature, True)

    def _cosine_consistency_loss(self, embeddings):
        """dino.py:1575-1594."""
        return _UniCosineLossFn.apply(embeddings)

    def _batch_dict(self, batch):
        return {k: v.to(self.model.device, non_blocking=True)
                for k, v in MultiModalDINO._views_dict(batch).items()}

    def reference_training_step(self, batch, batch_idx):
        """dino.py:1637-1668 composed literally through the general path."""
        s, t, emb = self.model(batch)
        loss = self.dino_loss(s, t)
        if self.cosine_loss_alpha > 0:
            cos = self._cosine_consistency_loss(emb)
            loss = loss + self.cosine_loss_alpha * cos
            self.log("cosine_loss", cos, on_step=True, on_epoch=True, prog_bar=True)
        self.model.update_teacher()
        self.log("train_loss", loss, on_step=True, on_epoch=True, prog_bar=True)
        return loss


# ============================================================================ multimodal SimCLR
class MultiModalSimCLRModel(_ArenaModule):
    """other_ssl/multimodal_simclr/multimodal_simclr.py:12-47 on the HIP engine: ImageEncoder +
    SpectrogramEncoder towers with ProjectionHead(output_dim, projection_dim) each; one arena
    Parameter per tower (``arena_image``, ``arena_audio``)."""

    def __init__(self, output_dim=256, projection_dim=256, device=None, precision="bf16", seed=0,
                 negatives="global", mode_seed=1234, group=None):
        super().__init__()
        self.output_dim, self.projection_dim = output_dim, projection_dim
        self.device = _device(device)
        store = ParamStore(simclr_sd(output_dim, projection_dim), self.device, seed=seed,
                           has_teacher=False, groups=SimCLREngine.GROUPS)
        self._ranges = tuple(store.group_range(i) for i in range(2))
        self._bind(store, [("arena_image",) + self._ranges[0], ("arena_audio",) + self._ranges[1]])
        self.hp = Hyper(weight_decay=0.0)
        self.engine = None
        if self.device.type == "cuda":
            self.engine = SimCLREngine(store, output_dim, projection_dim, self.hp,
                                       act_dtype=_DT[precision], negatives=negatives, seed=mode_seed,
                                       group=group)

    def arena_ranges(self):
        return self._ranges

    @staticmethod
    def _batch_dict(batch):
        img1, spec1, img2, spec2 = batch
        return {"img1": img1, "spec1": spec1, "img2": img2, "spec2": spec2}

    def forward(self, batch, mode=None):
        """batch = (aug_img1, aug_spec1, aug_img2, aug_spec2) -> (z1, z2) [B, projection_dim],
        differentiable; the modality pair is drawn on the host per call (line 32)."""
        eng = self._need_engine()
        b = {k: v.to(self.device).float() for k, v in self._batch_dict(batch).items()}
        return _SimCLRForwardFn.apply(eng, b, mode, self.arena_ranges(), *self.trainable_arenas())


class _SimCLRForwardFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, eng, batch, mode, ranges, *arenas):
        _begin_forward(eng)
        eng.forward(batch, mode)
        z1, z2 = eng.outputs()
        ctx.eng, ctx.token, ctx.ranges = eng, eng.fwd_count, ranges
        return z1.clone(), z2.clone()

    @staticmethod
    def backward(ctx, d1, d2):
        _check_token(ctx)
        eng = ctx.eng
        B, P = eng.last["B"], eng.P
        dev = eng.store.device
        z = torch.zeros(B, P, device=dev)
        dreps = torch.cat([z if d1 is None else d1.float(), z if d2 is None else d2.float()]).view(-1)
        _begin_backward(eng)
        eng.backward(dreps=dreps)
        _finish_backward(eng)
        return (None, None, None, None) + _arena_grads(eng, ctx.ranges, 1.0)


class _SimCLRFusedFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, eng, batch, mode, ranges, *arenas):
        _begin_forward(eng)
        loss = eng.forward(batch, mode)
        ctx.eng, ctx.token, ctx.ranges = eng, eng.fwd_count, ranges
        return loss.clone().view(())

    @staticmethod
    def backward(ctx, g):
        _check_token(ctx)
        eng = ctx.eng
        _begin_backward(eng)
        eng.backward()
        _finish_backward(eng)
        return (None, None, None, None) + _arena_grads(eng, ctx.ranges, g)


class MultiModalSimCLRLightning(_LightningShaped):
    """multimodal_simclr.py:49-112: training_step = forward (random modality pair) + NT-Xent;
    Adam(lr) without weight decay, stepped only on the tower(s) used (their grads; the other
    tower's grad stays None), CosineAnnealingLR(T_max=num_epochs)."""

    def __init__(self, projection_dim=256, output_dim=256, learning_rate=0.0001, num_epochs=100,
                 use_mixed_precision=True, device=None, precision=None, seed=0, negatives="global",
                 mode_seed=1234, group=None):
        super().__init__()
        self._set_hparams(dict(projection_dim=projection_dim, output_dim=output_dim,
                               learning_rate=learning_rate, num_epochs=num_epochs,
                               use_mixed_precision=use_mixed_precision))
        self.output_dim, self.projection_dim = output_dim, projection_dim
        self.learning_rate, self.num_epochs = learning_rate, num_epochs
        self.use_mixed_precision = use_mixed_precision
        self.precision = precision or ("bf16" if use_mixed_precision else "32")
        self.logged, self.logged_history = {}, {}
        self.model = MultiModalSimCLRModel(output_dim, projection_dim, device, self.precision, seed,
                                           negatives, mode_seed, group)

    def nt_xent_loss(self, reps, temperature=0.07):
        """multimodal_simclr.py:74-89 (fused HIP kernels; differentiable w.r.t. reps)."""
        return _NtXentFn.apply(reps, temperature)

    def training_step(self, batch, batch_idx, mode=None):
        m = self.model
        eng = m._need_engine()
        b = {k: v.to(m.device, non_blocking=True).float() for k, v in m._batch_dict(batch).items()}
        loss = _SimCLRFusedFn.apply(eng, b, mode, m.arena_ranges(), *m.trainable_arenas())
        self.log("train_loss", loss, on_step=True, on_epoch=True, prog_bar=True)
        return loss

    def reference_training_step(self, batch, batch_idx, mode=None):
        z1, z2 = self.model(batch, mode)
        loss = self.nt_xent_loss(torch.cat([z1, z2], dim=0))
        self.log("train_loss", loss, on_step=True, on_epoch=True, prog_bar=True)
        return loss

    def configure_optimizers(self):
        opt = FlatAdam(self.model.trainable_arenas(), lr=self.learning_rate)
        return {"optimizer": opt, "lr_scheduler": {"scheduler": _cosine(opt, self.num_epochs),
                                                   "monitor": "train_loss"}}

    def state_dict(self, *args, destination=None, prefix="", keep_vars=False):
        return self.model.state_dict(destination=destination, prefix=prefix + "model.",
                                     keep_vars=keep_vars)
