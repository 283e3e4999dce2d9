"""Reference-shaped model API over the HIP training engine.

Class names, constructor arguments, forward() signatures/returns and state-dict keys follow
the reference (paths relative to its AVMNIST_Experiments/):

  CentralMultiModalEncoder          models/dino.py:454-468   (``--model multi_central``)
  ProjectionHead                    models/dino.py:1240-1254
  MultiModalDINO                    models/dino.py:588-727
  MultiModalDINOWithMSE             models/dino.py:1156-1171
  MultiModalDINOWithINFONCE         models/dino.py:1053-1068
  MultiModalDINOSemiSupervised      models/dino.py:964-980
  MultiModalDINO*Lightning          models/dino.py:730-962, 982-1051, 1070-1154, 1173-1238

Encoder classes are architecture descriptors (the compute is the engine's fused kernels);
the models own a flat parameter arena (params.ParamStore) whose tensors are exposed under the
reference's state-dict keys.  The *Lightning wrappers keep the reference's training_step /
dino_loss / mse_loss / infoNCE_loss / supervised_loss / configure_optimizers surface; the step
itself runs on the device with no host synchronisation (see engine.py).
"""
import math

import torch

from . import ops
from .engine import Hyper, MultiCentralEngine, SimCLREngine, UniModalEngine, adam_step, ema_step
from .params import ParamStore
from .spec import HEAD_NAMES, multimodal_dino_sd, simclr_sd, unimodal_dino_sd

_DT = {"bf16": torch.bfloat16, "16-mixed": torch.bfloat16, "bf16-mixed": torch.bfloat16,
       "32": torch.float32, "fp32": torch.float32, "f32": torch.float32}


# ============================================================================ encoders
class BaseMultiModalEncoder:
    """models/dino.py:203-211 -- descriptor base."""

    arch = None

    def __init__(self, output_dim=256, encoder_output_dim=512, fusion_dropout=0.3):
        self.output_dim = output_dim
        self.encoder_output_dim = encoder_output_dim
        self.fusion_dropout = fusion_dropout


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


# ============================================================================ DINO models
def _device(device):
    if device is not None:
        return torch.device(device)
    return torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")


class MultiModalDINO:
    """Student/teacher multimodal DINO (models/dino.py:588-727) on the HIP engine."""

    mode = "default"

    def __init__(self, encoder_class=CentralMultiModalEncoder, encoder_kwargs=None, output_dim=256,
                 encoder_output_dim=512, projection_dim=128, momentum=0.996, center_momentum=0.9,
                 dropout=0.3, device=None, precision="bf16", seed=0):
        encoder_kwargs = dict(encoder_kwargs or {})
        encoder_kwargs["output_dim"] = output_dim
        encoder_kwargs["encoder_output_dim"] = encoder_output_dim
        enc = encoder_class(**encoder_kwargs)
        if getattr(enc, "arch", None) != "multi_central":
            raise NotImplementedError(
                f"{encoder_class.__name__}: only CentralMultiModalEncoder (multi_central) runs on the "
                f"MI355X engine in this release (BASELINE hot path)")
        self.student_spec = enc
        self.projection_dim, self.output_dim = projection_dim, output_dim
        self.encoder_output_dim = encoder_output_dim
        self.momentum, self.center_momentum, self.dropout = momentum, center_momentum, dropout
        self.device = _device(device)
        self.store = ParamStore(multimodal_dino_sd(self.mode, encoder_output_dim, output_dim,
                                                   projection_dim), self.device, seed=seed)
        self.hp = Hyper(momentum=momentum, center_momentum=center_momentum, dropout=dropout,
                        fusion_dropout=enc.fusion_dropout)
        self.engine = None
        if self.device.type == "cuda":
            self.engine = MultiCentralEngine(self.store, self.mode, encoder_output_dim, output_dim,
                                             projection_dim, self.hp, act_dtype=_DT[precision], seed=seed)
        self.training = True

    # ---------------------------------------------------------------- nn.Module-like surface
    def train(self, mode=True):
        self.training = mode
        return self

    def eval(self):
        return self.train(False)

    def state_dict(self):
        return self.store.state_dict()

    def load_state_dict(self, sd, strict=True):
        self.store.load_state_dict(sd, strict)

    def named_parameters(self):
        for k in self.store.spec:
            if k in self.store.s_offs or k in self.store.t_offs:
                yield k, self.store[k]

    def parameters(self):
        return [v for _, v in self.named_parameters()]

    @property
    def center(self):
        return self.store["center"]

    def _need_engine(self):
        if self.engine is None:
            raise RuntimeError("the HIP engine needs a ROCm device (no CPU fallback)")
        return self.engine

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

    def forward(self, batch):
        """batch = (global_images, global_audios, local_images, local_audios), each
        [B, V, 1, H, W] -> (student_outputs [G+L,B,P], teacher_outputs [G,B,P] centred, None).
        Updates the centre, like the reference."""
        eng = self._need_engine()
        eng.forward({k: v.to(self.device) for k, v in self._views_dict(batch).items()}, training=False)
        s, t = eng.outputs()
        eng.update_center()
        return s.clone(), t.clone(), None

    __call__ = forward


class _WithHeads(MultiModalDINO):
    def forward(self, batch):
        """batch = (image, audio, views) -> (image_out, audio_out, student_out, teacher_out)."""
        image, audio, views = batch
        eng = self._need_engine()
        b = self._views_dict(views)
        b.update(image=image, audio=audio)
        if self.mode == "semi_supervised":
            b["label"] = torch.zeros(image.shape[0], dtype=torch.long)
        eng.forward({k: v.to(self.device) for k, v in b.items()}, training=False)
        s, t = eng.outputs()
        eng.update_center()
        zi, za = eng.last_head_outputs()
        return zi.clone(), za.clone(), s.clone(), t.clone()

    __call__ = forward


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


# ============================================================================ Lightning-shaped
class FlatAdam:
    """torch.optim.Adam(lr, weight_decay) semantics (L2 added to the gradient) over the flat
    gradient arena -- one kernel for all live parameters (configure_optimizers, dino.py:953-962)."""

    def __init__(self, store, hp):
        self.store, self.hp = store, hp
        self.param_groups = [{"lr": hp.lr, "initial_lr": hp.lr, "weight_decay": hp.wd}]

    def zero_grad(self, set_to_none=False):
        self.store.grad.zero_()

    def step(self):
        self.hp.lr = self.param_groups[0]["lr"]
        adam_step(self.store, self.hp)


class CosineAnnealingLR:
    """torch.optim.lr_scheduler.CosineAnnealingLR(T_max), stepped once per epoch."""

    def __init__(self, optimizer, T_max, eta_min=0.0):
        self.opt, self.T_max, self.eta_min = optimizer, T_max, eta_min
        self.base = optimizer.param_groups[0]["initial_lr"]
        self.last_epoch = 0

    def step(self):
        self.last_epoch += 1
        t = self.last_epoch
        self.opt.param_groups[0]["lr"] = self.eta_min + (self.base - self.eta_min) * (
            1 + math.cos(math.pi * t / self.T_max)) / 2

    def get_last_lr(self):
        return [self.opt.param_groups[0]["lr"]]


class MultiModalDINOLightning:
    """Training wrapper (models/dino.py:730-962).  training_step runs forward + losses + EMA on
    the device; backward_and_step() finishes the step (gradients + all-reduce + Adam), which is
    what Lightning's automatic optimisation does after training_step."""

    model_class = MultiModalDINO

    def __init__(self, data_dir="data/avmnist", data_augmentation="burst_noise", dino_model=None,
                 encoder_class=CentralMultiModalEncoder, encoder_kwargs=None, projection_dim=256,
                 output_dim=256, encoder_output_dim=512, momentum=0.996, center_momentum=0.9,
                 student_temperature=0.1, teacher_temperature=0.04, learning_rate=0.0001,
                 use_mixed_precision=True, num_epochs=100, weight_decay=1e-6, dropout=0.3,
                 alpha=1, device=None, precision=None, seed=0):
        self.hparams = dict(data_dir=data_dir, data_augmentation=data_augmentation,
                            encoder_class=encoder_class.__name__, encoder_kwargs=encoder_kwargs,
                            projection_dim=projection_dim, output_dim=output_dim,
                            encoder_output_dim=encoder_output_dim, momentum=momentum,
                            center_momentum=center_momentum, student_temperature=student_temperature,
                            teacher_temperature=teacher_temperature, learning_rate=learning_rate,
                            use_mixed_precision=use_mixed_precision, num_epochs=num_epochs,
                            weight_decay=weight_decay, dropout=dropout, alpha=alpha)
        self.encoder_class, self.encoder_kwargs = encoder_class, encoder_kwargs
        self.learning_rate, self.num_epochs = learning_rate, num_epochs
        self.student_temperature, self.teacher_temperature = student_temperature, teacher_temperature
        self.weight_decay, self.alpha = weight_decay, alpha
        self.precision = precision or ("bf16" if use_mixed_precision else "32")
        if dino_model is None:
            dino_model = self.model_class(encoder_class=encoder_class, encoder_kwargs=encoder_kwargs,
                                          output_dim=output_dim, encoder_output_dim=encoder_output_dim,
                                          projection_dim=projection_dim, momentum=momentum,
                                          center_momentum=center_momentum, dropout=dropout,
                                          device=device, precision=self.precision, seed=seed)
        self.model = dino_model
        hp = self.model.hp
        hp.tau_s, hp.tau_t = student_temperature, teacher_temperature
        hp.lr, hp.wd, hp.alpha = learning_rate, weight_decay, float(alpha)
        self.logged = {}
        self._optim = None

    # ---------------------------------------------------------------- losses (reference API)
    def dino_loss(self, student_outputs, teacher_outputs, alignment_loss=None):
        """dino.py:822-854 -- fused HIP kernel; differentiable w.r.t. student_outputs."""
        return _DinoLossFn.apply(student_outputs, teacher_outputs, self.student_temperature,
                                 self.teacher_temperature, False)

    def mse_loss(self, image_outputs, audio_outputs):
        """dino.py:1193-1211."""
        return _MseLossFn.apply(image_outputs, audio_outputs)

    # ---------------------------------------------------------------- step
    def _batch_dict(self, batch):
        if self.model.mode == "default":
            return self.model._views_dict(batch)
        image, audio, labels, views = batch
        d = self.model._views_dict(views)
        d.update(image=image, audio=audio, label=labels)
        return d

    def log(self, name, value, **kw):
        self.logged[name] = value

    def training_step(self, batch, batch_idx):
        """Forward + losses (+ centre update) + teacher EMA (before backward, as dino.py:871).
        Returns the loss as a device tensor."""
        eng = self.model._need_engine()
        b = {k: v.to(self.model.device, non_blocking=True) for k, v in self._batch_dict(batch).items()}
        loss = eng.forward(b, training=True)
        eng.update_center()
        self.model.update_teacher()
        self.log("train_loss", loss)
        return loss

    def backward_and_step(self, optimizer=None):
        eng = self.model._need_engine()
        eng.backward()
        if eng.grad_hook is not None:
            eng.grad_hook(self.model.store.grad)
        (optimizer or self.configure_optimizers()["optimizer"]).step()
        eng.step_idx += 1

    def configure_optimizers(self):
        """Adam(lr, weight_decay) + CosineAnnealingLR(T_max=num_epochs) (dino.py:953-962)."""
        if self._optim is None:
            opt = FlatAdam(self.model.store, self.model.hp)
            self._optim = {"optimizer": opt,
                           "lr_scheduler": {"scheduler": CosineAnnealingLR(opt, T_max=self.num_epochs)}}
        return self._optim

    def forward(self, batch):
        return self.model(batch)

    def _probe_kind(self):
        enc = self.model.student_spec
        return getattr(enc, "kind", None) or enc.arch

    def on_train_epoch_end(self, traindata=None, validdata=None):
        """Linear probe (dino.py:878-951 / 1670-1735) over iterables of (images, audios,
        labels) device batches (the reference's AVMNIST loaders, batch 128); logs val_loss and
        mlp_acc.  No data: nothing to do (the on-disk loader is outside the hot path)."""
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
        self.log("mlp_acc", out["mlp_acc"])
        return out

    def state_dict(self):
        return {"model." + k: v for k, v in self.model.state_dict().items()}

    def load_state_dict(self, sd, strict=True):
        self.model.load_state_dict({k[len("model."):]: v for k, v in sd.items() if k.startswith("model.")},
                                   strict)

    def parameters(self):
        return self.model.parameters()


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

MODEL_MAP = {"multi_central": CentralMultiModalEncoder}


# ============================================================================ unimodal DINO
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


class UniModalDINO:
    """Student/teacher unimodal DINO (models/dino.py:1257-1398) on the HIP engine."""

    def __init__(self, encoder_class=ImageEncoder, encoder_kwargs=None, output_dim=256,
                 projection_dim=128, momentum=0.996, center_momentum=0.9, dropout=0.3,
                 device=None, precision="bf16", seed=0, cosine_loss_alpha=0.0):
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
        self.store = ParamStore(unimodal_dino_sd(enc.kind, output_dim, projection_dim), self.device,
                                seed=seed)
        self.hp = Hyper(momentum=momentum, center_momentum=center_momentum, dropout=dropout)
        self.engine = None
        if self.device.type == "cuda":
            self.engine = UniModalEngine(self.store, enc.kind, output_dim, projection_dim, self.hp,
                                         act_dtype=_DT[precision], cos_alpha=cosine_loss_alpha,
                                         seed=seed)
        self.training = True

    train, eval = MultiModalDINO.train, MultiModalDINO.eval
    state_dict, load_state_dict = MultiModalDINO.state_dict, MultiModalDINO.load_state_dict
    named_parameters, parameters = MultiModalDINO.named_parameters, MultiModalDINO.parameters
    center = MultiModalDINO.center
    _need_engine = MultiModalDINO._need_engine
    update_teacher = MultiModalDINO.update_teacher
    update_center = MultiModalDINO.update_center

    def forward(self, batch):
        """batch = (global_images, global_audios, local_images, local_audios) -> (student_outputs
        [G+L,B,P], teacher_outputs [G,B,P] centred, embeddings [G+L,B,D]); updates the centre."""
        eng = self._need_engine()
        eng.forward({k: v.to(self.device) for k, v in MultiModalDINO._views_dict(batch).items()},
                    training=False)
        s, t, e = eng.outputs()
        eng.update_center()
        return s.clone(), t.clone(), e.clone()

    __call__ = forward


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


class UniModalDINOLightning(MultiModalDINOLightning):
    """models/dino.py:1490-1693: unimodal DINO loss (teacher centred per view) + optional
    cosine-consistency term (cosine_loss_alpha, default 0.3), EMA before backward, Adam(L2)."""

    model_class = UniModalDINO

    def __init__(self, data_dir="data/avmnist", dino_model=None, encoder_class=ImageEncoder,
                 encoder_kwargs=None, projection_dim=128, output_dim=256, momentum=0.996,
                 center_momentum=0.9, student_temperature=0.1, teacher_temperature=0.04,
                 learning_rate=0.0001, use_mixed_precision=True, weight_decay=1e-6,
                 cosine_loss_alpha=0.3, dropout=0.3, num_epochs=10, data_augmentation="burst_noise",
                 use_original_model=True, device=None, precision=None, seed=0):
        self.hparams = dict(data_dir=data_dir, encoder_class=encoder_class.__name__,
                            encoder_kwargs=encoder_kwargs, projection_dim=projection_dim,
                            output_dim=output_dim, momentum=momentum, center_momentum=center_momentum,
                            student_temperature=student_temperature,
                            teacher_temperature=teacher_temperature, learning_rate=learning_rate,
                            use_mixed_precision=use_mixed_precision, weight_decay=weight_decay,
                            cosine_loss_alpha=cosine_loss_alpha, dropout=dropout,
                            num_epochs=num_epochs, data_augmentation=data_augmentation)
        if not use_original_model:
            raise NotImplementedError("UniModalDINOV2 is not on the MI355X hot path")
        self.learning_rate, self.num_epochs = learning_rate, num_epochs
        self.student_temperature, self.teacher_temperature = student_temperature, teacher_temperature
        self.weight_decay, self.cosine_loss_alpha = weight_decay, cosine_loss_alpha
        self.precision = precision or ("bf16" if use_mixed_precision else "32")
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
        self.logged = {}
        self._optim = None

    def dino_loss(self, student_outputs, teacher_outputs):
        """dino.py:1596-1635 (teacher additionally centred by its per-view batch mean)."""
        return _DinoLossFn.apply(student_outputs, teacher_outputs, self.student_temperature,
                                 self.teacher_temperature, True)

    def _cosine_consistency_loss(self, embeddings):
        """dino.py:1575-1594."""
        return _UniCosineLossFn.apply(embeddings)

    def _batch_dict(self, batch):
        return MultiModalDINO._views_dict(batch)

    def training_step(self, batch, batch_idx):
        eng = self.model._need_engine()
        b = {k: v.to(self.model.device, non_blocking=True) for k, v in self._batch_dict(batch).items()}
        loss = eng.forward(b, training=True)
        eng.update_center()
        self.model.update_teacher()
        self.log("train_loss", loss)
        return loss


UNIMODAL_MODEL_MAP = {"image_simple": ImageEncoder, "spectrogram_simple": SpectrogramEncoder,
                      "spectrogram_central": SpectrogramEncoderCentral}



# ============================================================================ multimodal SimCLR
class MultiModalSimCLRModel:
    """other_ssl/multimodal_simclr/multimodal_simclr.py:12-47 on the HIP engine: ImageEncoder +
    SpectrogramEncoder towers with ProjectionHead(output_dim, projection_dim) each."""

    def __init__(self, output_dim=256, projection_dim=256, device=None, precision="bf16", seed=0,
                 negatives="global", mode_seed=1234):
        self.output_dim, self.projection_dim = output_dim, projection_dim
        self.device = _device(device)
        self.store = ParamStore(simclr_sd(output_dim, projection_dim), self.device, seed=seed,
                                has_teacher=False, groups=SimCLREngine.GROUPS)
        self.hp = Hyper(weight_decay=0.0)
        self.engine = None
        if self.device.type == "cuda":
            self.engine = SimCLREngine(self.store, output_dim, projection_dim, self.hp,
                                       act_dtype=_DT[precision], negatives=negatives, seed=mode_seed)
        self.training = True

    train, eval = MultiModalDINO.train, MultiModalDINO.eval
    state_dict, load_state_dict = MultiModalDINO.state_dict, MultiModalDINO.load_state_dict
    named_parameters, parameters = MultiModalDINO.named_parameters, MultiModalDINO.parameters
    _need_engine = MultiModalDINO._need_engine

    @staticmethod
    def _batch_dict(batch):
        img1, spec1, img2, spec2 = batch
        return {"img1": img1, "spec1": spec1, "img2": img2, "spec2": spec2}

    def forward(self, batch, mode=None):
        """batch = (aug_img1, aug_spec1, aug_img2, aug_spec2) -> (z1, z2) [B, projection_dim]."""
        eng = self._need_engine()
        eng.forward({k: v.to(self.device).float() for k, v in self._batch_dict(batch).items()}, mode)
        z1, z2 = eng.outputs()
        return z1.clone(), z2.clone()

    __call__ = forward


class _NtXentFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, reps, temperature):
        from . import contrastive
        from .engine import Workspace
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


class MultiModalSimCLRLightning:
    """multimodal_simclr.py:49-112: training_step = forward (random modality pair) + NT-Xent;
    backward_and_step() = backward + Adam(lr) on the used towers (Lightning's automatic
    optimisation); CosineAnnealingLR(T_max=num_epochs) per epoch."""

    def __init__(self, projection_dim=256, output_dim=256, learning_rate=0.0001, num_epochs=100,
                 use_mixed_precision=True, device=None, precision=None, seed=0, negatives="global",
                 mode_seed=1234):
        self.hparams = dict(projection_dim=projection_dim, output_dim=output_dim,
                            learning_rate=learning_rate, num_epochs=num_epochs,
                            use_mixed_precision=use_mixed_precision)
        self.output_dim, self.projection_dim = output_dim, projection_dim
        self.learning_rate, self.num_epochs = learning_rate, num_epochs
        self.precision = precision or ("bf16" if use_mixed_precision else "32")
        self.model = MultiModalSimCLRModel(output_dim, projection_dim, device, self.precision, seed,
                                           negatives, mode_seed)
        self.model.hp.lr = learning_rate
        self.logged = {}
        self._optim = None

    def forward(self, batch):
        return self.model(batch)

    def nt_xent_loss(self, reps, temperature=0.07):
        """multimodal_simclr.py:74-89 (fused HIP kernels; differentiable w.r.t. reps)."""
        return _NtXentFn.apply(reps, temperature)

    def log(self, name, value, **kw):
        self.logged[name] = value

    def training_step(self, batch, batch_idx):
        eng = self.model._need_engine()
        b = {k: v.to(self.model.device, non_blocking=True).float()
             for k, v in self.model._batch_dict(batch).items()}
        loss = eng.forward(b)
        self.log("train_loss", loss)
        return loss

    def backward_and_step(self, optimizer=None):
        eng = self.model._need_engine()
        eng.backward()
        if eng.grad_hook is not None:
            eng.grad_hook(self.model.store.grad)
        opt = optimizer or self.configure_optimizers()["optimizer"]
        self.model.hp.lr = opt.param_groups[0]["lr"]
        eng.adam()

    def configure_optimizers(self):
        if self._optim is None:
            opt = FlatAdam(self.model.store, self.model.hp)
            self._optim = {"optimizer": opt,
                           "lr_scheduler": {"scheduler": CosineAnnealingLR(opt, T_max=self.num_epochs),
                                            "monitor": "train_loss"}}
        return self._optim

    def state_dict(self):
        return {"model." + k: v for k, v in self.model.state_dict().items()}

    def load_state_dict(self, sd, strict=True):
        self.model.load_state_dict({k[len("model."):]: v for k, v in sd.items() if k.startswith("model.")},
                                   strict)

    def parameters(self):
        return self.model.parameters()
