"""Epoch-end linear probe (BASELINE config 5's "linear-probe eval"):
``on_train_epoch_end`` of the DINO Lightning modules (models/dino.py:878-951 multimodal,
1670-1735 unimodal) with ``DownstreamClassifier`` (1764-1814), on libavdino kernels.

Reference semantics kept:
  * the encoder is a frozen DEEP COPY of the student (here: a second ParamStore filled from the
    student arena and buffer arena) -- nothing the probe does touches the trained model;
  * ``model_downstream.train()`` puts the copy in TRAIN mode for the probe epoch: batch-stat
    BatchNorm whose running statistics update the copy, and the CentralNet fusion dropout
    (0.3) active; the copy gets no gradient (torch.no_grad);
  * classifier Linear(output_dim, 128) - ReLU - Linear(128, 10), default init, trained with
    AdamW(lr = learning_rate, weight_decay 0.01) one step per batch; ``val_loss`` = the mean
    training loss of the epoch;
  * ``evaluate()`` puts the copy in EVAL mode (running statistics, no dropout): mean CE over
    the batches and ``mlp_acc`` = 100 * correct / total with torch.max's first-maximum argmax.
The reference runs the probe under fp16 autocast + GradScaler on CUDA; here the classifier is
fp32 (the GradScaler only matters on overflow) and the encoder copy runs in the engine's
activation dtype.  Per-batch losses stay on the device (no host sync inside the epoch).
"""
import torch

from . import ops
from .capture import GraphedStep
from .engine import F32, ConvBranch, StepState, UniEncoder, Workspace
from .params import ParamStore
from .spec import MULTI_ENCODERS, UNI_ALIASES, UNI_ENCODERS

from collections import OrderedDict


def classifier_sd(D, hidden=128, num_classes=10):
    sd = OrderedDict()
    sd["classifier.0.weight"] = ((hidden, D), "w")
    sd["classifier.0.bias"] = ((hidden,), "b")
    sd["classifier.2.weight"] = ((num_classes, hidden), "w")
    sd["classifier.2.bias"] = ((num_classes,), "b")
    return sd


class _MultiEncoder:
    """The multimodal student (SimpleMultiModalEncoder.forward, dino.py:229-234; the
    CentralMultiModalEncoder of 454-468 or the 3x3 encoders of 214-227) without gradients:
    both conv branches, their Linears into the cat buffer, fusion."""

    def __init__(self, arch, E, D, act, gm, fusion_dropout):
        self.E, self.D, self.gm, self.p = E, D, gm, fusion_dropout
        istack, ilin, astack, alin, _sd = MULTI_ENCODERS[arch]
        self.img = ConvBranch(istack("student"), act)
        self.aud = ConvBranch(astack("student"), act)
        self.ilin, self.alin = "student." + ilin, "student." + alin

    def __call__(self, ws, st, x_img, x_aud, N, train, seed, seed_off=None):
        E = self.E
        if train:
            fi, _ = self.img.forward(ws, st, "pi", x_img, N, 1, True, False)
            fa, _ = self.aud.forward(ws, st, "pa", x_aud, N, 1, True, False)
            st.flush_nbt()
        else:
            fi = self.img.forward_eval(ws, st, "pi", x_img, N)
            fa = self.aud.forward_eval(ws, st, "pa", x_aud, N)
        cat = ws.get("p.cat", N * 2 * E)
        ops.linear_fwd(fi, st[self.ilin + ".weight"], st[self.ilin + ".bias"],
                       cat, N, out_ld=2 * E, out_off=0, mode=self.gm)
        ops.linear_fwd(fa, st[self.alin + ".weight"], st[self.alin + ".bias"],
                       cat, N, out_ld=2 * E, out_off=E, mode=self.gm)
        h = ws.get("p.fh", N * E)
        ops.linear_fwd(cat, st["student.fusion.0.weight"], st["student.fusion.0.bias"], h, N,
                       x_ld=2 * E, mode=self.gm)
        r = ws.get("p.fr", N * E)
        ops.act_fwd(h, r, 0, None, None, N, 1, E, self.p if train else 0.0, seed, seed_off)
        out = ws.get("p.feat", N * self.D)
        ops.linear_fwd(r, st["student.fusion.3.weight"], st["student.fusion.3.bias"], out, N,
                       mode=self.gm)
        return out


class _UniEncoder:
    def __init__(self, kind, act, gm):
        self.enc = UniEncoder(kind, "student", act, gm)

    def __call__(self, ws, st, x, N, train):
        if train:
            out, _ = self.enc.forward(ws, st, "pu", x, N, 1, False)
            st.flush_nbt()
            return out
        return self.enc.forward_eval(ws, st, "pu", x, N)


class LinearProbe:
    """One probe epoch over a trained DINO model's student.

    source: the trained model's ParamStore (MultiModalDINO*.store / UniModalDINO.store);
    kind: a MODEL_MAP key ("multi_central", "multi_simple") or an UNIMODAL_MODEL_MAP key;
    E/D: encoder_output_dim / output_dim.
    """

    def __init__(self, source, kind, D, E=None, lr=1e-4, weight_decay=0.01, act_dtype=F32,
                 fusion_dropout=0.3, seed=0, classifier_state=None, use_graph=True):
        dev = source.device
        self.store = ParamStore(source.spec, dev, has_teacher=source.teacher is not None)
        self.store.student.copy_(source.student)          # copy.deepcopy(model.student)
        self.store.buf_arena.copy_(source.buf_arena)
        source.flush_nbt()
        self.store.nbt_arena.copy_(source.nbt_arena)
        self.kind = UNI_ALIASES.get(kind, kind)
        self.D = D
        self.gm = ops.GEMM_BF16_MFMA if act_dtype == torch.bfloat16 else ops.GEMM_F32_MFMA
        self.act = act_dtype
        self.ws = Workspace(dev)
        self.multimodal = self.kind in MULTI_ENCODERS
        if self.multimodal:
            self.enc = _MultiEncoder(self.kind, E, D, act_dtype, self.gm, fusion_dropout)
        else:
            self.enc = _UniEncoder(self.kind, act_dtype, self.gm)
            self.modality = UNI_ENCODERS[self.kind][0]
        self.cls = ParamStore(classifier_sd(D), dev, seed=seed, has_teacher=False)
        if classifier_state is not None:
            self.cls.load_state_dict(classifier_state)
        self.lr, self.wd = lr, weight_decay
        self.t = 0
        self.seed = seed
        # step count, AdamW bias corrections and the dropout counter offset on the device, so a
        # training batch is one replayable hipGraph (a 128-sample batch is launch-bound: ~50
        # launches, 0.65 ms issued eagerly); the ragged last batch of an epoch runs eagerly
        self.sstate = StepState(dev, lr, (0.9, 0.999)) if dev.type == "cuda" else None
        self.use_graph = use_graph and dev.type == "cuda"
        self.graph = (GraphedStep(warmup=2, deps=lambda: (ops.alloc_epoch(), self.ws.epoch))
                      if self.use_graph else None)

    def _features(self, images, audios, train, seed_off=None):
        ws, N = self.ws, (images if images is not None else audios).shape[0]
        if self.multimodal:
            xi = ws.get("p.in.img", N * 784, self.act)
            xa = ws.get("p.in.aud", N * 12544, self.act)
            ops.stage_views(images.contiguous(), 1, None, 0, None, N, 784, xi)
            ops.stage_views(audios.contiguous(), 1, None, 0, None, N, 12544, xa)
            if seed_off is not None:      # device counter: seed + t * StepState.SEED_STRIDE
                return self.enc(ws, self.store, xi, xa, N, train, self.seed * 7919, seed_off)
            return self.enc(ws, self.store, xi, xa, N, train, self.seed * 7919 + self.t)
        src, HW = (images, 784) if self.modality == "image" else (audios, 12544)
        x = ws.get("p.in.x", N * HW, self.act)
        ops.stage_views(src.contiguous(), 1, None, 0, None, N, HW, x)
        return self.enc(ws, self.store, x, N, train)

    def _logits(self, feat, N):
        ws, c = self.ws, self.cls
        h = ws.get("p.h", N * 128)
        ops.linear_fwd(feat, c["classifier.0.weight"], c["classifier.0.bias"], h, N)
        r = ws.get("p.r", N * 128)
        ops.act_fwd(h, r, 0, None, None, N, 1, 128, 0.0, 0)
        logits = ws.get("p.logits", N * 10)
        ops.linear_fwd(r, c["classifier.2.weight"], c["classifier.2.bias"], logits, N)
        return h, r, logits

    def train_batch(self, images, audios, labels, loss_out):
        """One classifier step; loss_out: 1-element device slot for this batch's mean CE.
        With ``use_graph`` the batch is copied into fixed buffers and the step replayed as a
        hipGraph per batch size (after two eager batches of that size)."""
        if self.sstate is not None:
            self.sstate.set_lr(self.lr)   # (a host-side schedule change; eager)
        # host step count (AdamW bias corrections of the host-state path, snapshot()): counted
        # here, outside the captured body, so graph-replayed batches advance it too
        self.t += 1
        if not self.use_graph:
            self._train_step(images, audios, labels, loss_out)
            return
        ws = self.ws

        def fixed(name, t):
            if t is None:
                return None
            b = ws.get(name, t.numel(), t.dtype).view_as(t)
            b.copy_(t)
            return b
        bi, ba, bl = fixed("p.src.img", images), fixed("p.src.aud", audios), fixed("p.src.lab", labels)
        slot = ws.get("p.loss", 1)
        key = tuple(None if t is None else (tuple(t.shape), t.dtype) for t in (images, audios, labels))
        self.graph.run(key, lambda: self._train_step(bi, ba, bl, slot))
        loss_out.copy_(slot)

    def _train_step(self, images, audios, labels, loss_out):
        ws, c = self.ws, self.cls
        N = (images if images is not None else audios).shape[0]
        dev_state = self.sstate is not None
        if dev_state:
            self.sstate.begin()           # t += 1, bias corrections, dropout offset
        feat = self._features(images, audios, True,
                              self.sstate.seed_off if dev_state and self.multimodal else None)
        h, r, logits = self._logits(feat, N)
        parts, dl = ws.get("p.parts", N), ws.get("p.dl", N * 10)
        ops.softmax_xent(logits, 10, N, 10, labels, 0, False, False, 1.0 / N, parts, dl, 10, False)
        ops.sum_to(parts, N, 1.0 / N, loss_out)
        dr = ws.get("p.dr", N * 128)
        ops.linear_bwd(dl, r, c["classifier.2.weight"], c.grad_of("classifier.2.weight"),
                       c.grad_of("classifier.2.bias"), dr, N)
        dh = ws.get("p.dh", N * 128)
        ops.act_bwd(h, dr, dh, 0, None, None, N, 1, 128, 0.0, 0)
        ops.linear_bwd(dh, feat, c["classifier.0.weight"], c.grad_of("classifier.0.weight"),
                       c.grad_of("classifier.0.bias"), None, N)
        b1, b2 = 0.9, 0.999
        if dev_state:
            ops.adam_dev(c.student, c.grad, c.adam_m, c.adam_v, c.n_live, self.sstate.hyp, b1, b2,
                         1e-8, self.wd, decoupled=True)
        else:
            ops.adamw(c.student, c.grad, c.adam_m, c.adam_v, c.n_live, self.lr, b1, b2, 1e-8,
                      self.wd, 1 - b1 ** self.t, 1 - b2 ** self.t)

    def evaluate(self, batches):
        """evaluate() (dino.py:913-947): eval-mode copy; returns (mean loss, accuracy %, logits)."""
        ws = self.ws
        losses, correct, logits_all, n = [], [], [], 0
        for images, audios, labels in batches:
            N = images.shape[0]
            feat = self._features(images, audios, False)
            _, _, logits = self._logits(feat, N)
            parts = ws.get("p.parts", N)
            ops.softmax_xent(logits, 10, N, 10, labels, 0, False, False, 1.0 / N, parts, None, 10,
                             False)
            l1 = torch.empty(1, device=logits.device)
            ops.sum_to(parts, N, 1.0 / N, l1)
            ok = torch.empty(N, device=logits.device)
            ops.argmax_correct(logits, 10, N, 10, labels, ok)
            c1 = torch.empty(1, device=logits.device)
            ops.sum_to(ok, N, 1.0, c1)
            losses.append(l1)
            correct.append(c1)
            logits_all.append(logits.view(N, 10).clone())
            n += N
        loss = torch.cat(losses).mean().item()
        acc = 100.0 * torch.cat(correct).sum().item() / n
        return loss, acc, torch.cat(logits_all)

    def run_epoch(self, train_batches, valid_batches):
        """on_train_epoch_end: returns {"val_loss", "mlp_acc", "eval_loss", "train_losses"}."""
        train_batches = list(train_batches)
        losses = torch.empty(len(train_batches), device=self.store.device)
        for i, (images, audios, labels) in enumerate(train_batches):
            self.train_batch(images, audios, labels, losses[i:i + 1])
        ev_loss, acc, logits = self.evaluate(valid_batches)
        return {"val_loss": losses.mean().item(), "mlp_acc": acc, "eval_loss": ev_loss,
                "train_losses": losses, "logits": logits}
