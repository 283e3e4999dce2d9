"""Flat parameter arenas in HBM.

All trainable tensors of a model live in one contiguous fp32 arena so that the teacher EMA,
Adam and the DDP gradient all-reduce are each ONE launch / ONE collective over a contiguous
range, instead of the reference's per-parameter Python loops (update_teacher dino.py:635-646,
torch.optim.Adam, DDP buckets).

Student arena layout   [ heads | ema-live | ema-dead ]
Teacher arena layout            [ ema-live | ema-dead ]     (same order as the student's)
Gradient / Adam state  [ heads | ema-live ]

  * ema-live / ema-dead: parameters of ``student.*`` and ``student_projection.*`` (EMA'd
    into ``teacher.*`` / ``teacher_projection.*``).  "dead" = the CentralNet fc1/fc2
    layers, built but never executed (unimodal.py:124-125, 182-183): they get no gradient
    (Adam skips them, as torch.optim.Adam skips grad=None) but are EMA'd like every other
    parameter, exactly as the reference does.
  * heads: student-side parameters with no teacher copy (MSE / InfoNCE projection heads,
    semi-supervised classifiers; or every parameter of a teacher-less model such as SimCLR).

Every parameter is exposed as a view into its arena under its reference state-dict key, so
``state_dict()`` / ``load_state_dict()`` interoperate with reference checkpoints.
"""
import math
from collections import OrderedDict

import torch

ALIGN = 16  # floats (64 B) per parameter slot


def _is_param(kind):
    return kind in ("w", "b", "bn_w", "bn_b")


def _dead(key):
    return ".fc1." in key or ".fc2." in key


def _teacher_of(key):
    if key.startswith("student_projection."):
        return "teacher_projection." + key[len("student_projection."):]
    if key.startswith("student."):
        return "teacher." + key[len("student."):]
    return None


class ParamStore:
    def __init__(self, sd_spec, device, seed=0, has_teacher=True, groups=None):
        """groups: optional list of key prefixes; the head parameters are laid out group by
        group in that order (each group one contiguous range, see group_range), e.g. SimCLR's
        image and audio towers, which Adam steps independently."""
        self.spec = OrderedDict(sd_spec)
        self.device = torch.device(device)
        keys = [k for k, (_s, kind) in self.spec.items() if _is_param(kind)]
        tkeys = {_teacher_of(k) for k in keys if has_teacher and _teacher_of(k) in self.spec}
        ema = [k for k in keys if has_teacher and _teacher_of(k) in self.spec]
        heads = [k for k in keys if k not in ema and k not in tkeys]
        ema_live = [k for k in ema if not _dead(k)]
        ema_dead = [k for k in ema if _dead(k)]

        def layout(order):
            offs, o = OrderedDict(), 0
            for k in order:
                n = int(math.prod(self.spec[k][0]))
                offs[k] = (o, n)
                o += -(-n // ALIGN) * ALIGN
            return offs, o

        self.groups = list(groups or [])
        if self.groups:
            def gidx(k):
                for i, g in enumerate(self.groups):
                    if k.startswith(g):
                        return i
                return len(self.groups)
            heads = sorted(heads, key=gidx)   # stable: spec order inside a group
        s_order = heads + ema_live + ema_dead
        self.s_offs, s_total = layout(s_order)
        self.n_heads = sum(-(-self.s_offs[k][1] // ALIGN) * ALIGN for k in heads)
        self.n_live = self.n_heads + sum(-(-self.s_offs[k][1] // ALIGN) * ALIGN for k in ema_live)
        self.n_ema = s_total - self.n_heads  # ema-live + ema-dead
        self.student = torch.zeros(s_total, dtype=torch.float32, device=self.device)
        self.grad = torch.zeros(self.n_live, dtype=torch.float32, device=self.device)
        self.adam_m = torch.zeros_like(self.grad)
        self.adam_v = torch.zeros_like(self.grad)
        self.adam_step = 0
        if has_teacher and ema:
            self.t_offs = OrderedDict((_teacher_of(k), (self.s_offs[k][0] - self.n_heads, self.s_offs[k][1]))
                                      for k in ema_live + ema_dead)
            self.teacher = torch.zeros(self.n_ema, dtype=torch.float32, device=self.device)
        else:
            self.t_offs = OrderedDict()
            self.teacher = None
        self.live_keys = heads + ema_live
        # float buffers (BN running stats, DINO centre) share one arena so DDP's per-forward
        # buffer broadcast (rank 0 -> all) is a single collective
        fkeys = [k for k, (_s, kind) in self.spec.items() if kind in ("rm", "rv", "center")]
        self.buf_offs, nbuf = layout(fkeys)
        self.buf_arena = torch.zeros(max(nbuf, ALIGN), dtype=torch.float32, device=self.device)
        self.buffers = OrderedDict()
        # num_batches_tracked counters: one int64 arena, bumped once per forward for all BN
        # layers (bump_nbt / flush_nbt) instead of one add launch per layer
        nkeys = [k for k, (_s, kind) in self.spec.items() if kind == "nbt"]
        self.nbt_index = {k: i for i, k in enumerate(nkeys)}
        self.nbt_arena = torch.zeros(max(len(nkeys), 1), dtype=torch.int64, device=self.device)
        self._nbt_pending, self._nbt_cache = {}, {}
        for k, (shape, kind) in self.spec.items():
            if kind in ("rm", "rv", "center"):
                self.buffers[k] = self._view(self.buf_arena, self.buf_offs, k)
            elif kind == "nbt":
                i = self.nbt_index[k]
                self.buffers[k] = self.nbt_arena[i:i + 1].view(shape)
        self.reset_parameters(seed)

    def group_range(self, i):
        """(offset, length) of head group i in the student / grad / Adam arenas."""
        keys = [k for k in self.live_keys if k.startswith(self.groups[i])]
        lo = min(self.s_offs[k][0] for k in keys)
        hi = max(self.s_offs[k][0] + -(-self.s_offs[k][1] // ALIGN) * ALIGN for k in keys)
        return lo, hi - lo

    # ------------------------------------------------------------------ views
    def _view(self, arena, offs, key):
        o, n = offs[key]
        return arena[o:o + n].view(self.spec[key][0])

    def __getitem__(self, key):
        """Parameter or buffer tensor (a view into the arena for parameters)."""
        if key in self.s_offs:
            return self._view(self.student, self.s_offs, key)
        if key in self.t_offs:
            return self._view(self.teacher, self.t_offs, key)
        return self.buffers[key]

    def bump_nbt(self, key, inc):
        """Record num_batches_tracked += inc for one BN layer (applied by flush_nbt)."""
        self._nbt_pending[key] = self._nbt_pending.get(key, 0) + inc

    def flush_nbt(self):
        """Apply the recorded counter increments: one avd_counters_add launch on the current
        stream (the index / value tensors are cached per increment pattern, so no host copy per
        step)."""
        if not self._nbt_pending:
            return
        sig = tuple(sorted(self._nbt_pending.items()))
        self._nbt_pending = {}
        c = self._nbt_cache.get(sig)
        if c is None:
            idx = torch.tensor([self.nbt_index[k] for k, _ in sig], dtype=torch.int64, device=self.device)
            val = torch.tensor([v for _, v in sig], dtype=torch.int64, device=self.device)
            c = self._nbt_cache[sig] = (idx, val)
        if self.nbt_arena.device.type != "cuda":     # host-side store (checkpoint / state-dict work)
            self.nbt_arena.index_add_(0, c[0], c[1])
            return
        from . import ops
        ops.counters_add(self.nbt_arena, c[0], c[1])

    def grad_of(self, key):
        o, n = self.s_offs[key]
        return self.grad[o:o + n].view(self.spec[key][0])

    # ------------------------------------------------------------------ init / io
    def reset_parameters(self, seed=0):
        """PyTorch's default init for the reference layers (Conv2d/Linear kaiming-uniform(a=sqrt 5)
        => U(+-1/sqrt(fan_in)) for weight and bias; BN weight 1, bias 0); the teacher starts as an
        exact copy of the student (dino.py:615-629)."""
        g = torch.Generator().manual_seed(seed)
        fan = {}
        for k, (shape, kind) in self.spec.items():
            if kind == "w":
                fan[k[:-len(".weight")]] = int(math.prod(shape[1:]))
        for k in self.s_offs:
            shape, kind = self.spec[k]
            if kind in ("w", "b"):
                b = 1.0 / math.sqrt(fan[k.rsplit(".", 1)[0]])
                v = (torch.rand(shape, generator=g, dtype=torch.float64) * 2 - 1) * b
            elif kind == "bn_w":
                v = torch.ones(shape, dtype=torch.float64)
            else:
                v = torch.zeros(shape, dtype=torch.float64)
            self[k].copy_(v.to(torch.float32))
        if self.teacher is not None:
            self.teacher.copy_(self.student[self.n_heads:])
        for k, b in self.buffers.items():
            kind = self.spec[k][1]
            b.fill_(1.0 if kind == "rv" else 0)
        self.adam_m.zero_()
        self.adam_v.zero_()
        self.adam_step = 0

    def state_dict(self):
        self.flush_nbt()
        return OrderedDict((k, self[k]) for k in self.spec)

    def load_state_dict(self, sd, strict=True):
        missing = [k for k in self.spec if k not in sd]
        unexpected = [k for k in sd if k not in self.spec]
        if strict and (missing or unexpected):
            raise KeyError(f"state_dict mismatch: missing={missing[:5]} unexpected={unexpected[:5]}")
        with torch.no_grad():
            for k, v in sd.items():
                if k in self.spec:
                    t = self[k]
                    v = torch.as_tensor(v)
                    if tuple(v.shape) != tuple(t.shape):
                        raise ValueError(f"{k}: shape {tuple(v.shape)} != {tuple(t.shape)}")
                    t.copy_(v.to(device=t.device, dtype=t.dtype))
