"""Data-parallel plumbing of the training step: one process per GPU,
``torch.distributed`` with backend ``nccl`` (= RCCL over xGMI) on MI355X, ``gloo`` in the CPU
tests.  Nothing here computes model math; it moves the engine's flat arenas.

* :class:`GradAllReduce` -- the per-step gradient exchange over the flat live-gradient arena
  (2.12 M f32 = 8.5 MB for mse/infonce; the reference's DDP buckets the same parameters, dead
  fc1/fc2 excluded because they have no gradient), then x 1/world (DDP's gradient
  averaging): the ranges the backward finishes first (heads, fusion, projection) go out as
  an early bucket from inside the captured step, the conv branches after it.
* :func:`broadcast_buffers` -- DDP ``broadcast_buffers=True`` semantics of the reference's
  Lightning DDP run: at the start of every forward rank 0's buffers (``center``, BN running
  stats, ``num_batches_tracked``) overwrite the other ranks' copies, so all ranks train from
  rank 0's centre.
* :func:`gather_rows` / :func:`scatter_rows_grad` -- global-negative contrastive losses
  (InfoNCE config 3, NT-Xent config 4): all-gather the local rows into the global batch, and
  route d(global rows) back to the owning rank with a SUM reduce-scatter, so each rank's loss
  gradient reaches every shard it touched (with DDP averaging this equals the single-device
  gradient of the global-batch loss).
"""
import torch
import torch.distributed as dist


def world(group=None):
    return dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1


# Test hook: issue every collective of the data-parallel path even at world 1 (an all-reduce,
# all-gather or reduce-scatter over one rank is the identity), so the RCCL branches -- the
# asynchronous buckets, all_gather_into_tensor, reduce_scatter_tensor -- and the graph-segmented
# step around them execute on a one-GPU box (tests/test_gpu_rccl.py).  Set through forced().
_FORCE = [False]


class forced:
    """``with dist.forced(): ...`` -- the data-parallel path at any initialised world size."""

    def __enter__(self):
        self.prev, _FORCE[0] = _FORCE[0], True
        return self

    def __exit__(self, *exc):
        _FORCE[0] = self.prev


def distributed(group=None):
    """Does the step exchange data with other ranks (world > 1, or forced at world 1)?"""
    if not (dist.is_available() and dist.is_initialized()):
        return False
    return _FORCE[0] or dist.get_world_size(group) > 1


def rank(group=None):
    return dist.get_rank(group) if dist.is_available() and dist.is_initialized() else 0


class GradAllReduce:
    """DDP's gradient averaging over the flat gradient arena, in buckets.

    A step's exchange is ``begin()`` (eager, before the step), any number of
    ``bucket(grad, ranges)`` calls as soon as the step has produced those ranges (an engine
    calls it at a host point inside its captured step, avdino.capture: with RCCL the collective
    runs on the process group's stream while the rest of the backward keeps the compute stream
    busy), then ``finish(grad)`` -- all-reduce whatever no bucket covered (within ``ranges``,
    default the whole arena) and make the caller's stream wait for every collective -- and
    ``scale(grad)`` (x 1/world over the reduced ranges; plain device work, so a captured step
    keeps it and the optimizer in its last graph segment).  ``hook(grad)`` = finish + scale.
    Every rank issues the same buckets in the same order (same ranges, same step structure).
    With no bucket it is one all-reduce over the arena.

    ``overlap``: issue the bucket collectives asynchronously (default: on RCCL only -- gloo's
    CUDA all-reduce stages through host memory on a worker thread, and left in flight under the
    next replayed graph segment it stalled each step ~20x, 167-215 ms vs 9-11 ms per 2-rank
    step); ``overlap=True`` under gloo runs the same pending / wait / scale order (tests)."""

    def __init__(self, group=None, overlap=None):
        self.group = group
        self.overlap = overlap
        self.pending, self.covered, self.reduced = [], [], []

    def world(self):
        return dist.get_world_size(self.group)

    def _async(self):
        return self.overlap if self.overlap is not None else dist.get_backend(self.group) == "nccl"

    def begin(self):
        """Start a step's exchange.  Collectives still pending from an earlier step that never
        reached finish() (an aborted step) are waited for and forgotten, so their ranges cannot
        suppress this step's reduction of the same ranges (ranks would diverge silently)."""
        for w in self.pending:
            w.wait()
        self.pending, self.covered, self.reduced = [], [], []

    def bucket(self, grad, ranges):
        if not distributed(self.group):
            return
        overlap = self._async()
        for lo, hi in ranges:
            if hi > lo:
                if any(lo < chi and clo < hi for clo, chi in self.covered):
                    raise RuntimeError(f"gradient bucket [{lo}, {hi}) overlaps one already issued "
                                       "this step (missing begin()?)")
                w = dist.all_reduce(grad[lo:hi], op=dist.ReduceOp.SUM, group=self.group,
                                    async_op=overlap)
                if overlap:
                    self.pending.append(w)
                self.covered.append((lo, hi))

    def finish(self, grad, ranges=None):
        """All-reduce the rest of ``ranges`` and wait for every collective of this step;
        records the reduced ranges for scale()."""
        self.reduced = []
        if distributed(self.group):
            want = [(0, grad.numel())] if ranges is None else list(ranges)
            rest = subtract_ranges(want, self.covered)
            for lo, hi in rest:
                self.pending.append(dist.all_reduce(grad[lo:hi], op=dist.ReduceOp.SUM,
                                                    group=self.group, async_op=True))
            for w in self.pending:
                w.wait()
            self.reduced = merge_ranges(self.covered + rest)
        self.pending, self.covered = [], []

    def scale(self, grad):
        n = self.world()
        for lo, hi in self.reduced:
            grad[lo:hi].mul_(1.0 / n)

    def __call__(self, grad, ranges=None):
        self.finish(grad, ranges)
        self.scale(grad)
        self.reduced = []


def merge_ranges(ranges):
    out = []
    for lo, hi in sorted(r for r in ranges if r[1] > r[0]):
        if out and lo <= out[-1][1]:
            out[-1] = (out[-1][0], max(out[-1][1], hi))
        else:
            out.append((lo, hi))
    return out


def subtract_ranges(want, cut):
    """Parts of the ranges ``want`` not covered by ``cut`` (both lists of [lo, hi))."""
    cut = merge_ranges(cut)
    out = []
    for lo, hi in merge_ranges(want):
        for clo, chi in cut:
            if chi <= lo or clo >= hi:
                continue
            if clo > lo:
                out.append((lo, clo))
            lo = max(lo, chi)
            if lo >= hi:
                break
        if lo < hi:
            out.append((lo, hi))
    return out


def grad_allreduce_hook(group=None):
    """fn(grad_arena) for the engines' ``grad_hook``: all-reduce SUM then average, with
    optional early buckets (:class:`GradAllReduce`)."""
    return GradAllReduce(group)


def broadcast_buffers(store, src=0, group=None):
    """Rank ``src``'s buffers to every rank: the f32 arena (centre, BN running stats) and the
    int64 num_batches_tracked counters (pending increments applied first)."""
    if distributed(group):
        dist.broadcast(store.buf_arena, src=src, group=group)
        store.flush_nbt()
        dist.broadcast(store.nbt_arena, src=src, group=group)


def broadcast_parameters(store, src=0, group=None):
    """Initial replication (DDP does this once at wrap time): student + teacher arenas."""
    if distributed(group):
        dist.broadcast(store.student, src=src, group=group)
        if store.teacher is not None:
            dist.broadcast(store.teacher, src=src, group=group)


def gather_rows(x, group=None, out=None):
    """[B, F] local rows -> [world*B, F] global rows in rank order (rank r owns rows
    r*B:(r+1)*B).  Every rank must pass the same B.  ``out``: a fixed destination (what a
    captured step's next segment reads, avdino.capture)."""
    n = dist.get_world_size(group)
    if not distributed(group):
        if out is not None:
            out.copy_(x)
            return out
        return x
    if out is None:
        out = torch.empty((n * x.shape[0],) + tuple(x.shape[1:]), device=x.device, dtype=x.dtype)
    if x.device.type == "cuda" and dist.get_backend(group) == "nccl":
        dist.all_gather_into_tensor(out, x.contiguous(), group=group)
    elif x.device.type == "cuda":   # gloo (the 1-GPU rehearsal): stage through host memory
        h = torch.empty(out.shape, dtype=x.dtype)
        dist.all_gather(list(h.chunk(n)), x.detach().cpu().contiguous(), group=group)
        out.copy_(h)
    else:
        dist.all_gather(list(out.chunk(n)), x.contiguous(), group=group)
    return out


def scatter_rows_grad(dx_all, group=None, out=None):
    """d loss / d(global rows) [world*B, F] from this rank -> SUM over ranks of each rank's
    contribution to MY rows [B, F] (the adjoint of :func:`gather_rows`); ``out`` as there."""
    n = dist.get_world_size(group)
    if not distributed(group):
        if out is not None:
            out.copy_(dx_all)
            return out
        return dx_all
    B = dx_all.shape[0] // n
    if out is None:
        out = torch.empty((B,) + tuple(dx_all.shape[1:]), device=dx_all.device, dtype=dx_all.dtype)
    if dx_all.device.type == "cuda" and dist.get_backend(group) == "nccl":
        dist.reduce_scatter_tensor(out, dx_all.contiguous(), op=dist.ReduceOp.SUM, group=group)
        return out
    # gloo has no reduce_scatter: all-reduce then keep my slice (same result, test backend)
    t = dx_all.detach().cpu().contiguous().clone()
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    r = dist.get_rank(group)
    out.copy_(t[r * B:(r + 1) * B])
    return out
