"""Data-parallel plumbing of the training step: one process per GPU,
``torch.distributed`` with backend ``nccl`` (= RCCL over xGMI) on MI355X, ``gloo`` in the CPU
tests.  Nothing here computes model math; it moves the engine's flat arenas.

* :func:`grad_allreduce_hook` -- the per-step gradient exchange: ONE all-reduce over the flat
  live-gradient arena (2.12 M f32 = 8.5 MB for mse/infonce; the reference's DDP buckets the
  same parameters, dead fc1/fc2 excluded because they have no gradient), then x 1/world
  (DDP's gradient averaging).
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


def rank(group=None):
    return dist.get_rank(group) if dist.is_available() and dist.is_initialized() else 0


def grad_allreduce_hook(group=None):
    """fn(grad_arena) for MultiCentralEngine(grad_hook=...): all-reduce SUM then average."""
    def hook(grad):
        n = dist.get_world_size(group)
        if n > 1:
            dist.all_reduce(grad, op=dist.ReduceOp.SUM, group=group)
            grad.mul_(1.0 / n)
    return hook


def broadcast_buffers(store, src=0, group=None):
    """Rank ``src``'s buffers to every rank: the f32 arena (centre, BN running stats) and the
    int64 num_batches_tracked counters (pending increments applied first)."""
    if dist.get_world_size(group) > 1:
        dist.broadcast(store.buf_arena, src=src, group=group)
        store.flush_nbt()
        dist.broadcast(store.nbt_arena, src=src, group=group)


def broadcast_parameters(store, src=0, group=None):
    """Initial replication (DDP does this once at wrap time): student + teacher arenas."""
    if dist.get_world_size(group) > 1:
        dist.broadcast(store.student, src=src, group=group)
        if store.teacher is not None:
            dist.broadcast(store.teacher, src=src, group=group)


def gather_rows(x, group=None):
    """[B, F] local rows -> [world*B, F] global rows in rank order (rank r owns rows
    r*B:(r+1)*B).  Every rank must pass the same B."""
    n = dist.get_world_size(group)
    if n == 1:
        return x
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


def scatter_rows_grad(dx_all, group=None):
    """d loss / d(global rows) [world*B, F] from this rank -> SUM over ranks of each rank's
    contribution to MY rows [B, F] (the adjoint of :func:`gather_rows`)."""
    n = dist.get_world_size(group)
    if n == 1:
        return dx_all
    B = dx_all.shape[0] // n
    if dx_all.device.type == "cuda" and dist.get_backend(group) == "nccl":
        out = torch.empty((B,) + tuple(dx_all.shape[1:]), device=dx_all.device, dtype=dx_all.dtype)
        dist.reduce_scatter_tensor(out, dx_all.contiguous(), op=dist.ReduceOp.SUM, group=group)
        return out
    # gloo has no reduce_scatter: all-reduce then keep my slice (same result, test backend)
    t = dx_all.detach().cpu().contiguous().clone()
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    r = dist.get_rank(group)
    return t[r * B:(r + 1) * B].to(dx_all.device)
