"""Multi-process (world_size 2, gloo, CPU) tests of the data-parallel plumbing in
avdino/dist.py: gradient averaging over the flat arena, rank-0 buffer broadcast (DDP
broadcast_buffers), and the global-negative all-gather whose gradient is routed back to the
owning shard -- checked against the float64 oracle's single-device InfoNCE / NT-Xent over the
global batch.  No GPU and no libavdino needed (the helpers move torch tensors only)."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "multimodal-ssl-avmnist_amd")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(fn, world=2):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_entry, args=(fn, r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    errs = [r for r in res if isinstance(r, str)]
    assert not errs, errs[0]
    return sorted(res, key=lambda r: r[0])


def _entry(fn, r, world, port, q):
    try:
        for p in (REPO, PKG):
            if p not in sys.path:
                sys.path.insert(0, p)
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=r, world_size=world)
        out = fn(r, world)
        dist.destroy_process_group()
        q.put((r, out))
    except Exception:  # report to the parent instead of hanging it
        import traceback
        q.put(traceback.format_exc())


# ----------------------------------------------------------------- grad all-reduce + buffers
def _grad_and_buffers(r, world):
    from avdino import dist as D
    from avdino.params import ParamStore
    from avdino.spec import multimodal_dino_sd
    store = ParamStore(multimodal_dino_sd("mse", 16, 16, 8), "cpu", seed=0)
    g = torch.Generator().manual_seed(100 + r)
    store.grad.copy_(torch.randn(store.grad.shape, generator=g))
    mine = store.grad.clone()
    D.grad_allreduce_hook()(store.grad)
    store.buf_arena.fill_(float(r + 1))           # ranks disagree before the broadcast
    D.broadcast_buffers(store)
    return mine.numpy(), store.grad.numpy(), store.buf_arena.numpy()


def test_grad_allreduce_and_buffer_broadcast():
    res = _run(_grad_and_buffers)
    mean = (res[0][1][0] + res[1][1][0]) / 2
    for _, (mine, avg, buf) in res:
        np.testing.assert_allclose(avg, mean, rtol=1e-6, atol=1e-7)
        assert np.all(buf == 1.0)                 # rank 0's buffers everywhere


def _bucketed(r, world):
    """GradAllReduce with early buckets (overlapping, unordered) + the remainder == flat."""
    from avdino import dist as D
    g = torch.Generator().manual_seed(300 + r)
    grad = torch.randn(1000, generator=g)
    flat = grad.clone()
    D.GradAllReduce()(flat)
    b = grad.clone()
    h = D.GradAllReduce()
    h.bucket(b, [(600, 800), (0, 128)])
    h.bucket(b, [(128, 200)])
    h(b)
    sub = grad.clone()                # only some ranges (SimCLR's used towers)
    h2 = D.GradAllReduce()
    h2.bucket(sub, [(0, 100)])
    h2(sub, ranges=[(0, 300), (500, 700)])
    return flat.numpy(), b.numpy(), sub.numpy(), grad.numpy()


def test_bucketed_allreduce_equals_flat():
    from avdino.dist import merge_ranges, subtract_ranges
    assert subtract_ranges([(0, 100)], [(10, 20), (50, 60)]) == [(0, 10), (20, 50), (60, 100)]
    assert subtract_ranges([(0, 10), (20, 30)], [(5, 25)]) == [(0, 5), (25, 30)]
    assert subtract_ranges([(0, 10)], [(0, 10)]) == []
    assert merge_ranges([(5, 6), (0, 5), (7, 9)]) == [(0, 6), (7, 9)]
    res = _run(_bucketed)
    raw = [x[1][3] for x in res]
    for _, (flat, b, sub, grad) in res:
        np.testing.assert_array_equal(flat, b)
        mean = (raw[0] + raw[1]) / 2
        np.testing.assert_allclose(flat, mean, rtol=1e-6, atol=1e-7)
        inside = np.zeros(1000, bool)
        inside[0:300] = inside[500:700] = True
        np.testing.assert_array_equal(sub[inside], flat[inside])
        np.testing.assert_array_equal(sub[~inside], grad[~inside])   # untouched outside


def _async_buckets(r, world):
    """The asynchronous bucket path (what RCCL runs: async_op=True, pending works waited in
    finish, x 1/world in scale) under gloo, in the engines' order begin -> bucket* -> finish ->
    scale, over two steps; the first step before it is ABORTED after a bucket (no finish), and
    begin() must keep its stale ranges from suppressing the next step's reduction."""
    from avdino import dist as D
    g = torch.Generator().manual_seed(500 + r)
    out = []
    h = D.GradAllReduce(overlap=True)
    aborted = torch.randn(1000, generator=g)
    h.begin()
    h.bucket(aborted, [(0, 400)])            # the step dies here: no finish()
    for step in range(2):
        grad = torch.randn(1000, generator=g)
        raw = grad.clone()
        flat = grad.clone()
        D.GradAllReduce()(flat)
        h.begin()
        assert not h.pending and not h.covered
        h.bucket(grad, [(0, 400)])          # early bucket (heads)
        h.bucket(grad, [(400, 650)])        # second bucket (encoder Linears)
        assert len(h.pending) == 2
        h.finish(grad)                       # the rest (conv weights) + wait
        assert h.reduced == [(0, 1000)] and not h.pending
        h.scale(grad)
        out.append((raw.numpy(), flat.numpy(), grad.numpy()))
    spare = torch.zeros(100)
    try:
        h.begin()
        h.bucket(spare, [(0, 10)])
        h.bucket(spare, [(5, 20)])           # overlaps: a protocol error, not a silent skip
        overlap_raised = False
    except RuntimeError:
        overlap_raised = True
    h.begin()
    return out, overlap_raised


def test_async_buckets_equal_flat_and_survive_an_aborted_step():
    res = _run(_async_buckets)
    for _, (steps, raised) in res:
        assert raised
        for k, (raw, flat, got) in enumerate(steps):
            mean = (res[0][1][0][k][0] + res[1][1][0][k][0]) / 2
            np.testing.assert_array_equal(got, flat)
            np.testing.assert_allclose(got, mean, rtol=1e-6, atol=1e-7)


# ----------------------------------------------------------------- global negatives
class _Gather(torch.autograd.Function):
    """gather_rows with its adjoint (scatter_rows_grad) as the backward."""

    @staticmethod
    def forward(ctx, x):
        from avdino import dist as D
        return D.gather_rows(x)

    @staticmethod
    def backward(ctx, g):
        from avdino import dist as D
        return D.scatter_rows_grad(g)


def _global_infonce(r, world, B=6, P=8, tau=0.07):
    """Sharded InfoNCE: rank r holds rows r*B:(r+1)*B of the global batch; loss_r = local mean
    of the row/column cross-entropies against the gathered other modality (the engine's
    global-negative mode).  Returns d(loss_r) routed to every owner, per rank."""
    rng = np.random.default_rng(7)
    zi = rng.normal(size=(world * B, P))
    za = rng.normal(size=(world * B, P))
    i = torch.tensor(zi[r * B:(r + 1) * B], requires_grad=True)
    a = torch.tensor(za[r * B:(r + 1) * B], requires_grad=True)
    ni = torch.nn.functional.normalize(i, dim=-1)
    na = torch.nn.functional.normalize(a, dim=-1)
    ni_all, na_all = _Gather.apply(ni), _Gather.apply(na)
    tgt = torch.arange(B) + r * B
    s_rows = ni @ na_all.T / tau                  # my rows of S
    s_cols = na @ ni_all.T / tau                  # my rows of S^T
    loss = 0.5 * (torch.nn.functional.cross_entropy(s_rows, tgt)
                  + torch.nn.functional.cross_entropy(s_cols, tgt))
    loss.backward()
    return loss.item(), i.grad.numpy(), a.grad.numpy(), zi, za


def test_global_negative_infonce_equals_single_device():
    from oracle import numpy_oracle as O
    res = _run(_global_infonce)
    world = len(res)
    zi, za = res[0][1][3], res[0][1][4]
    loss, dzi, dza = O.infonce_loss(zi, za)
    # DDP averages per-rank gradients: mean_r loss_r == global loss
    np.testing.assert_allclose(np.mean([x[1][0] for x in res]), loss, rtol=1e-10)
    gi = np.concatenate([x[1][1] for x in res]) / world
    ga = np.concatenate([x[1][2] for x in res]) / world
    np.testing.assert_allclose(gi, dzi, rtol=1e-8, atol=1e-12)
    np.testing.assert_allclose(ga, dza, rtol=1e-8, atol=1e-12)


def _global_ntxent(r, world, B=5, P=8, tau=0.07):
    """Sharded NT-Xent (SimCLR config 4): rank r holds its [2B] reps (view 1 rows then view 2
    rows of its B samples); similarities against all gathered reps, diagonal masked."""
    rng = np.random.default_rng(11)
    reps = rng.normal(size=(world, 2 * B, P))     # per-rank [z1; z2]
    x = torch.tensor(reps[r], requires_grad=True)
    n = torch.nn.functional.normalize(x, dim=-1)
    n_all = _Gather.apply(n)                       # [world*2B]: rank-major, view-major within
    S = n @ n_all.T / tau
    own = torch.arange(2 * B) + r * 2 * B
    S = S.masked_fill(torch.nn.functional.one_hot(own, world * 2 * B).bool(), float("-inf"))
    pos = torch.cat([torch.arange(B) + B, torch.arange(B)]) + r * 2 * B
    loss = torch.nn.functional.cross_entropy(S, pos)
    loss.backward()
    return loss.item(), x.grad.numpy(), reps


def test_global_negative_ntxent_equals_single_device():
    """Single-device reference over the global batch, with rows ordered [z1 of all; z2 of all]
    as the reference builds them (multimodal_simclr.py:74-89); the sharded layout is a row
    permutation of it, so loss and per-row gradients must agree after un-permuting."""
    from oracle import numpy_oracle as O
    res = _run(_global_ntxent)
    world = len(res)
    reps = res[0][1][2]
    B = reps.shape[1] // 2
    z1 = np.concatenate([reps[w, :B] for w in range(world)])
    z2 = np.concatenate([reps[w, B:] for w in range(world)])
    loss, dreps = O.nt_xent_loss(np.concatenate([z1, z2]))
    np.testing.assert_allclose(np.mean([x[1][0] for x in res]), loss, rtol=1e-10)
    for w, (_, (_, g, _)) in enumerate(res):
        np.testing.assert_allclose(g[:B] / world, dreps[w * B:(w + 1) * B], rtol=1e-8, atol=1e-12)
        np.testing.assert_allclose(g[B:] / world, dreps[world * B + w * B: world * B + (w + 1) * B],
                                   rtol=1e-8, atol=1e-12)
