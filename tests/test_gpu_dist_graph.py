"""Captured data-parallel steps at world 2: two processes, gloo, both on
cuda:0 (the 1-GPU rehearsal of the 8-GPU RCCL run).

* Global-negative InfoNCE (config 3) and NT-Xent (config 4) steps are captured graphs: the
  all-gather / reduce-scatter are host points between graph segments (avdino.capture), so
  ``use_graph`` no longer falls back to eager at world > 1.  Replayed steps == eager steps,
  bit for bit (losses, parameters, teacher, buffers).
* The gradient all-reduce in buckets (avdino.dist.GradAllReduce: heads / fusion / projection
  issued at a host point inside the backward, the two encoder Linears at a second one before
  the conv branches, the rest -- the conv weights -- at the step's last host point, followed
  by the 1/world scale and Adam in the last captured segment; SimCLR: the first tower under
  the second's backward) == one flat all-reduce of the arena, bit for bit (a 2-rank sum is
  order-free), and the buckets of every step cover the gradient arena exactly once."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

from tests.test_gpu_dist_dino import _run2  # noqa: E402

E, D, P, B, G, L = 32, 32, 16, 4, 2, 2


def _flat_hook():
    import torch.distributed as dist

    def hook(grad):
        dist.all_reduce(grad, op=dist.ReduceOp.SUM)
        grad.mul_(0.5)
    return hook


def _host(t):
    return t.detach().float().cpu().numpy()


class _Logged:
    """GradAllReduce that records the ranges each step's collectives reduce."""

    def __new__(cls):
        from avdino import dist as AD

        class L(AD.GradAllReduce):
            log = []

            def begin(self):
                super().begin()
                L.log.append([])

            def bucket(self, grad, ranges):
                L.log[-1].extend((lo, hi) for lo, hi in ranges if hi > lo)
                super().bucket(grad, ranges)

            def finish(self, grad, ranges=None):
                from avdino.dist import subtract_ranges
                want = [(0, grad.numel())] if ranges is None else list(ranges)
                L.log[-1].extend(subtract_ranges(want, self.covered))
                super().finish(grad, ranges)
        return L()


def _partition(ranges, n):
    """The ranges are disjoint and cover [0, n)."""
    rs = sorted(ranges)
    pos = 0
    for lo, hi in rs:
        if lo != pos:
            return False
        pos = hi
    return pos == n


def _multi(r, mode, graph, bucket, steps=5):
    from avdino import dist as AD
    from avdino.engine import Hyper, MultiCentralEngine
    from avdino.params import ParamStore
    from avdino.spec import multimodal_dino_sd
    from oracle.params import make_multimodal_batch
    store = ParamStore(multimodal_dino_sd(mode, E, D, P), "cuda", seed=11 + r)
    AD.broadcast_parameters(store)
    eng = MultiCentralEngine(store, mode, E, D, P, Hyper(dropout=0.3, fusion_dropout=0.3),
                             act_dtype=torch.bfloat16, seed=3,
                             grad_hook=_Logged() if bucket else _flat_hook(),
                             buffer_hook=AD.broadcast_buffers, negatives="global")
    eng.use_graph = graph
    batches = []
    for i in range(2):
        b = make_multimodal_batch(2 * B, G, L, 6100 + i)
        batches.append({k: torch.from_numpy(v[r * B:(r + 1) * B]).cuda() for k, v in b.items()})
    losses = [eng.step(batches[i % 2]).item() for i in range(steps)]
    store.flush_nbt()
    segs = [eng.graph.segments(k) for k in eng.graph.graphs]
    cover = None
    if bucket:
        log = type(eng.grad_hook).log
        cover = (len(log), all(_partition(s, store.grad.numel()) for s in log),
                 [len(s) for s in log])
    return dict(losses=losses, student=_host(store.student), teacher=_host(store.teacher),
                buf=_host(store.buf_arena), m=_host(store.adam_m), segs=segs, cover=cover)


def _simclr(r, graph, bucket, modes=(0, 1, 3, 2, 2, 2, 2, 3, 3)):
    from avdino import dist as AD
    from avdino.engine import Hyper, SimCLREngine
    from avdino.params import ParamStore
    from avdino.spec import simclr_sd
    from oracle.params import make_simclr_batch
    Ds, Ps = 32, 16
    store = ParamStore(simclr_sd(Ds, Ps), "cuda", seed=21 + r, has_teacher=False,
                       groups=list(SimCLREngine.GROUPS))
    AD.broadcast_parameters(store)
    eng = SimCLREngine(store, Ds, Ps, Hyper(lr=1e-3), act_dtype=torch.bfloat16, negatives="global",
                       grad_hook=AD.GradAllReduce() if bucket else _flat_hook())
    eng.use_graph = graph
    b = make_simclr_batch(2 * B, 6200)
    mine = {k: torch.from_numpy(v[r * B:(r + 1) * B]).cuda() for k, v in b.items()}
    losses = [eng.step(mine, mode=m).item() for m in modes]
    segs = {k: eng.graph.segments(k) for k in eng.graph.graphs}
    return dict(losses=losses, student=_host(store.student), m=_host(store.adam_m), segs=segs)


def _rank(r, world):
    out = {}
    for mode in ("infonce", "mse"):
        for graph, bucket in ((False, False), (False, True), (True, True)):
            out[(mode, graph, bucket)] = _multi(r, mode, graph, bucket)
    for graph, bucket in ((False, False), (False, True), (True, True)):
        out[("simclr", graph, bucket)] = _simclr(r, graph, bucket)
    return out


@pytest.fixture(scope="module")
def world2():
    return _run2(_rank)


def _same(a, b, keys):
    for k in keys:
        if isinstance(a[k], np.ndarray):
            assert np.array_equal(a[k], b[k]), k
        else:
            assert a[k] == b[k], (k, a[k], b[k])


@pytest.mark.parametrize("mode", ["infonce", "mse"])
def test_world2_graph_and_buckets_equal_eager_flat(world2, mode):
    keys = ("losses", "student", "teacher", "buf", "m")
    for res in world2:
        flat, buck, graph = (res[(mode, False, False)], res[(mode, False, True)],
                             res[(mode, True, True)])
        _same(flat, buck, keys)        # bucketed all-reduce == one flat all-reduce
        _same(buck, graph, keys)       # captured + replayed == eager
        assert len(graph["segs"]) == 1
        # segments: [gather, scatter,] early bucket, encoder-Linear bucket, final exchange
        # -> 6 (infonce) / 4 (mse)
        assert graph["segs"][0] == (6 if mode == "infonce" else 4), graph["segs"]
        for run in (buck, graph):   # every step's collectives partition the gradient arena
            nsteps, exact, nranges = run["cover"]
            assert nsteps == 5 and exact, run["cover"]
            assert min(nranges) >= 3, run["cover"]
    # DDP keeps the replicas identical (BN running stats: each rank's own last batch)
    _same(world2[0][(mode, True, True)], world2[1][(mode, True, True)], ("student", "teacher"))


def test_world2_simclr_graph_and_buckets_equal_eager_flat(world2):
    keys = ("losses", "student", "m")
    for res in world2:
        flat, buck, graph = (res[("simclr", False, False)], res[("simclr", False, True)],
                             res[("simclr", True, True)])
        _same(flat, buck, keys)
        _same(buck, graph, keys)
        # every mode's buffers sized first (0, 1, 3), then mode 2 (image/audio) 4 times:
        # captured on its third, replayed on its fourth; gather + scatter + the first
        # tower's bucket + the final exchange -> 5 segments
        assert graph["segs"].get((2, B)) == 5, graph["segs"]
    _same(world2[0][("simclr", True, True)], world2[1][("simclr", True, True)], ("student",))
