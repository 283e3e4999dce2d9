"""The RCCL code of the data-parallel step, executed.

Every world-2 test runs gloo (both ranks on one GPU), so the branches that only run under the
``nccl`` backend -- the asynchronous gradient buckets on the process group's stream
(avdino.dist.GradAllReduce), ``all_gather_into_tensor`` for the global negatives and
``reduce_scatter_tensor`` for their column gradients -- had never executed.  Here one process
initialises ``torch.distributed`` with ``nccl`` (= RCCL on ROCm) at world 1 and
``avdino.dist.forced()`` makes the engines take the data-parallel path anyway (an all-reduce /
all-gather / reduce-scatter over one rank is the identity): the graph-segmented step with its
host points, the buckets issued asynchronously inside the captured step, the gathered negatives.
Results must equal the plain single-GPU step bit for bit (losses, student, teacher, buffers,
Adam moments) for mse, infonce (global negatives) and SimCLR, and the RCCL calls must have run.
No hardware-queue setting is touched (the box's default 4)."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

E, D, P, B, G, L = 32, 32, 16, 8, 2, 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.fixture(scope="module")
def rccl():
    import torch.distributed as dist
    assert "GPU_MAX_HW_QUEUES" not in os.environ or int(os.environ["GPU_MAX_HW_QUEUES"]) <= 4
    os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0,
                            world_size=1, device_id=torch.device("cuda:0"))
    calls = {}
    orig = {n: getattr(dist, n) for n in ("all_reduce", "all_gather_into_tensor",
                                          "reduce_scatter_tensor", "broadcast")}

    def counted(n):
        def f(*a, **k):
            calls[n] = calls.get(n, 0) + 1
            return orig[n](*a, **k)
        return f
    for n in orig:
        setattr(dist, n, counted(n))
    try:
        assert dist.get_backend() == "nccl"
        yield calls
    finally:
        for n, f in orig.items():
            setattr(dist, n, f)
        torch.cuda.synchronize()
        dist.destroy_process_group()


def _host(t):
    return t.detach().float().cpu().numpy()


def _multi(mode, forced, steps=4):
    from avdino import dist as AD
    from avdino.engine import Hyper, MultiCentralEngine
    from avdino.params import ParamStore
    from avdino.spec import multimodal_dino_sd
    from oracle.params import make_multimodal_batch
    store = ParamStore(multimodal_dino_sd(mode, E, D, P), "cuda", seed=11)
    kw = dict(grad_hook=AD.GradAllReduce(), buffer_hook=AD.broadcast_buffers) if forced else {}
    eng = MultiCentralEngine(store, mode, E, D, P, Hyper(dropout=0.3, fusion_dropout=0.3),
                             act_dtype=torch.bfloat16, seed=3, negatives="global", **kw)
    eng.use_graph = True
    batches = [{k: torch.from_numpy(v).cuda() for k, v in make_multimodal_batch(B, G, L, 6300 + i).items()}
               for i in range(2)]
    if forced:
        AD.broadcast_parameters(store)
    losses = [eng.step(batches[i % 2]).item() for i in range(steps)]
    torch.cuda.synchronize()
    store.flush_nbt()
    segs = [eng.graph.segments(k) for k in eng.graph.graphs]
    return dict(losses=losses, student=_host(store.student), teacher=_host(store.teacher),
                buf=_host(store.buf_arena), m=_host(store.adam_m), segs=segs)


def _simclr(forced, modes=(0, 1, 3, 2, 2, 2, 2, 3)):
    from avdino import dist as AD
    from avdino.engine import Hyper, SimCLREngine
    from avdino.params import ParamStore
    from avdino.spec import simclr_sd
    from oracle.params import make_simclr_batch
    Ds, Ps = 32, 16
    store = ParamStore(simclr_sd(Ds, Ps), "cuda", seed=21, has_teacher=False,
                       groups=list(SimCLREngine.GROUPS))
    kw = dict(grad_hook=AD.GradAllReduce()) if forced else {}
    eng = SimCLREngine(store, Ds, Ps, Hyper(lr=1e-3), act_dtype=torch.bfloat16, negatives="global", **kw)
    eng.use_graph = True
    b = {k: torch.from_numpy(v).cuda() for k, v in make_simclr_batch(B, 6400).items()}
    losses = [eng.step(b, mode=m).item() for m in modes]
    torch.cuda.synchronize()
    segs = {k: eng.graph.segments(k) for k in eng.graph.graphs}
    return dict(losses=losses, student=_host(store.student), m=_host(store.adam_m), segs=segs)


def _same(a, b, keys):
    for k in keys:
        if isinstance(a[k], np.ndarray):
            assert np.array_equal(a[k], b[k]), k
        else:
            assert a[k] == b[k], (k, a[k], b[k])


@pytest.mark.parametrize("mode", ["infonce", "mse"])
def test_rccl_step_equals_single_gpu_step(rccl, mode):
    from avdino import dist as AD
    plain = _multi(mode, False)
    n0 = dict(rccl)
    with AD.forced():
        run = _multi(mode, True)
    _same(plain, run, ("losses", "student", "teacher", "buf", "m"))
    assert plain["segs"] == [1]
    # gather + scatter (infonce), early bucket, encoder-Linear bucket, final exchange
    assert run["segs"] == [6 if mode == "infonce" else 4], run["segs"]
    d = {k: rccl.get(k, 0) - n0.get(k, 0) for k in rccl}
    assert d.get("all_reduce", 0) >= 3 * 4 and d.get("broadcast", 0) >= 4, d
    if mode == "infonce":
        assert d.get("all_gather_into_tensor", 0) >= 2 * 4 and d.get("reduce_scatter_tensor", 0) >= 2 * 4, d


def test_rccl_simclr_step_equals_single_gpu_step(rccl):
    from avdino import dist as AD
    plain = _simclr(False)
    n0 = dict(rccl)
    with AD.forced():
        run = _simclr(True)
    _same(plain, run, ("losses", "student", "m"))
    assert run["segs"].get((2, B)) == 5, run["segs"]
    d = {k: rccl.get(k, 0) - n0.get(k, 0) for k in rccl}
    assert d.get("all_gather_into_tensor", 0) > 0 and d.get("reduce_scatter_tensor", 0) > 0, d
    assert d.get("all_reduce", 0) > 0, d
