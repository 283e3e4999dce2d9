"""Graph-replayed training steps (capture.GraphedStep + StepState): a step captured once as a
hipGraph and replayed must be the eager step, bit for bit, on every later step -- fresh dropout
masks (the counter offset lives in device memory), the right Adam bias corrections (device step
count), BN running statistics / counters, centre, teacher EMA -- for the three engines."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

from oracle import spec as OS  # noqa: E402
from oracle.params import make_multimodal_batch, make_simclr_batch, make_state  # noqa: E402


def _dev(b):
    return {k: torch.from_numpy(v).cuda() for k, v in b.items()}


def _run_multi(mode, graph, steps=5, precision=torch.bfloat16):
    from avdino.engine import Hyper, MultiCentralEngine
    from avdino.params import ParamStore
    from avdino.spec import multimodal_dino_sd
    E, D, P, B, G, L = 32, 32, 16, 8, 2, 4
    store = ParamStore(multimodal_dino_sd(mode, E, D, P), "cuda")
    store.load_state_dict({k: torch.from_numpy(np.array(v)) for k, v in
                           make_state(OS.multimodal_dino_spec(mode, E, D, P), 401).items()})
    eng = MultiCentralEngine(store, mode, E, D, P, Hyper(dropout=0.3, fusion_dropout=0.3),
                             act_dtype=precision, seed=3)
    eng.use_graph = graph
    batches = [_dev(make_multimodal_batch(B, G, L, 4000 + i)) for i in range(2)]
    losses = [eng.step(batches[i % 2]).item() for i in range(steps)]
    return store, losses, eng


@pytest.mark.parametrize("mode", ["mse", "semi_supervised", "default"])
def test_graph_replay_equals_eager_multimodal(mode):
    s0, l0, _ = _run_multi(mode, False)
    s1, l1, e1 = _run_multi(mode, True)
    assert len(e1.graph.graphs) == 1           # captured once, replayed for steps 4, 5
    assert l0 == l1, (l0, l1)
    assert len(set(l1[2:])) > 1 or len(set(l1)) > 1
    assert torch.equal(s0.student, s1.student)
    assert torch.equal(s0.teacher, s1.teacher)
    assert torch.equal(s0.buf_arena, s1.buf_arena)
    s0.flush_nbt()
    s1.flush_nbt()
    assert torch.equal(s0.nbt_arena, s1.nbt_arena)
    assert torch.equal(s0.adam_m, s1.adam_m) and torch.equal(s0.adam_v, s1.adam_v)
    assert int(e1.sstate.t.item()) == 5


def test_graph_dropout_masks_change_per_replay():
    """The same batch every step: with the device seed offset, replays differ (fresh masks)
    exactly as eager steps do; with dropout 0 the only change is the parameter update."""
    from avdino.engine import Hyper, MultiCentralEngine
    from avdino.params import ParamStore
    from avdino.spec import multimodal_dino_sd
    E, D, P, B, G, L = 32, 32, 16, 8, 2, 4
    outs = []
    for graph in (False, True):
        store = ParamStore(multimodal_dino_sd("mse", E, D, P), "cuda", seed=5)
        eng = MultiCentralEngine(store, "mse", E, D, P, Hyper(lr=0.0, weight_decay=0.0, dropout=0.5,
                                                              fusion_dropout=0.5, momentum=1.0),
                                 act_dtype=torch.float32, seed=9)
        eng.use_graph = graph
        b = _dev(make_multimodal_batch(B, G, L, 4100))
        outs.append([eng.step(b).item() for _ in range(6)])
    assert outs[0] == outs[1]
    assert len(set(outs[1])) == 6     # lr 0, EMA off: only the masks (and BN running stats) move


def test_graph_replay_equals_eager_unimodal():
    from avdino.engine import Hyper, UniModalEngine
    from avdino.params import ParamStore
    from avdino.spec import unimodal_dino_sd
    res = []
    for graph in (False, True):
        store = ParamStore(unimodal_dino_sd("image_simple", 64, 32), "cuda", seed=2)
        eng = UniModalEngine(store, "image_simple", 64, 32, Hyper(dropout=0.3),
                             act_dtype=torch.bfloat16, cos_alpha=0.3, seed=4)
        eng.use_graph = graph
        bs = [_dev(make_multimodal_batch(16, 2, 2, 4200 + i, with_originals=False)) for i in range(2)]
        res.append(([eng.step(bs[i % 2]).item() for i in range(5)], store))
    assert res[0][0] == res[1][0]
    assert torch.equal(res[0][1].student, res[1][1].student)
    assert torch.equal(res[0][1].teacher, res[1][1].teacher)


def test_graph_replay_equals_eager_simclr():
    from avdino.engine import Hyper, SimCLREngine
    from avdino.params import ParamStore
    from avdino.spec import simclr_sd
    modes = [0, 2, 1, 3, 2, 0, 3, 2, 2, 1]
    res = []
    for graph in (False, True):
        store = ParamStore(simclr_sd(64, 32), "cuda", seed=3, has_teacher=False,
                           groups=SimCLREngine.GROUPS)
        eng = SimCLREngine(store, 64, 32, Hyper(weight_decay=0.0), act_dtype=torch.bfloat16,
                           negatives="local")
        eng.use_graph = graph
        b = make_simclr_batch(8, 4300)
        b = {k: torch.from_numpy(v).cuda() for k, v in b.items()}
        res.append(([eng.step(b, m).item() for m in modes], store, eng))
    assert res[0][0] == res[1][0]
    assert torch.equal(res[0][1].student, res[1][1].student)
    assert res[1][2].adam_t == res[0][2].adam_t
    assert [int(s.t.item()) for s in res[1][2].sstates] == res[0][2].adam_t


@pytest.mark.parametrize("graph", [False, True])
@pytest.mark.parametrize("mode", ["mse", "semi_supervised"])
def test_pipelined_teacher_equals_sequential(mode, graph):
    """engine.pipeline: the next batch's teacher forward under this step's backward (fourth
    stream, the next step's dropout offset) gives the sequential step's losses and parameters
    bit for bit; only the teacher's BN running statistics run one batch ahead."""
    from avdino.engine import Hyper, MultiCentralEngine
    from avdino.params import ParamStore
    from avdino.spec import multimodal_dino_sd
    E, D, P, B, G, L = 32, 32, 16, 8, 2, 4
    res = []
    for pipe in (False, True):
        store = ParamStore(multimodal_dino_sd(mode, E, D, P), "cuda")
        store.load_state_dict({k: torch.from_numpy(np.array(v)) for k, v in
                               make_state(OS.multimodal_dino_spec(mode, E, D, P), 402).items()})
        eng = MultiCentralEngine(store, mode, E, D, P, Hyper(dropout=0.3, fusion_dropout=0.3),
                                 act_dtype=torch.bfloat16, seed=5)
        eng.use_graph = graph
        eng.pipeline = pipe
        batches = [_dev(make_multimodal_batch(B, G, L, 4200 + i)) for i in range(2)]
        losses = [eng.step(batches[i % 2], next_batch=batches[(i + 1) % 2]).item()
                  for i in range(6)]
        res.append((store, losses, eng))
    (s0, l0, _), (s1, l1, e1) = res
    assert l0 == l1, (l0, l1)
    assert len(set(l1)) > 1
    if graph:
        assert len(e1.graph.graphs) == 1
    assert torch.equal(s0.student, s1.student)
    assert torch.equal(s0.teacher, s1.teacher)
    assert torch.equal(s0.adam_m, s1.adam_m) and torch.equal(s0.adam_v, s1.adam_v)
    # the student's BN buffers match; the pipelined teacher has seen one more batch
    sb = [k for k in s0.buffers if k.startswith("student.") or k == "center"]
    assert sb
    for k in sb:
        assert torch.equal(s0[k], s1[k]), k
    assert e1._t_ready is not None


def test_graph_recaptured_after_workspace_growth_simclr():
    """a graph captured for SimCLR's image/image mode (small staged input) before the
    audio/audio mode is first seen must not be replayed after that mode's eager warm-up grows
    the shared workspace buffers (the old graph would address freed memory): it is re-captured,
    and every step equals the eager run bit for bit."""
    from avdino.engine import Hyper, SimCLREngine
    from avdino.params import ParamStore
    from avdino.spec import simclr_sd
    modes = [0, 0, 0, 0, 1, 1, 1, 0, 0, 3, 3, 3, 0, 1]
    res = []
    for graph in (False, True):
        store = ParamStore(simclr_sd(64, 32), "cuda", seed=3, has_teacher=False,
                           groups=SimCLREngine.GROUPS)
        eng = SimCLREngine(store, 64, 32, Hyper(weight_decay=0.0), act_dtype=torch.bfloat16,
                           negatives="local")
        eng.use_graph = graph
        b = {k: torch.from_numpy(v).cuda() for k, v in make_simclr_batch(8, 4400).items()}
        res.append(([eng.step(b, m).item() for m in modes], store, eng))
    assert res[0][0] == res[1][0], (res[0][0], res[1][0])
    assert torch.equal(res[0][1].student, res[1][1].student)
    g = res[1][2].graph
    # mode 0 was captured before mode 1 grew the buffers, then captured again
    assert g.captures > len(g.graphs), (g.captures, list(g.graphs))


def test_only_graph_goes_stale_and_is_recaptured():
    """The pool-reset branch of GraphedStep.run (capture.py): the ONLY captured graph goes stale
    (one of the engine's workspaces grows after its capture), is dropped together with its
    memory pool, and the step runs eagerly, captures again on a fresh pool and replays -- every
    step equal to the eager run.  Another workspace growing (a probe's) retires nothing."""
    from avdino.engine import Workspace
    s0, l0, _ = _run_multi("mse", False, steps=8)
    from avdino.engine import Hyper, MultiCentralEngine
    from avdino.params import ParamStore
    from avdino.spec import multimodal_dino_sd
    E, D, P, B, G, L = 32, 32, 16, 8, 2, 4
    store = ParamStore(multimodal_dino_sd("mse", E, D, P), "cuda")
    store.load_state_dict({k: torch.from_numpy(np.array(v)) for k, v in
                           make_state(OS.multimodal_dino_spec("mse", E, D, P), 401).items()})
    eng = MultiCentralEngine(store, "mse", E, D, P, Hyper(dropout=0.3, fusion_dropout=0.3),
                             act_dtype=torch.bfloat16, seed=3)
    eng.use_graph = True
    batches = [_dev(make_multimodal_batch(B, G, L, 4000 + i)) for i in range(2)]
    losses = []
    for i in range(4):                  # 2 eager, capture, replay
        losses.append(eng.step(batches[i % 2]).item())
    assert eng.graph.captures == 1 and eng.graph.pool is not None
    Workspace("cuda").get("probe", 1 << 20)       # someone else's scratch: still replayed
    losses.append(eng.step(batches[0]).item())
    assert eng.graph.captures == 1 and len(eng.graph.graphs) == 1
    eng.ws.get("grown.elsewhere", 1 << 20)        # the engine's own workspace moves
    losses.append(eng.step(batches[1]).item())    # stale: dropped with its pool, eager
    assert not eng.graph.graphs and eng.graph.pool is None
    losses.append(eng.step(batches[0]).item())    # captured again on a new pool
    assert eng.graph.captures == 2 and eng.graph.pool is not None
    losses.append(eng.step(batches[1]).item())    # replayed
    assert losses == l0, (losses, l0)
    assert torch.equal(s0.student, store.student) and torch.equal(s0.teacher, store.teacher)
