"""Multimodal SimCLR training-step parity (BASELINE config 4) and the
global-negative data-parallel path (8(e)), HIP engine (fp32 parity mode) vs the float64
oracle, which is pinned to the reference by tests/test_oracle_golden.py on the same dims and
seeds (tests/golden/simclr_small*.npz).

Tolerances: loss 3e-5 abs; z1/z2 1e-5 rel-L2; gradients 1e-3 rel-L2 (median 1e-4; near-zero
biases feeding a BatchNorm 1e-4 abs); BN running stats 1e-5; Adam: the towers not used by the
step are bit-unchanged, the used ones match torch.optim.Adam (no weight decay) applied to our
gradients to 1e-6.  World-2 (gloo, both ranks on cuda:0): each rank's all-reduced gradient
equals the oracle's global-negative data-parallel gradient to 1e-3."""
import os
import socket
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

from oracle import numpy_oracle as O  # noqa: E402
from oracle import spec as OS  # noqa: E402
from oracle.params import make_simclr_batch, make_state  # noqa: E402

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "multimodal-ssl-avmnist_amd")
D, P, B, PSEED, BSEED = 256, 256, 4, 107, 1007   # = tests/golden/simclr_small


def rel(a, b):
    a = np.asarray(a, np.float64).ravel()
    b = np.asarray(b, np.float64).ravel()
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30)


def host(t):
    return t.detach().float().cpu().numpy().astype(np.float64)


def build(act=torch.float32, negatives="global", device="cuda"):
    from avdino.engine import Hyper, SimCLREngine
    from avdino.params import ParamStore
    from avdino.spec import simclr_sd
    sd = simclr_sd(D, P)
    assert list(sd.keys()) == list(OS.simclr_spec(D, P).keys())
    store = ParamStore(sd, device, has_teacher=False, groups=SimCLREngine.GROUPS)
    state = make_state(OS.simclr_spec(D, P), PSEED)
    store.load_state_dict({k: torch.from_numpy(np.array(v)) for k, v in state.items()})
    hp = Hyper(lr=1e-4, weight_decay=0.0)
    return store, SimCLREngine(store, D, P, hp, act_dtype=act, negatives=negatives), state


def check_grads(store, ref_grads, towers):
    prefixes = tuple(("image_", "audio_")[t] for t in towers)
    used = [k for k in store.live_keys if k.startswith(prefixes)]
    assert sorted(used) == sorted(ref_grads.keys())
    errs = {}
    for k in used:
        g, r = host(store.grad_of(k)), ref_grads[k]
        if np.linalg.norm(r) < 1e-4:
            assert np.linalg.norm(g - r) <= 1e-4, (k, np.linalg.norm(g - r))
            continue
        errs[k] = rel(g, r)
    worst = sorted(errs.items(), key=lambda kv: -kv[1])[:4]
    print("worst grad errors:", worst)
    assert worst[0][1] < 1e-3, worst
    assert np.median(list(errs.values())) < 1e-4


@pytest.mark.parametrize("mode", [0, 1, 2, 3])
def test_simclr_step_matches_oracle(mode):
    store, eng, state = build()
    batch = make_simclr_batch(B, BSEED)
    ref = O.simclr_step(state, batch, mode)
    loss = eng.forward({k: torch.from_numpy(v).cuda() for k, v in batch.items()}, mode)
    z1, z2 = eng.outputs()
    assert abs(loss.item() - ref["loss"]) < 3e-5, (loss.item(), ref["loss"])
    assert rel(host(z1), ref["z1"]) < 1e-5 and rel(host(z2), ref["z2"]) < 1e-5
    eng.backward()
    towers = eng.used_towers()
    assert towers == sorted({0 if mode in (0, 2) else 1, 0 if mode in (0, 3) else 1})
    check_grads(store, ref["grads"], towers)
    # BN running stats: the reference's calls in order
    new = {k: np.asarray(v, np.float64) for k, v in state.items() if k.endswith(("running_mean", "running_var"))}
    for call in ref["bn_stats"]:
        for bk, st in call:
            new[bk + ".running_mean"], new[bk + ".running_var"] = O.bn_running_update(
                new[bk + ".running_mean"], new[bk + ".running_var"], st)
    for k, v in new.items():
        assert rel(host(store.buffers[k]), v) < 1e-5, k
    # Adam: unused tower bit-unchanged, used towers = torch.optim.Adam(lr) on our gradients
    pre = store.student.clone()
    ours = {k: host(store.grad_of(k)) for k in store.live_keys}
    eng.adam()
    for t in (0, 1):
        o, n = eng.ranges[t]
        if t not in towers:
            assert torch.equal(store.student[o:o + n], pre[o:o + n])
    for k in store.live_keys:
        if k.startswith(tuple(("image_", "audio_")[t] for t in towers)):
            p_ref, _, _ = O.adam_step(host(pre[store.s_offs[k][0]:store.s_offs[k][0] + store.s_offs[k][1]]),
                                      ours[k].ravel(), 0, 0, 1, 1e-4, 0.0)
            assert rel(host(store[k]).ravel(), p_ref) < 1e-6, k


def test_simclr_mode_draw_and_lightning_api():
    from avdino.models import MultiModalSimCLRLightning
    m = MultiModalSimCLRLightning(projection_dim=32, output_dim=32, precision="32", device="cuda")
    modes = [m.model.engine.draw_mode() for _ in range(64)]
    assert set(modes) == {0, 1, 2, 3}
    b = make_simclr_batch(4, 5)
    batch = tuple(torch.from_numpy(b[k]) for k in ("img1", "spec1", "img2", "spec2"))
    opt = m.configure_optimizers()["optimizer"]
    loss = m.training_step(batch, 0, mode=2)
    opt.zero_grad()
    loss.backward()
    opt.step()
    assert np.isfinite(loss.item())
    assert m.model.arena_image.grad is not None and m.model.arena_audio.grad is not None
    loss = m.training_step(batch, 1, mode=0)        # image/image: the audio tower gets no grad
    opt.zero_grad(set_to_none=True)
    loss.backward()
    assert m.model.arena_image.grad is not None and m.model.arena_audio.grad is None
    opt.step()
    reps = torch.randn(8, 32, device="cuda", requires_grad=True)
    lv = m.nt_xent_loss(reps)
    lv.backward()
    ref, dref = O.nt_xent_loss(reps.detach().double().cpu().numpy())
    assert abs(lv.item() - ref) < 1e-5 and rel(host(reps.grad), dref) < 1e-5


# ------------------------------------------------------------------ world 2 (gloo on cuda:0)
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _entry(fn, r, world, port, q):
    try:
        for p_ in (REPO, PKG):
            if p_ not in sys.path:
                sys.path.insert(0, p_)
        import torch.distributed as dist
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=r, world_size=world)
        out = fn(r, world)
        dist.destroy_process_group()
        q.put((r, out))
    except Exception:
        import traceback
        q.put(traceback.format_exc())


def _run2(fn):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_entry, args=(fn, r, 2, port, q)) for r in range(2)]
    for p_ in procs:
        p_.start()
    res = [q.get(timeout=240) for _ in procs]
    for p_ in procs:
        p_.join(timeout=60)
    errs = [x for x in res if isinstance(x, str)]
    assert not errs, errs[0]
    return sorted(res, key=lambda x: x[0])


def _simclr_rank(r, world, mode=2):
    from avdino import dist as AD
    store, eng, _ = build()
    eng.grad_hook = AD.grad_allreduce_hook()
    batch = make_simclr_batch(2 * B, BSEED)        # global batch 2B; rank r owns rows r*B..
    mine = {k: torch.from_numpy(v[r * B:(r + 1) * B]).cuda() for k, v in batch.items()}
    loss = eng.forward(mine, mode)
    eng.backward()
    eng.grad_hook(store.grad)
    return loss.item(), {k: host(store.grad_of(k)) for k in store.live_keys}


def test_simclr_global_negatives_world2_matches_oracle():
    res = _run2(_simclr_rank)
    state = make_state(OS.simclr_spec(D, P), PSEED)
    ref = O.simclr_step(state, make_simclr_batch(2 * B, BSEED), 2, shards=2)
    # mean of the ranks' local-mean losses = the global-batch loss
    assert abs((res[0][1][0] + res[1][1][0]) / 2 - ref["loss"]) < 3e-5
    for _, (_, grads) in res:
        errs = [rel(grads[k], ref["grads"][k]) for k in ref["grads"]
                if np.linalg.norm(ref["grads"][k]) > 1e-4]
        assert max(errs) < 1e-3 and np.median(errs) < 1e-4, (max(errs), np.median(errs))


def _infonce_rank(r, world):
    from avdino import contrastive
    from avdino.engine import Workspace
    g = np.random.default_rng(77)
    zi, za = g.normal(size=(2, 2 * B, 32)).astype(np.float32)
    ws = Workspace("cuda")
    ti, ta = torch.from_numpy(zi[r * B:(r + 1) * B]).cuda(), torch.from_numpy(za[r * B:(r + 1) * B]).cuda()
    dzi, dza = torch.empty(B * 32, device="cuda"), torch.empty(B * 32, device="cuda")
    parts = torch.empty(2 * B, device="cuda")
    scale = contrastive.infonce(ws, ti.view(-1), ta.view(-1), B, 32, dzi, dza, parts)
    return host(parts).sum() * scale, host(dzi).reshape(B, 32), host(dza).reshape(B, 32)


def test_infonce_global_negatives_world2_matches_oracle():
    """InfoNCE (config 3) with all-gathered negatives: the mean of the ranks' losses and the
    per-rank gradients (x 1/world, DDP averaging) equal the single-device InfoNCE over the
    global batch."""
    res = _run2(_infonce_rank)
    g = np.random.default_rng(77)
    zi, za = g.normal(size=(2, 2 * B, 32))
    lref, diref, daref = O.infonce_loss(zi, za)
    assert abs((res[0][1][0] + res[1][1][0]) / 2 - lref) < 1e-5
    di = np.concatenate([res[0][1][1], res[1][1][1]]) / 2
    da = np.concatenate([res[0][1][2], res[1][1][2]]) / 2
    assert rel(di, diref) < 1e-5 and rel(da, daref) < 1e-5
