"""A full multimodal-DINO data-parallel step at world 2 (SURVEY 8(e) "parity
for N ranks"): two processes, gloo, both on cuda:0 (the 1-GPU rehearsal of the 8-GPU RCCL run),
each owning half the global batch, against the DDP-simulating oracle
(oracle/numpy_oracle.multimodal_step_ddp): per-rank BatchNorm statistics and centre, rank-0
buffers broadcast before the forward, gradients averaged by one all-reduce of the flat arena,
and -- InfoNCE, BASELINE config 3 -- negatives all-gathered across ranks.  Also the trainer's
strategy="ddp" wiring (avdino.trainer.Trainer) drives the same step.

Tolerances as tests/test_gpu_step.py (fp32 kernels vs float64), except the audio-encoder
gradients: with 4 samples per rank-local BatchNorm group, fp32 rounding moves max-pool argmax
near-ties, so they get 2.5x the reference's own fp32-vs-float64 error (1.5x single-device)."""
import os
import socket
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

from oracle import numpy_oracle as O  # noqa: E402
from oracle import spec as OS  # noqa: E402
from oracle.params import make_multimodal_batch, make_state  # noqa: E402

from tests.test_gpu_step import AUDIO_TOL, HP, rel, zero_grad_keys  # noqa: E402

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "multimodal-ssl-avmnist_amd")
E, D, P, B, G, L = 32, 32, 16, 4, 2, 2
PSEED, BSEED = 501, 5001


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _entry(fn, args, r, world, port, q):
    try:
        for p_ in (REPO, PKG):
            if p_ not in sys.path:
                sys.path.insert(0, p_)
        import torch.distributed as dist
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=r, world_size=world)
        out = fn(r, world, *args)
        dist.destroy_process_group()
        q.put((r, out))
    except Exception:
        import traceback
        q.put(traceback.format_exc())


def _run2(fn, *args):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_entry, args=(fn, args, r, 2, port, q)) for r in range(2)]
    for p_ in procs:
        p_.start()
    res = [q.get(timeout=240) for _ in procs]
    for p_ in procs:
        p_.join(timeout=60)
    errs = [x for x in res if isinstance(x, str)]
    assert not errs, errs[0]
    return [x[1] for x in sorted(res, key=lambda x: x[0])]


def _host(t):
    return t.detach().float().cpu().numpy().astype(np.float64)


def _engine_rank(r, world, mode):
    from avdino import dist as AD
    from avdino.engine import Hyper, MultiCentralEngine
    from avdino.params import ParamStore
    from avdino.spec import multimodal_dino_sd
    store = ParamStore(multimodal_dino_sd(mode, E, D, P), "cuda")
    # rank 1 starts from different parameters / buffers: DDP's initial broadcast and the
    # per-forward buffer broadcast must make it rank 0's
    st = make_state(OS.multimodal_dino_spec(mode, E, D, P), PSEED + 17 * r)
    store.load_state_dict({k: torch.from_numpy(np.array(v)) for k, v in st.items()})
    AD.broadcast_parameters(store)
    hp = Hyper(lr=HP["lr"], weight_decay=HP["wd"], momentum=HP["momentum"],
               center_momentum=HP["center_momentum"], student_temperature=HP["tau_s"],
               teacher_temperature=HP["tau_t"], dropout=0.0, fusion_dropout=0.0)
    eng = MultiCentralEngine(store, mode, E, D, P, hp, act_dtype=torch.float32,
                             grad_hook=AD.grad_allreduce_hook(), buffer_hook=AD.broadcast_buffers,
                             negatives="global")
    batch = make_multimodal_batch(2 * B, G, L, BSEED)
    mine = {k: torch.from_numpy(v[r * B:(r + 1) * B]).cuda() for k, v in batch.items()}
    eng.buffer_hook(store)
    loss = eng.forward(mine)
    eng.update_center()
    eng.backward()
    eng.grad_hook(store.grad)
    store.flush_nbt()
    return (loss.item(), {k: _host(store.grad_of(k)) for k in store.live_keys},
            _host(store["center"]),
            {k: _host(store.buffers[k]) for k in store.buffers if k.endswith(("running_mean", "running_var"))})


@pytest.mark.parametrize("mode", ["mse", "infonce", "semi_supervised", "default"])
def test_dino_step_world2_matches_ddp_oracle(mode):
    res = _run2(_engine_rank, mode)
    state = make_state(OS.multimodal_dino_spec(mode, E, D, P), PSEED)
    outs, grads = O.multimodal_step_ddp(state, make_multimodal_batch(2 * B, G, L, BSEED), mode, HP, 2)
    zero = zero_grad_keys(grads)
    for r, (loss, g, center, running) in enumerate(res):
        assert abs(loss - outs[r]["loss"]) < 3e-5, (r, loss, outs[r]["loss"])
        assert rel(center, outs[r]["center_after"]) < 1e-5
        for k, v in running.items():
            assert rel(v, outs[r]["state"][k]) < 1e-5, (r, k)
        errs = {k: rel(g[k], grads[k]) for k in g if k not in zero}
        for k, e in errs.items():
            bound = AUDIO_TOL * 2.5 / 1.5 if k.startswith("student.audio_encoder") else 1e-3
            assert e < bound, (k, e, bound)
        assert np.median(list(errs.values())) < 1e-4
    # the two ranks hold the same averaged gradient
    for k in res[0][1]:
        assert np.array_equal(res[0][1][k], res[1][1][k]), k


def _trainer_rank(r, world):
    """strategy="ddp" through the Lightning-shaped loop: one batch per rank per step."""
    from avdino.models import CentralMultiModalEncoder, MultiModalDINOWithMSELightning
    from avdino.trainer import Trainer
    m = MultiModalDINOWithMSELightning(encoder_class=CentralMultiModalEncoder, encoder_output_dim=E,
                                       output_dim=D, projection_dim=P, dropout=0.0, precision="32",
                                       device="cuda", learning_rate=HP["lr"], weight_decay=HP["wd"],
                                       momentum=HP["momentum"], center_momentum=HP["center_momentum"],
                                       student_temperature=HP["tau_s"], teacher_temperature=HP["tau_t"])
    m.model.hp.fusion_dropout = 0.0
    st = make_state(OS.multimodal_dino_spec("mse", E, D, P), PSEED + 17 * r)
    m.load_state_dict({"model." + k: torch.from_numpy(np.array(v)) for k, v in st.items()})
    batches = []
    for i in range(2):
        b = make_multimodal_batch(2 * B, G, L, BSEED + i)
        t = {k: torch.from_numpy(v[r * B:(r + 1) * B]).cuda() for k, v in b.items()}
        batches.append((t["image"], t["audio"], t["label"], (t["g_img"], t["g_aud"], t["l_img"], t["l_aud"])))
    Trainer(max_epochs=1, strategy="ddp").fit(m, batches)
    return _host(m.model.store.student), _host(m.model.store.teacher)


def test_trainer_ddp_world2_keeps_replicas_identical():
    (s0, t0), (s1, t1) = _run2(_trainer_rank)
    assert np.array_equal(s0, s1) and np.array_equal(t0, t1)
