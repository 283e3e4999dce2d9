"""The Lightning-shaped boundary: the model classes are
nn.Modules whose ``training_step`` returns a differentiable loss, ``loss.backward()`` runs the
engine's backward into the arena Parameters' ``.grad`` and ``configure_optimizers()``'s
optimizer steps them -- driven here exactly as Lightning's automatic optimisation does
(training_step -> zero_grad -> backward -> optimizer.step; run_dino.py:356-373,
models/dino.py:856-876, 953-962), against the float64 oracle.

Tolerances as tests/test_gpu_step.py (fp32 kernels vs float64 truth).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

from oracle import numpy_oracle as O  # noqa: E402
from oracle import spec as OS  # noqa: E402
from oracle.params import make_multimodal_batch, make_state  # noqa: E402

from tests.test_gpu_step import HP, check_grads, host, rel, zero_grad_keys  # noqa: E402

E, D, P, B, G, L = 32, 32, 16, 4, 2, 4


def make_module(mode, pseed, precision="32"):
    from avdino.models import MULTIMODAL_WRAPPERS, CentralMultiModalEncoder
    m = MULTIMODAL_WRAPPERS[mode](encoder_class=CentralMultiModalEncoder, encoder_output_dim=E,
                                  output_dim=D, projection_dim=P, dropout=0.0, precision=precision,
                                  device="cuda", learning_rate=HP["lr"], weight_decay=HP["wd"],
                                  momentum=HP["momentum"], center_momentum=HP["center_momentum"],
                                  student_temperature=HP["tau_s"], teacher_temperature=HP["tau_t"])
    m.model.hp.fusion_dropout = 0.0          # hard-coded 0.3 in the reference; 0 for parity
    state = make_state(OS.multimodal_dino_spec(mode, E, D, P), pseed)
    # the reference checkpoint's keys: "model." + MultiModalDINO* state-dict keys
    m.load_state_dict({"model." + k: torch.from_numpy(np.array(v)) for k, v in state.items()})
    return m, state


def as_batch(b, mode):
    t = {k: torch.from_numpy(v).cuda() for k, v in b.items()}
    views = (t["g_img"], t["g_aud"], t["l_img"], t["l_aud"])
    if mode == "default":
        return views
    return (t["image"], t["audio"], t["label"], views)


def lightning_step(m, opt, batch, i=0):
    """Lightning 2.x automatic optimisation: optimizer.step(closure), closure = training_step
    -> zero_grad -> backward."""
    out = {}

    def closure():
        loss = m.training_step(batch, i)
        opt.zero_grad()
        loss.backward()
        out["loss"] = loss
        return loss

    opt.step(closure)
    return out["loss"]


@pytest.mark.parametrize("mode", ["mse", "default", "infonce", "semi_supervised"])
def test_lightning_loop_matches_oracle(mode):
    m, state = make_module(mode, 201)
    assert isinstance(m, torch.nn.Module) and isinstance(m.model, torch.nn.Module)
    batch = make_multimodal_batch(B, G, L, 2001)
    ref = O.multimodal_step(state, batch, mode, HP)
    conf = m.configure_optimizers()
    opt, sched = conf["optimizer"], conf["lr_scheduler"]["scheduler"]
    assert isinstance(opt, torch.optim.Optimizer)
    st = m.model.store
    pre = {k: host(st[k]) for k in st.live_keys}
    loss = lightning_step(m, opt, as_batch(batch, mode))
    assert loss.requires_grad is False or loss.grad_fn is not None
    assert abs(loss.item() - ref["loss"]) < 3e-5, (loss.item(), ref["loss"])
    assert rel(host(st["center"]), ref["center_after"]) < 1e-5
    # the arena Parameter's .grad is the engine's gradient arena (autograd delivered it)
    g = m.model.arena.grad
    assert g is not None and torch.equal(g, st.grad)
    zero = zero_grad_keys(ref["grads"])
    errs = {k: rel(host(st.grad_of(k)), ref["grads"][k]) for k in st.live_keys if k not in zero}
    check_grads(errs)
    for k in st.t_offs:       # EMA from the PRE-step student (update_teacher before backward)
        assert rel(host(st[k]), ref["state"][k]) < 1e-6, k
    ours = {k: host(st.grad_of(k)) for k in st.live_keys}
    post = O.adam_update_state(pre, ours, {}, 1, HP)
    for k in st.live_keys:
        assert rel(host(st[k]), post[k]) < 1e-6, k
    sched.step()
    assert opt.param_groups[0]["lr"] < HP["lr"]


@pytest.mark.parametrize("mode", ["mse", "infonce"])
def test_general_path_equals_fused_path(mode):
    """model(batch) -> the reference's loss methods -> backward gives the fused
    training_step's gradients (reference_training_step composes dino.py:1214-1238 / 1130-1154
    literally)."""
    batch = make_multimodal_batch(B, G, L, 2002)
    grads, losses = [], []
    for fused in (True, False):
        m, _ = make_module(mode, 202)
        opt = m.configure_optimizers()["optimizer"]
        b = as_batch(batch, mode)
        loss = m.training_step(b, 0) if fused else m.reference_training_step(b, 0)
        opt.zero_grad()
        loss.backward()
        grads.append(m.model.arena.grad.clone())
        losses.append(loss.item())
    assert abs(losses[0] - losses[1]) < 1e-5, losses
    assert rel(host(grads[1]), host(grads[0])) < 1e-5


def test_loss_is_a_fresh_tensor_per_step():
    """each step's loss must survive the next step (no reused workspace slot)."""
    m, _ = make_module("mse", 203)
    opt = m.configure_optimizers()["optimizer"]
    ls = []
    for i in range(3):
        ls.append(lightning_step(m, opt, as_batch(make_multimodal_batch(B, G, L, 2100 + i), "mse"), i))
    vals = [x.item() for x in ls]
    assert len(set(vals)) == 3, vals
    assert abs(np.mean(vals) - np.mean([float(v) for v in m.logged_history["train_loss"]])) < 1e-6


def test_stale_backward_raises():
    m, _ = make_module("mse", 204)
    l1 = m.training_step(as_batch(make_multimodal_batch(B, G, L, 2200), "mse"), 0)
    m.training_step(as_batch(make_multimodal_batch(B, G, L, 2201), "mse"), 1)
    with pytest.raises(RuntimeError, match="stale"):
        l1.backward()


def test_trainer_fit_equals_engine_steps(tmp_path):
    """avdino.trainer.Trainer (Lightning's loop) over 3 batches == 3 engine.step() calls from
    the same state, bit for bit; ModelCheckpoint writes a checkpoint that load_from_checkpoint
    restores."""
    from avdino.engine import Hyper, MultiCentralEngine
    from avdino.params import ParamStore
    from avdino.spec import multimodal_dino_sd
    from avdino.trainer import ModelCheckpoint, Trainer
    batches = [as_batch(make_multimodal_batch(B, G, L, 2300 + i), "mse") for i in range(3)]
    m, state = make_module("mse", 205)
    ck = ModelCheckpoint(dirpath=str(tmp_path), monitor="train_loss", mode="min")
    tr = Trainer(max_epochs=1, callbacks=[ck])
    tr.fit(m, batches)
    store = ParamStore(multimodal_dino_sd("mse", E, D, P), "cuda")
    store.load_state_dict({k: torch.from_numpy(np.array(v)) for k, v in state.items()})
    hp = Hyper(lr=HP["lr"], weight_decay=HP["wd"], momentum=HP["momentum"],
               center_momentum=HP["center_momentum"], student_temperature=HP["tau_s"],
               teacher_temperature=HP["tau_t"], dropout=0.0, fusion_dropout=0.0)
    eng = MultiCentralEngine(store, "mse", E, D, P, hp, act_dtype=torch.float32)
    losses = []
    for b in batches:
        image, audio, label, (gi, ga, li, la) = b
        losses.append(eng.step(dict(g_img=gi, g_aud=ga, l_img=li, l_aud=la, image=image,
                                    audio=audio, label=label)).item())
    assert torch.equal(store.student, m.model.store.student)
    assert torch.equal(store.teacher, m.model.store.teacher)
    assert torch.equal(store.buf_arena, m.model.store.buf_arena)
    assert abs(tr.callback_metrics["train_loss"] - np.mean(losses)) < 1e-6
    assert ck.best_model_path.endswith(".ckpt")
    from avdino.models import MultiModalDINOWithMSELightning
    m2 = MultiModalDINOWithMSELightning.load_from_checkpoint(ck.best_model_path, device="cuda",
                                                             precision="32")
    for k, v in m.state_dict().items():
        assert torch.equal(v.cpu(), m2.state_dict()[k].cpu()), k


def test_ddp_rank_hooks_single_process():
    """strategy='ddp' at world 1 installs nothing (the reference's auto strategy)."""
    from avdino.trainer import Trainer
    m, _ = make_module("mse", 206)
    tr = Trainer(max_epochs=1, strategy="ddp")
    tr.fit(m, [as_batch(make_multimodal_batch(B, G, L, 2400), "mse")])
    assert m.model.engine.grad_hook is None
