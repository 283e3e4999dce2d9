"""training_structures.pretrain_dino (dino_train.py:104-186; BASELINE config 1's path) on the
device against the float64 oracle, which is pinned to the reference's own pretrain_dino run
(tests/golden/pretrain_image_simple*.npz, tests/test_oracle_golden.py):
  * avdino.training_structures.pretrain_dino -- the reference loop over the nn.Module model
    (autograd through the engine, FlatAdam in AdamW mode, EMA after the step);
  * UniModalEngine(step_order="pretrain").step -- the same step fused (bench --workload uni),
    eager and graph-replayed.
Tolerances (fp32 engine): per-step loss 1e-4 over 4 steps (the loss-curve bound of north_star),
final parameters 2e-2 rel (AdamW moves near-zero-gradient entries by +-lr)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

from oracle import numpy_oracle as O  # noqa: E402
from oracle import spec as S  # noqa: E402
from oracle.params import make_multimodal_batch, make_state  # noqa: E402
from tests import golden_util as gu  # noqa: E402

HP = dict(momentum=0.996, center_momentum=0.9)


def _setup():
    fx = gu.load("pretrain_image_simple_f64")
    D, P, B, epochs, nb, pseed, bseed = [int(x) for x in fx["meta_dims"]]
    state = make_state(S.unimodal_dino_spec("image", D, P), pseed)
    batches = [make_multimodal_batch(B, 2, 0, bseed + i, with_originals=False) for i in range(nb)]
    ref = O.pretrain_dino(state, batches, epochs, float(fx["meta_lr"]), HP)
    return fx, (D, P, B, epochs, nb), state, batches, ref


def test_pretrain_dino_loop_matches_oracle(tmp_path):
    from avdino.models import ImageEncoder, UniModalDINO
    from avdino.training_structures import pretrain_dino, unimodal_dino_loss
    fx, (D, P, B, epochs, nb), state, batches, ref = _setup()
    m = UniModalDINO(encoder_class=ImageEncoder, output_dim=D, projection_dim=P, dropout=0.0,
                     precision="32", device="cuda")
    m.load_state_dict({k: torch.from_numpy(np.array(v)) for k, v in state.items()})
    loader = [tuple(torch.from_numpy(b[k]).cuda() for k in ("g_img", "g_aud", "l_img", "l_aud"))
              for b in batches]
    pretrain_dino(m, loader, unimodal_dino_loss, num_epochs=epochs, learning_rate=float(fx["meta_lr"]),
                  save_path=str(tmp_path / "p" / "m.pt"), log_path=str(tmp_path / "p" / "log.csv"))
    steps = torch.cat(m.step_losses).cpu().numpy()
    np.testing.assert_allclose(steps, ref["step_losses"], atol=1e-4, rtol=0)
    np.testing.assert_allclose(m.epoch_losses, ref["epoch_losses"], atol=1e-4, rtol=0)
    for k, v in ref["state"].items():
        if k.endswith("num_batches_tracked"):
            assert int(m.store[k].item()) == int(v), k
        elif np.linalg.norm(v) > 0:
            e = gu.rel_err(m.store[k].detach().cpu().numpy(), v)
            assert e < 2e-2, (k, e)


@pytest.mark.parametrize("graph", [False, True])
def test_engine_pretrain_order_matches_oracle(graph):
    from avdino.engine import Hyper, UniModalEngine
    from avdino.params import ParamStore
    from avdino.spec import unimodal_dino_sd
    fx, (D, P, B, epochs, nb), state, batches, ref = _setup()
    store = ParamStore(unimodal_dino_sd("image_simple", D, P), "cuda")
    store.load_state_dict({k: torch.from_numpy(np.array(v)) for k, v in state.items()})
    eng = UniModalEngine(store, "image_simple", D, P, Hyper(lr=float(fx["meta_lr"]), dropout=0.0),
                         act_dtype=torch.float32, step_order="pretrain")
    eng.use_graph = graph
    eng.graph.warmup = 1
    dev = [{k: torch.from_numpy(v).cuda() for k, v in b.items()} for b in batches]
    losses = [eng.step(dev[i % nb]).item() for i in range(epochs * nb)]
    np.testing.assert_allclose(losses, ref["step_losses"], atol=1e-4, rtol=0)
    for k in store.t_offs:
        e = gu.rel_err(store[k].detach().cpu().numpy(), ref["state"][k])
        assert e < 2e-2, (k, e)
    assert gu.rel_err(store["center"].cpu().numpy(), ref["state"]["center"]) < 1e-4
