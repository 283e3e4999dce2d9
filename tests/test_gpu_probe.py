"""Epoch-end linear probe parity: avdino.probe.LinearProbe (fp32) vs the
float64 oracle's linear_probe, which tests/test_oracle_golden.py pins to the reference's
DownstreamClassifier run on the same dims/seeds (tests/golden/probe_*.npz).

Tolerances: per-batch training losses and eval loss 3e-5 abs; accuracy exact; eval logits
1e-4 rel-L2; final classifier parameters max(1e-5, 3x the reference's fp32-vs-float64 error)
rel-L2 (three AdamW steps);
the encoder copy's running statistics 1e-5."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

from oracle import numpy_oracle as O  # noqa: E402
from oracle import spec as OS  # noqa: E402
from oracle.params import make_multimodal_batch, make_state  # noqa: E402
from tests import golden_util as gu  # noqa: E402

CASES = {"probe_multi_central": ("multi_central", 32, 32, 16, 6, 3, 2, 111, 1011),
         "probe_image_simple": ("image_simple", 0, 64, 32, 6, 3, 2, 112, 1012)}
LR = 1e-3


def rel(a, b):
    a = np.asarray(a, np.float64).ravel()
    b = np.asarray(b, np.float64).ravel()
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30)


def host(t):
    return t.detach().float().cpu().numpy().astype(np.float64)


@pytest.mark.parametrize("case", list(CASES))
def test_linear_probe_matches_oracle(case):
    from avdino.params import ParamStore
    from avdino.probe import LinearProbe
    from avdino.spec import multimodal_dino_sd, unimodal_dino_sd
    kind, E, D, P, B, nt, nv, pseed, bseed = CASES[case]
    if kind == "multi_central":
        sd, ospec = multimodal_dino_sd("default", E, D, P), OS.multimodal_dino_spec("default", E, D, P)
    else:
        sd, ospec = unimodal_dino_sd(kind, D, P), OS.unimodal_dino_spec(kind, D, P)
    state = make_state(ospec, pseed)
    src = ParamStore(sd, "cuda")
    src.load_state_dict({k: torch.from_numpy(np.array(v)) for k, v in state.items()})
    cls = make_state(OS.classifier_spec(D), pseed + 1)
    probe = LinearProbe(src, kind, D, E, lr=LR, fusion_dropout=0.0,
                        classifier_state={k: torch.from_numpy(v) for k, v in cls.items()})
    train = [make_multimodal_batch(B, 1, 0, bseed + i) for i in range(nt)]
    valid = [make_multimodal_batch(B, 1, 0, bseed + 1000 + i) for i in range(nv)]

    def dev(b):
        return (torch.from_numpy(b["image"]).cuda(), torch.from_numpy(b["audio"]).cuda(),
                torch.from_numpy(b["label"]).cuda())

    out = probe.run_epoch([dev(b) for b in train], [dev(b) for b in valid])
    ref = O.linear_probe(state, kind, train, valid, cls, LR)
    assert abs(ref["eval_loss"] - float(gu.load(case + "_f64")["eval_loss"])) < 1e-8
    np.testing.assert_allclose(host(out["train_losses"]), ref["train_losses"], atol=3e-5, rtol=0)
    assert abs(out["val_loss"] - ref["val_loss"]) < 3e-5
    assert abs(out["eval_loss"] - ref["eval_loss"]) < 3e-5
    assert out["mlp_acc"] == ref["mlp_acc"]
    assert rel(host(out["logits"]), ref["logits"]) < 1e-4
    f32, f64 = gu.load(case), gu.load(case + "_f64")
    for k, v in ref["classifier"].items():
        # AdamW's first steps are ~lr*sign(g): entries with |g| at rounding level flip sign
        # between fp32 and float64 -- the reference's own fp32 run misses by up to 1.8e-5
        bound = max(1e-5, 3 * gu.rel_err(f32["cls/" + k], f64["cls/" + k]))
        assert rel(host(probe.cls[k]), v) < bound, (k, rel(host(probe.cls[k]), v), bound)
    for k, v in ref["running"].items():
        assert rel(host(probe.store[k]), v) < 1e-5, k
    # the trained model is untouched (the probe works on a deep copy)
    assert rel(host(src["student.fusion.0.weight" if kind == "multi_central" else
                        "student.projection.0.weight"]),
               state["student.fusion.0.weight" if kind == "multi_central" else
                     "student.projection.0.weight"]) == 0


def test_probe_graph_replay_equals_eager():
    """The probe's training batches replayed as hipGraphs (fixed input buffers, device step
    count / bias corrections / dropout offset) equal the eager batches bit for bit, with the
    fusion dropout on and a ragged last batch (run eagerly)."""
    from avdino.params import ParamStore
    from avdino.probe import LinearProbe
    from avdino.spec import multimodal_dino_sd
    kind, E, D, P = "multi_central", 32, 32, 16
    state = make_state(OS.multimodal_dino_spec("default", E, D, P), 211)
    cls = make_state(OS.classifier_spec(D), 212)
    batches = [make_multimodal_batch(8 if i < 6 else 5, 1, 0, 2100 + i) for i in range(7)]

    def dev(b):
        return (torch.from_numpy(b["image"]).cuda(), torch.from_numpy(b["audio"]).cuda(),
                torch.from_numpy(b["label"]).cuda())

    outs = []
    for use_graph in (False, True):
        src = ParamStore(multimodal_dino_sd("default", E, D, P), "cuda")
        src.load_state_dict({k: torch.from_numpy(np.array(v)) for k, v in state.items()})
        probe = LinearProbe(src, kind, D, E, lr=LR, fusion_dropout=0.3, use_graph=use_graph,
                            classifier_state={k: torch.from_numpy(v) for k, v in cls.items()})
        out = probe.run_epoch([dev(b) for b in batches], [dev(b) for b in batches[:2]])
        outs.append((out, probe.cls.student.clone(), probe.store.buf_arena.clone()))
        if use_graph:
            assert probe.graph.captures >= 1
    (o0, c0, b0), (o1, c1, b1) = outs
    assert torch.equal(o0["train_losses"], o1["train_losses"])
    assert o0["eval_loss"] == o1["eval_loss"] and o0["mlp_acc"] == o1["mlp_acc"]
    assert torch.equal(c0, c1) and torch.equal(b0, b1)
