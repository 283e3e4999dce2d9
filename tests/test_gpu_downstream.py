"""Downstream evaluation on the device (avdino.downstream) against the
reference's own results: the golden fixtures downstream_* were produced by running the
reference's train_knn_classifier / train_downstream / compute_classification_metrics
(training_structures/dino_train.py:47-102, 188-369) on CPU (tests/golden/gen_golden.py), and
the float64 oracle restating them is pinned to those fixtures (tests/test_oracle_golden.py).

Tolerances (fp32 engine): features rel-L2 1e-5; kNN predictions and neighbours identical;
per-epoch losses 1e-4 abs, accuracies and test predictions identical; classifier 1e-4.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

from oracle import numpy_oracle as O  # noqa: E402
from oracle import spec as S  # noqa: E402
from oracle.params import make_multimodal_batch, make_state  # noqa: E402
from tests import golden_util as gu  # noqa: E402


def grel(a, b):
    a = np.asarray(a, np.float64).ravel()
    b = np.asarray(b, np.float64).ravel()
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30)


def _model(kind, E, D, P, pseed):
    from avdino.models import (CentralMultiModalEncoder, ImageEncoder, MultiModalDINO,
                               SpectrogramEncoder, UniModalDINO)
    if kind == "multi_central":
        m = MultiModalDINO(encoder_class=CentralMultiModalEncoder, output_dim=D, encoder_output_dim=E,
                           projection_dim=P, dropout=0.0, precision="32", device="cuda")
        m.hp.fusion_dropout = 0.0
        spec = S.multimodal_dino_spec("default", E, D, P)
    else:
        enc = {"image_simple": ImageEncoder, "spectrogram_simple": SpectrogramEncoder}[kind]
        m = UniModalDINO(encoder_class=enc, output_dim=D, projection_dim=P, dropout=0.0,
                         precision="32", device="cuda")
        spec = S.unimodal_dino_spec(kind, D, P)
    state = make_state(spec, pseed)
    m.load_state_dict({k: torch.from_numpy(np.array(v)) for k, v in state.items()})
    return m, state


def _loader(B, n, seed):
    out = []
    for i in range(n):
        b = make_multimodal_batch(B, 1, 0, seed + i)
        out.append(tuple(torch.from_numpy(b[k]).cuda() for k in ("image", "audio", "label")))
    return out


@pytest.mark.parametrize("case", ["downstream_multi_central", "downstream_image_simple"])
def test_downstream_matches_reference(case, tmp_path):
    from avdino import downstream as DS
    fx = gu.load(case)
    fx64 = gu.load(case + "_f64")
    E, D, P, B, nt, nv, ne, epochs, pseed, bseed = [int(x) for x in fx["meta_dims"]]
    kind, lr = str(fx["meta_kind"]), float(fx["meta_lr"])
    model, state = _model(kind, E, D, P, pseed)
    tr, va, te = _loader(B, nt, bseed), _loader(B, nv, bseed + 1000), _loader(B, ne, bseed + 2000)
    # frozen eval-mode features (FeatureExtractor) vs the oracle (pinned to the fixture)
    fe = DS.FeatureExtractor(model)
    trf, trl = DS.feature_extraction_loop("cuda", fe, tr)
    tef, tel = DS.feature_extraction_loop("cuda", fe, te)
    pm = O._ProbeModel(state, kind, make_state(S.classifier_spec(D), pseed + 1))
    ref_tr = np.concatenate([pm.features(make_multimodal_batch(B, 1, 0, bseed + i), True) for i in range(nt)])
    assert grel(trf.cpu().numpy(), ref_tr) < 1e-5
    # kNN: the reference's sklearn predictions / neighbours, exactly
    knn, acc = DS.train_knn_classifier(model, tr, te, n_neighbors=5)
    np.testing.assert_array_equal(knn.predict(tef).cpu().numpy(), fx64["knn_pred"])
    # neighbour order: identical except where two neighbours are equidistant to f32 resolution
    nb, rnb = knn.kneighbors(tef).cpu().numpy(), fx64["knn_nbr"]
    qf, xf = np.asarray(fx64["feat_test"], np.float64), np.asarray(fx64["feat_train"], np.float64)
    d64 = ((qf[:, None, :] - xf[None]) ** 2).sum(-1)
    for i in np.nonzero((nb != rnb).any(1))[0]:
        assert set(nb[i]) == set(rnb[i]), i
        dd = np.take(d64[i], nb[i])
        j = np.nonzero(nb[i] != rnb[i])[0]
        assert np.ptp(dd[j]) <= 1e-5 * dd[j].max(), (i, dd)
    assert acc == pytest.approx(float(fx64["knn_acc"]))
    # the MLP probe: 3 epochs AdamW + cosine LR, best-val checkpoint, test evaluation
    cls = {k: torch.from_numpy(np.array(v)) for k, v in make_state(S.classifier_spec(D), pseed + 1).items()}
    clf = DS.train_downstream(model, tr, va, te, num_epochs=epochs, learning_rate=lr,
                              save_path=str(tmp_path / "d" / "m.pt"),
                              train_log_path=str(tmp_path / "d" / "train.csv"),
                              test_log_path=str(tmp_path / "d" / "test.csv"), classifier_state=cls)
    hist = np.array([[h["train_loss"], h["val_loss"], h["val_accuracy"]] for h in clf.history])
    np.testing.assert_allclose(hist[:, :2], fx64["history"][:, :2], atol=1e-4, rtol=0)
    np.testing.assert_array_equal(hist[:, 2], fx64["history"][:, 2])
    met = DS.compute_classification_metrics(clf, te)
    np.testing.assert_array_equal(met["predictions"], fx64["test_preds"])
    assert met["accuracy"] == pytest.approx(float(fx64["test_acc"]))
    np.testing.assert_array_equal(met["confusion_matrix"], fx64["confusion_matrix"])
    for k, v in clf.classifier_state_dict().items():
        assert gu.compare(fx64, "cls/" + k, v.cpu().numpy(), rel=1e-4)[0], k
    # the trained model itself was never touched (deep copy)
    for k, v in state.items():
        assert np.allclose(model.store[k].detach().cpu().numpy(), v), k


def test_knn_device_matches_oracle_large():
    """KNeighborsClassifier on the device at AVMNIST scale (55,000 train features of width 256,
    5,000 queries in two GEMM chunks) vs the float64 restatement: identical neighbours and
    predictions on every row whose 5th/6th-nearest distance gap is above f32 resolution."""
    from avdino.downstream import KNeighborsClassifier
    g = torch.Generator(device="cuda").manual_seed(9)
    N, M, Dm, C = 55000, 5000, 256, 10
    X = torch.randn(N, Dm, generator=g, device="cuda")
    Q = torch.randn(M, Dm, generator=g, device="cuda")
    y = torch.randint(0, C, (N,), generator=g, device="cuda")
    knn = KNeighborsClassifier(5, query_chunk=4096).fit(X, y)
    pred = knn.predict(Q)
    nbr = knn.kneighbors(Q)
    Xd, Qd = X.double(), Q.double()
    d = (Qd * Qd).sum(1, keepdim=True) - 2 * Qd @ Xd.T + (Xd * Xd).sum(1)[None]
    top = d.topk(6, dim=1, largest=False)
    gap = (top.values[:, 5] - top.values[:, 4]) / top.values[:, 4].abs()
    ok = gap > 1e-5
    assert ok.float().mean() > 0.98
    ref_nbr = top.indices[:, :5]
    assert torch.equal(nbr[ok], ref_nbr[ok])
    votes = torch.zeros(M, C, dtype=torch.int64, device="cuda").scatter_add_(1, y[ref_nbr], torch.ones_like(ref_nbr))
    ref_pred = votes.argmax(1)       # first maximum = smallest class
    assert torch.equal(pred[ok], ref_pred[ok])
    assert abs(knn.score(Q, ref_pred) - 1.0) < 0.02
