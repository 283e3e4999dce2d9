"""Device data path on the GPU: avd_augment_views against the numpy
restatement (oracle/augment.py) -- bit-exact for records without noise, |diff| <= 1e-5 with
noise (device logf/cosf vs numpy) -- and the HBM-resident AVMNIST loader feeding a training
step through the C ABI."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from avdino import augment as A  # noqa: E402
from avdino import ops  # noqa: E402
from oracle import augment as OA  # noqa: E402

from .test_augment_data import _fake_avmnist  # noqa: E402


def _records(chain, B, V, H, W, seed):
    aug = A.ViewAugmenter.__new__(A.ViewAugmenter)
    aug.rng, aug.H, aug.W = np.random.default_rng(seed), H, W
    return A.ViewAugmenter.records(aug, chain, B, V)


@pytest.mark.parametrize("view,mod", [("global", "image"), ("local", "image"),
                                      ("global", "audio"), ("local", "audio")])
@pytest.mark.parametrize("order", [0, 1])
def test_augment_kernel_matches_oracle(view, mod, order):
    H = W = 28 if mod == "image" else 112
    N, B, V = 11, 5, 3
    rng = np.random.default_rng(4)
    src = rng.integers(0, 256, (N, H * W), dtype=np.uint8)
    idx = rng.integers(0, N, B)
    lut = OA.normalise_lut(mod)
    rec, gm = _records(A.default_chains()[view][mod], B, V, H, W, 9)
    seed = 0xDEADBEEF12345
    out = torch.empty((B, V, H, W) if order == 0 else (V, B, H, W), device="cuda")
    ops.augment_views(torch.from_numpy(src).cuda(), torch.from_numpy(idx).cuda(),
                      torch.from_numpy(lut).cuda(), torch.from_numpy(rec).cuda(),
                      None if gm is None else torch.from_numpy(gm.view(np.int32)).cuda(),
                      4, seed, V, H, W, out, order)
    got = out.cpu().numpy()
    ref = OA.augment_views(src, idx, lut, rec, gm, V, H, W, seed, order)
    noisy = (rec[:, 21] != 0).reshape(B, V)
    if order == 1:
        noisy = noisy.T
    np.testing.assert_array_equal(got[~noisy], ref[~noisy])
    np.testing.assert_allclose(got[noisy], ref[noisy], rtol=0, atol=1e-5)
    assert np.isfinite(got).all()


def test_augment_identity_is_the_normalised_row():
    rng = np.random.default_rng(5)
    src = torch.from_numpy(rng.integers(0, 256, (7, 12544), dtype=np.uint8)).cuda()
    lut = torch.from_numpy(OA.normalise_lut("audio")).cuda()
    aug = A.ViewAugmenter(src, lut, 112, 112, seed=1)
    out = aug.identity([6, 0, 3])
    ref = lut.cpu().numpy()[src.cpu().numpy()[[6, 0, 3]]].reshape(3, 1, 112, 112)
    np.testing.assert_array_equal(out.cpu().numpy(), ref)
    with pytest.raises(IndexError):
        aug.identity([7])


def test_loader_batches_feed_a_training_step(tmp_path):
    from avdino.data import AVMNISTDinoLoader
    from avdino.engine import Hyper, MultiCentralEngine
    from avdino.params import ParamStore
    from avdino.spec import multimodal_dino_sd
    root = _fake_avmnist(tmp_path, n=40)
    loader = AVMNISTDinoLoader(root, batch_size=8, train_size=36, val_size=4, seed=3,
                               multimodal_mode="mse")
    assert len(loader.train_idx) == 36 and len(loader) == 5
    batches = list(loader)
    assert len(batches) == 5
    img, aud, lab, (gi, ga, li, la) = batches[0]
    assert img.shape == (8, 1, 28, 28) and aud.shape == (8, 1, 112, 112) and lab.shape == (8,)
    assert gi.shape == (8, 2, 1, 28, 28) and ga.shape == (8, 2, 1, 112, 112)
    assert li.shape == (8, 4, 1, 28, 28) and la.shape == (8, 4, 1, 112, 112)
    assert img.min() >= 0 and img.max() <= 1
    E, D, P = 32, 32, 16
    store = ParamStore(multimodal_dino_sd("mse", E, D, P), "cuda:0")
    eng = MultiCentralEngine(store, "mse", E, D, P, Hyper(dropout=0.0, fusion_dropout=0.0))
    batch = dict(image=img, audio=aud, label=lab, g_img=gi, g_aud=ga, l_img=li, l_aud=la)
    loss = eng.step(batch).item()
    assert np.isfinite(loss)
