"""Host side of the data path: the AVMNIST file contract, the split, the
augmentation parameter draws and the numpy restatement of the device augmentation kernel.
No GPU: nothing here launches a kernel (tests/test_gpu_augment.py holds the device parity)."""
import numpy as np
import pytest
import torch

from avdino import augment as A
from avdino import data as D
from oracle import augment as OA


def _fake_avmnist(root, n=40, seed=0, img_dtype=np.uint8):
    """A tiny AVMNIST directory in the reference's layout (get_data.py:545-551)."""
    rng = np.random.default_rng(seed)
    (root / "image").mkdir()
    (root / "audio").mkdir()
    for split in ("train", "test"):
        np.save(root / "image" / f"{split}_data.npy",
                rng.integers(0, 256, (n, 28, 28)).astype(img_dtype))
        mm = np.memmap(root / "audio" / f"{split}_data_augmented_burst_noise.npy", mode="w+",
                       dtype=np.uint8, shape=(n, 112, 112))
        mm[:] = rng.integers(0, 256, (n, 112, 112), dtype=np.uint8)
        mm.flush()
        np.save(root / f"{split}_labels.npy", rng.integers(0, 10, n))
    return str(root) + "/"


def test_paths_and_prepare_data(tmp_path):
    p = D.avmnist_paths("/d/", "burst_noise")
    assert p["train"] == ("/d/image/train_data.npy", "/d/audio/train_data_augmented_burst_noise.npy",
                          "/d/train_labels.npy")
    with pytest.raises(FileNotFoundError):
        D.prepare_data(str(tmp_path) + "/")
    D.prepare_data(_fake_avmnist(tmp_path))


@pytest.mark.parametrize("img_dtype", [np.uint8, np.float64])
def test_arrays_normalisation_and_bytes(tmp_path, img_dtype):
    root = _fake_avmnist(tmp_path, img_dtype=img_dtype)
    arr = D.AVMNISTArrays(*D.avmnist_paths(root)["train"])
    li, la = arr.luts()
    # BaseAVMNISTDataset._process_image_audio: image/255, (audio/255 - 0)/1, float64 -> float32
    img = np.asarray(arr.image_data[3], np.float64).reshape(28, 28)
    np.testing.assert_array_equal(li[img.astype(np.uint8)], (img / 255.0).astype(np.float32))
    aud = np.asarray(arr.audio_data[5])
    np.testing.assert_array_equal(la[aud], ((aud / 255.0 - 0.0) / 1.0).astype(np.float32))
    d = arr.to_device("cpu")
    assert d["image"].dtype == torch.uint8 and d["image"].shape == (40, 784)
    assert d["audio"].shape == (40, 12544) and d["labels"].dtype == torch.int64


def test_non_byte_images_rejected(tmp_path):
    root = _fake_avmnist(tmp_path)
    np.save(tmp_path / "image" / "train_data.npy", np.full((40, 28, 28), 0.5))
    arr = D.AVMNISTArrays(*D.avmnist_paths(root)["train"])
    with pytest.raises(ValueError):
        arr.to_device("cpu")


def test_random_split_partition():
    tr, va = D.random_split_indices(60, [55, 5], torch.Generator().manual_seed(3))
    assert len(tr) == 55 and len(va) == 5
    assert sorted(np.concatenate([tr, va]).tolist()) == list(range(60))
    with pytest.raises(ValueError):
        D.random_split_indices(60, [50, 5])


def test_chain_validation_and_order():
    for ch in A.default_chains()["global"].values():
        A.validate_chain(ch)
        assert A.fixed_order(ch)          # the reference's default chains: the gather kernel
    # any Compose order is accepted (the stage-by-stage kernel runs it) ...
    A.validate_chain([("affine", {}, 1.0), ("crop", {}, 1.0)])
    assert not A.fixed_order([("gaussian_noise", {}, 1.0), ("frequency_mask", {}, 1.0)])
    # ... but a kind twice or an unknown kind is not (one record slot per transform kind)
    with pytest.raises(NotImplementedError):
        A.validate_chain([("crop", {}, 1.0), ("crop", {}, 1.0)])
    with pytest.raises(NotImplementedError):
        A.validate_chain([("elastic", {}, 1.0)])
    custom = A.custom_audio_chain({"time_mask": {"time_mask_param": 10},
                                   "gaussian_noise": {"std": 0.05}},
                                  {"time_mask": 0.5, "gaussian_noise": 0.3})
    assert [c[0] for c in custom] == ["time_mask", "gaussian_noise"]


def test_parameter_draws_follow_the_transforms():
    rng = np.random.default_rng(0)
    n = 20000
    rec, gm = A.sample_records(rng, A.default_chains()["local"]["audio"], n, 112, 112)
    flags = rec[:, 23].astype(int)
    crop = (flags & 1) > 0
    assert abs(crop.mean() - 0.7) < 0.02                      # RandomApply p=0.7
    top, left, h, w = rec[crop, 0], rec[crop, 1], rec[crop, 2], rec[crop, 3]
    assert (top >= 0).all() and (left >= 0).all() and (top + h <= 112).all() and (left + w <= 112).all()
    area = h * w / 112.0 ** 2
    assert area.min() > 0.45 and area.max() < 0.95           # scale (0.5, 0.9), rounding slack
    tw = (flags & 8) > 0
    assert rec[tw, 16].min() >= 0.7 and rec[tw, 16].max() <= 1.3
    width = rec[:, 18] - rec[:, 17]
    assert width.min() >= 0 and width.max() <= 24 and (rec[:, 18] <= 112).all()
    assert abs((rec[:, 21] > 0).mean() - 0.7) < 0.02 and set(np.unique(rec[:, 21])) <= {0.0, np.float32(0.1)}
    on = rec[:, 22] >= 0
    assert abs(on.mean() - 0.9) < 0.02
    k = int(0.6 * 784)                                         # exactly int(ratio * groups)
    bits = np.unpackbits(gm.view(np.uint8), bitorder="little").reshape(n, -1)
    assert (bits.sum(1) == k).all()
    ri, gi = A.sample_records(rng, A.default_chains()["local"]["image"], n, 28, 28)
    er = ri[:, 26] > 0
    assert abs(er.mean() - 0.3) < 0.02 and gi is None
    ea = ri[er, 26] * ri[er, 27] / 784.0
    assert ea.min() > 0.01 and ea.max() < 0.2                  # scale (0.02, 0.15)


def test_inverse_affine_matches_torchvision_formula():
    m = A._inverse_affine(np.array([90.0]), np.array([2.0]), np.array([-3.0]), np.array([2.0]))[0]
    # rotation by 90 deg, scale 2: [cos, sin; -sin, cos]/2, then the translation terms
    np.testing.assert_allclose(m, [0.0, 0.5, 1.5, -0.5, 0.0, 1.0], atol=1e-12)


def _rec(**kw):
    r = np.zeros(A.REC, np.float32)
    r[22] = -1
    for k, v in kw.items():
        r[k] = v
    return r


def test_oracle_identity_crop_and_translation():
    rng = np.random.default_rng(1)
    img = OA.normalise_lut("image")[rng.integers(0, 256, (28, 28))]
    np.testing.assert_array_equal(OA.augment_one(img, _rec(), None, 0, 0), img)
    full = _rec()
    full[0:4] = [0, 0, 28, 28]
    full[23] = 1
    np.testing.assert_array_equal(OA.augment_one(img, full, None, 0, 0), img)
    sh = _rec()
    sh[4:10] = A._inverse_affine(np.zeros(1), np.array([3.0]), np.array([-2.0]), np.ones(1))[0]
    sh[23] = 2
    out = OA.augment_one(img, sh, None, 0, 0)
    np.testing.assert_array_equal(out[:26, 3:], img[2:, :25])   # shifted right 3, up 2
    assert (out[:, :3] == 0).all() and (out[26:] == 0).all()


def test_oracle_masks_time_stretch_and_groups():
    img = np.arange(112 * 112, dtype=np.float32).reshape(112, 112) / 12544.0
    r = _rec()
    r[17:21] = [10, 20, 50, 55]
    out = OA.augment_one(img, r, None, 0, 0)
    assert (out[10:20] == 0).all() and (out[:, 50:55] == 0).all()
    np.testing.assert_array_equal(out[0, :50], img[0, :50])
    tw = _rec()
    tw[16], tw[23] = 2.0, 8
    out = OA.augment_one(img, tw, None, 0, 0)
    np.testing.assert_array_equal(out[:, :56], img[:, 0:112:2])  # t = 2c, integer: exact taps
    assert (out[:, 56:] == 0).all()                                # ceil(112/2) frames
    gm = A._group_bits(np.random.default_rng(2), 1, 784, 100)
    g = _rec()
    g[22] = 0
    out = OA.augment_one(img, g, gm, 0, 0)
    masked = (out.reshape(28, 4, 28, 4) == 0).all(axis=(1, 3))
    bit = np.unpackbits(gm.view(np.uint8), bitorder="little")[:784].reshape(28, 28) == 1
    np.testing.assert_array_equal(masked, bit)                   # img > 0 except pixel 0
    np.testing.assert_array_equal(out[~np.repeat(np.repeat(bit, 4, 0), 4, 1)],
                                  img[~np.repeat(np.repeat(bit, 4, 0), 4, 1)])


def test_oracle_noise_statistics():
    z = OA.gauss(12345, 7, np.arange(200000))
    assert abs(z.mean()) < 0.01 and abs(z.std() - 1.0) < 0.01


def _random_record(rng, chain, H, W):
    rec, gm = A.sample_records(rng, chain, 1, H, W)
    return rec[0], gm


@pytest.mark.parametrize("view", ["global", "local"])
@pytest.mark.parametrize("mod", ["image", "audio"])
def test_sequential_oracle_equals_gather_oracle_in_fixed_order(view, mod):
    """A chain in the gather kernel's order gives the same views stage by stage (Compose
    semantics) as walked backwards per output pixel: the two restatements agree bit for bit."""
    H = 28 if mod == "image" else 112
    rng = np.random.default_rng(11)
    chain = [(k, kw, 1.0 if k != "erasing" else 0.5) for k, kw, _p in A.default_chains()[view][mod]]
    kinds = A.chain_kinds(chain)
    img = OA.normalise_lut("image")[rng.integers(0, 256, (H, H))]
    for r in range(6):
        rec, gm = _random_record(rng, chain, H, H)
        if gm is not None:
            rec[22] = 0
        np.testing.assert_array_equal(OA.augment_one_seq(img, rec, gm, 5, r, kinds),
                                      OA.augment_one(img, rec, gm, 5, r))


def test_sequential_oracle_follows_the_chain_order():
    """Masks before the time stretch are stretched with the image; after it they are not."""
    img = np.arange(1, 112 * 112 + 1, dtype=np.float32).reshape(112, 112) / 12544.0
    r = _rec()
    r[19:21] = [40, 50]        # time mask, columns [40, 50)
    r[16], r[23] = 2.0, 8      # time stretch by 2 (t = 2c)
    K = OA
    before = OA.augment_one_seq(img, r, None, 0, 0, [K.K_TMASK, K.K_TWARP])
    after = OA.augment_one_seq(img, r, None, 0, 0, [K.K_TWARP, K.K_TMASK])
    assert (before[:, 20:25] == 0).all() and (before[:, 25:56] > 0).all()
    assert (after[:, 40:50] == 0).all() and (after[:, 20:25] > 0).all()
