"""The device augmentation's chains and pure-torch stages pinned to the REFERENCE's own code
(fixtures from tests/golden/gen_augment_golden.py, which ran utils/get_data.py here with
recording placeholders for the absent torchvision / torchaudio):

* the transform chains MultiModalAugmentation builds (get_data.py:121-231) -- default and from the
  reference's configs/config_multimodal_dino.yaml through its own process_augment_config -- equal
  avdino.augment's chains: same transforms, order, probabilities and arguments;
* __call__'s control flow (233-257): global views through the global chains, then local views
  through the local chains, stacked view-first per sample;
* GroupedMasking.forward (60-108) and GaussianNoise.forward (21-27) -> GroupedMasking pixel outputs
  equal the stage-by-stage restatement (oracle/augment.py augment_one_seq) bit for bit, given the
  reference's own randperm / randn draws.
No GPU (tests/test_gpu_augment.py pins the kernels to the same restatement)."""
import json
import os

import numpy as np
import pytest
import yaml

from avdino import augment as A
from oracle import augment as OA

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")
REPO = os.path.dirname(HERE)

KIND = {"RandomResizedCrop": "crop", "RandomRotation": "rotation", "RandomAffine": "affine",
        "RandomErasing": "erasing", "TimeWarpWithStretch": "time_warp",
        "FrequencyMasking": "frequency_mask", "TimeMasking": "time_mask",
        "GaussianNoise": "gaussian_noise", "GroupedMasking": "grouped_masking"}
# constructor arguments that do not change what the device computes: the output size (every
# chain keeps the stored 28x28 / 112x112), antialias (the crops only up-sample), the stretch's
# target length (= the width), and defaults spelled out on one side only
_IGNORED = {"size", "antialias", "target_length"}
_DEFAULTS = {"degrees": 0, "group_size": 4}


def _norm_kw(kw):
    out = {}
    for k, v in kw.items():
        if k in _IGNORED or (k in _DEFAULTS and v == _DEFAULTS[k]):
            continue
        out[k] = [float(x) for x in v] if isinstance(v, (list, tuple)) else float(v)
    return out


def _ref_chain(entries):
    chain = []
    for e in entries:
        kw, p = dict(e["kwargs"]), e["p"]
        if e["cls"] == "RandomErasing":      # its own p, not a RandomApply
            p = kw.pop("p")
        chain.append((KIND[e["cls"]], _norm_kw(kw), float(p)))
    return chain


def _our_chain(chain):
    return [(k, _norm_kw(kw), float(p)) for k, kw, p in chain]


@pytest.fixture(scope="module")
def gold():
    with open(os.path.join(GOLD, "augment_chains.json")) as f:
        return json.load(f)


def test_default_chains_equal_the_references(gold):
    ours = A.default_chains()
    for view in ("global", "local"):
        for mod in ("image", "audio"):
            assert _our_chain(ours[view][mod]) == _ref_chain(gold["default"][view][mod]), (view, mod)


def test_config_chains_equal_the_references(gold):
    with open(os.path.join(REPO, "configs", "config_multimodal_dino.yaml")) as f:
        cfg = yaml.safe_load(f)
    best = A.process_augment_config(cfg)
    assert best == gold["process_augment_config"]
    aug = A.MultiModalAugmentation(2, 4, augment_values=best)
    ref = gold["config_multimodal_dino"]
    for view, tr in (("global", aug.global_transforms), ("local", aug.local_transforms)):
        for mod in ("image", "audio"):
            assert _our_chain(tr[mod]) == _ref_chain(ref[view][mod]), (view, mod)
    # the config's audio chains are in YAML key order, which the gather kernel cannot walk
    assert not A.fixed_order(aug.global_transforms["audio"])


def test_call_control_flow(gold):
    call = gold["call"]
    G, L = call["n_global_views"], call["n_local_views"]
    # per view: image then audio; G global views, then L local ones
    assert call["sequence"] == ["global.image", "global.audio"] * G + ["local.image", "local.audio"] * L
    # stacked view-first per sample; the DataLoader's collate puts the batch in front, which is
    # the [B, V, 1, H, W] layout MultiModalAugmentation.__call__ returns here
    assert call["shapes"] == [[G, 1, 28, 28], [G, 1, 112, 112], [L, 1, 28, 28], [L, 1, 112, 112]]


def _bits(idx, ng=784):
    words = (ng + 31) // 32
    gm = np.zeros((1, words), np.uint32)
    for g in np.asarray(idx):
        gm[0, g >> 5] |= np.uint32(1) << np.uint32(g & 31)
    return gm


def _rec():
    r = np.zeros(A.REC, np.float32)
    r[22] = -1
    return r


def test_grouped_masking_pixels_equal_the_references():
    z = np.load(os.path.join(GOLD, "augment_ref.npz"))
    lut = z["lut"]
    for r in range(3):
        img = lut[z["src_u8"][r]]
        idx = z[f"gm{r}_idx"]
        assert len(idx) == int(float(z[f"gm{r}_ratio"]) * 784)    # exactly int(ratio * groups)
        rec = _rec()
        rec[22] = 0
        out = OA.augment_one_seq(img, rec, _bits(idx), 0, 0, [OA.K_GMASK])
        np.testing.assert_array_equal(out, z[f"gm{r}_out"])


def test_noise_then_grouped_masking_equal_the_references():
    """GaussianNoise adds randn * std to every pixel, GroupedMasking then zeroes whole groups
    (noise included): the restatement given the reference's randn draws is bit-identical."""
    z = np.load(os.path.join(GOLD, "augment_ref.npz"))
    lut = z["lut"]
    for r in range(2):
        img = lut[z["src_u8"][3 + r]]
        rec = _rec()
        rec[21] = np.float32(z[f"nz{r}_std"])
        rec[22] = 0
        out = OA.augment_one_seq(img, rec, _bits(z[f"nz{r}_idx"]), 0, 0, [OA.K_NOISE, OA.K_GMASK],
                                 noise=z[f"nz{r}_noise"])
        np.testing.assert_array_equal(out, z[f"nz{r}_out"])
        assert (out != img).mean() > 0.5      # the noise reached the unmasked pixels
