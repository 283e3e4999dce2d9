"""Golden vectors for the device augmentation, made by running the REFERENCE's own transform
code in this container (the reference never runs on the GPU box; this writes small fixtures).

    python tests/golden/gen_augment_golden.py [--out tests/golden]

What is pinned (VERDICT r2 "What's missing" 2):

* ``augment_chains.json`` -- the structure of ``MultiModalAugmentation`` (utils/get_data.py:110-231)
  as the reference builds it: every view's image / audio chain (transform class, constructor
  arguments, RandomApply probability, order), for the default transforms and for
  ``augment_values`` = the reference's own ``process_augment_config`` of its shipped
  configs/config_multimodal_dino.yaml; plus the call sequence of ``__call__`` (233-257).
  torchvision / torchaudio are absent here, so their classes are *recording* placeholders
  (written to /tmp, never part of this repo) that keep their constructor arguments and log
  their calls; the reference's own classes (GaussianNoise, GroupedMasking,
  TimeWarpWithStretch) are the real ones.
* ``augment_ref.npz`` -- pixel outputs of the reference's pure-torch transforms on seeded
  inputs, with the random draws they consumed re-drawn from the same torch seed:
  ``GroupedMasking.forward`` (60-108: randperm(ng)[:k]) at three mask ratios, and
  ``GaussianNoise.forward`` (21-27: x + randn_like(x) * std) followed by GroupedMasking (the
  order of the reference's local audio chain, 189-191).

TimeWarpWithStretch / FrequencyMasking / TimeMasking / RandomResizedCrop / RandomAffine call
torchaudio / torchvision kernels that are absent, so their pixel output stays "parity
unpinned" (oracle/augment.py restates their published algorithms).
"""
import argparse
import json
import os
import sys
import textwrap

import numpy as np

REF = "/root/reference/AVMNIST_Experiments"
STUB_DIR = "/tmp/avdino_aug_stubs"
HERE = os.path.dirname(os.path.abspath(__file__))

# recording placeholders: Compose / RandomApply keep their children, every class keeps its
# constructor arguments, __call__ logs (class, id) and returns its input unchanged
_REC = textwrap.dedent('''
    LOG = []
    class _Rec:
        def __init__(self, *args, **kwargs):
            self.args, self.kwargs = list(args), dict(kwargs)
        def __call__(self, x, *a, **k):
            LOG.append((type(self).__name__, id(self)))
            return x
    class Compose(_Rec):
        def __init__(self, transforms):
            super().__init__()
            self.transforms = list(transforms)
        def __call__(self, x):
            LOG.append(("Compose", id(self)))
            for t in self.transforms:
                x = t(x)
            return x
    class RandomApply(_Rec):
        def __init__(self, transforms, p=0.5):
            super().__init__()
            self.transforms, self.p = list(transforms), p
''')
STUBS = {
    "lightning/__init__.py": "from . import pytorch\n",
    "lightning/pytorch/__init__.py": textwrap.dedent("""
        import torch.nn as nn
        class LightningModule(nn.Module):
            def save_hyperparameters(self, *a, **k): pass
            def log(self, *a, **k): pass
        class LightningDataModule: pass
        class Callback: pass
        def seed_everything(*a, **k): pass
        """),
    "lightning/pytorch/callbacks.py": "class ModelCheckpoint: pass\nclass EarlyStopping: pass\n",
    "lightning/pytorch/loggers.py": "class CSVLogger: pass\n",
    "optuna/__init__.py": "from . import integration\n",
    "optuna/integration/__init__.py": "from . import pytorch_lightning\n",
    "optuna/integration/pytorch_lightning.py": "class PyTorchLightningPruningCallback: pass\n",
    "torchvision/__init__.py": "from . import transforms, models\n",
    "torchvision/transforms.py": _REC + "".join(
        f"class {n}(_Rec): pass\n"
        for n in ["RandomResizedCrop", "RandomRotation", "RandomAffine", "RandomErasing",
                  "ElasticTransform", "GaussianBlur", "Resize", "ToTensor", "Normalize",
                  "RandomCrop", "Lambda"]),
    "torchvision/models/__init__.py": "",
    "torchvision/models/mobilenetv3.py": "def mobilenet_v3_small(*a, **k): raise RuntimeError('stub')\n",
    "torchvision/models/resnet.py": "def resnet18(*a, **k): raise RuntimeError('stub')\n",
    "torchaudio/__init__.py": "from . import transforms\n",
    "torchaudio/transforms.py": _REC.replace("LOG = []", "from torchvision.transforms import LOG")
    + "".join(f"class {n}(_Rec): pass\n"
              for n in ["TimeStretch", "FrequencyMasking", "TimeMasking", "Spectrogram"]),
    "torchmetrics/__init__.py": "",
    "torchmetrics/classification.py": "class Accuracy:\n    def __init__(self, *a, **k): pass\n",
    "torchinfo/__init__.py": "def summary(*a, **k): raise RuntimeError('stub')\n",
}


def write_stubs():
    for rel, src in STUBS.items():
        path = os.path.join(STUB_DIR, rel)
        os.makedirs(os.path.dirname(path), exist_ok=True)
        with open(path, "w") as f:
            f.write(src)
    sys.path.insert(0, REF)
    sys.path.insert(0, STUB_DIR)


def _jsonable(v):
    if isinstance(v, (list, tuple)):
        return [_jsonable(x) for x in v]
    if isinstance(v, (int, float, str, bool)) or v is None:
        return v
    return repr(v)


def describe(t):
    """One chain entry: {cls, kwargs, p} (RandomApply unwrapped; p = 1 for a bare transform)."""
    name = type(t).__name__
    if name == "RandomApply":
        assert len(t.transforms) == 1
        inner = describe(t.transforms[0])
        inner["p"] = float(t.p)
        return inner
    if name == "GaussianNoise":
        kw = {"std": float(t.std)}
    elif name == "GroupedMasking":
        kw = {"mask_ratio": float(t.mask_ratio), "group_size": int(t.group_size)}
    elif name == "TimeWarpWithStretch":
        kw = {"min_factor": float(t.min_factor), "max_factor": float(t.max_factor),
              "target_length": int(t.target_length)}
    else:
        kw = {k: _jsonable(v) for k, v in t.kwargs.items()}
        if t.args:
            kw["_args"] = _jsonable(t.args)
    return {"cls": name, "kwargs": kw, "p": 1.0}


def chains_of(aug):
    out = {}
    for view, tr in (("global", aug.global_transforms), ("local", aug.local_transforms)):
        out[view] = {mod: [describe(t) for t in tr[mod].transforms] for mod in ("image", "audio")}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=HERE)
    args = ap.parse_args()
    write_stubs()
    import torch
    import yaml
    from torchvision import transforms as tv
    from utils.get_data import GaussianNoise, GroupedMasking, MultiModalAugmentation
    from hyperparameter_tuning.objective_augment import process_augment_config

    with open(os.path.join(REF, "configs", "config_multimodal_dino.yaml")) as f:
        cfg = yaml.safe_load(f)
    best = process_augment_config(None, cfg, is_hyperparameter_search=False)
    fx = {"default": chains_of(MultiModalAugmentation()),
          "config_multimodal_dino": chains_of(MultiModalAugmentation(augment_values=best)),
          "process_augment_config": best}

    # __call__ control flow: which chain runs for which view, in what order, and the stacking
    aug = MultiModalAugmentation(n_global_views=2, n_local_views=3)
    names = {id(aug.global_transforms["image"]): "global.image",
             id(aug.global_transforms["audio"]): "global.audio",
             id(aug.local_transforms["image"]): "local.image",
             id(aug.local_transforms["audio"]): "local.audio"}
    tv.LOG.clear()
    img, aud = torch.zeros(1, 28, 28), torch.zeros(1, 112, 112)
    gi, ga, li, la = aug(img, aud)
    fx["call"] = {"n_global_views": 2, "n_local_views": 3,
                  "sequence": [names[i] for c, i in tv.LOG if c == "Compose"],
                  "shapes": [list(t.shape) for t in (gi, ga, li, la)]}
    with open(os.path.join(args.out, "augment_chains.json"), "w") as f:
        json.dump(fx, f, indent=1, sort_keys=True)

    # pixel fixtures: the reference's pure-torch transforms on normalised uint8 rows
    rng = np.random.default_rng(2024)
    u8 = rng.integers(0, 256, (6, 112, 112), dtype=np.uint8)
    lut = (np.arange(256, dtype=np.float64) / 255.0).astype(np.float32)    # get_data.py:467
    npz = {"src_u8": u8, "lut": lut}
    ratios = [0.15, 0.6, float(best["augmentations"]["local_views"]["grouped_masking"]["mask_ratio"])]
    for r, ratio in enumerate(ratios):
        x = torch.from_numpy(lut[u8[r]]).reshape(1, 112, 112)
        seed = 100 + r
        torch.manual_seed(seed)
        y = GroupedMasking(mask_ratio=ratio)(x.clone())
        torch.manual_seed(seed)
        ng = (112 // 4) * (112 // 4)
        masked = torch.randperm(ng)[:int(ratio * ng)]
        npz[f"gm{r}_ratio"] = np.float64(ratio)
        npz[f"gm{r}_idx"] = masked.numpy().astype(np.int64)
        npz[f"gm{r}_out"] = y.numpy().reshape(112, 112)
    # GaussianNoise then GroupedMasking (the local audio chain's last two stages)
    for r, (std, ratio) in enumerate([(0.1, 0.6), (0.18046730961749252, 0.15)]):
        x = torch.from_numpy(lut[u8[3 + r]]).reshape(1, 112, 112)
        seed = 200 + r
        torch.manual_seed(seed)
        y = GroupedMasking(mask_ratio=ratio)(GaussianNoise(std=std)(x.clone()))
        torch.manual_seed(seed)
        noise = torch.randn_like(x)
        ng = (112 // 4) * (112 // 4)
        masked = torch.randperm(ng)[:int(ratio * ng)]
        npz[f"nz{r}_std"] = np.float64(std)
        npz[f"nz{r}_ratio"] = np.float64(ratio)
        npz[f"nz{r}_noise"] = noise.numpy().reshape(112, 112)
        npz[f"nz{r}_idx"] = masked.numpy().astype(np.int64)
        npz[f"nz{r}_out"] = y.numpy().reshape(112, 112)
    np.savez_compressed(os.path.join(args.out, "augment_ref.npz"), **npz)
    print("wrote augment_chains.json, augment_ref.npz")


if __name__ == "__main__":
    main()
