"""Device-side multi-crop view augmentation.

The reference builds every view of every sample on CPU workers, one torchvision / torchaudio
transform at a time (``MultiModalAugmentation``, AVMNIST_Experiments/utils/get_data.py:110-257).
Here the host only draws the random parameters -- a few floats per (sample, view), vectorised
over the batch with numpy, following the published ``get_params`` rules of each transform --
and one HIP launch per (modality, view group) does the pixel work on the dataset rows that
already sit in HBM (``avd_augment_views``, csrc/augment.hip).

Transform chains (defaults, get_data.py:122-193) and how each stage is realised:

* ``RandomResizedCrop(size, scale, ratio=(3/4, 4/3))`` -- torchvision's 10-attempt area/aspect
  draw with the centre-crop fallback; bilinear resize of the integer box (the crops never
  shrink, so ``antialias=True`` changes nothing).
* ``RandomRotation(d)`` / ``RandomAffine(0, translate, scale)`` -- torchvision's inverse affine
  matrix about the image centre (``_get_inverse_affine_matrix``), nearest sampling, zero fill.
* ``TimeWarpWithStretch`` (get_data.py:29-58) -- |phase_vocoder| of a zero-phase spectrogram is
  the linear interpolation of magnitudes at t*rate (zero past the end), trimmed to the width.
* ``FrequencyMasking`` / ``TimeMasking`` -- torchaudio ``mask_along_axis``: width
  ``floor(U*param)``, start ``floor(U*(size - U*param))``; rows / columns set to 0.
* ``RandomErasing(p=0.3, scale=(0.02, 0.15), ratio=(0.3, 3.3))`` -- torchvision's draw, value 0.
* ``GaussianNoise(std)`` (get_data.py:21-27), ``GroupedMasking(ratio, 4)`` (get_data.py:60-108:
  exactly ``int(ratio * groups)`` distinct 4x4 groups zeroed).
* ``RandomApply([t], p)`` -- applied when U < p.

The random streams are numpy's, not torch's global generator, so individual views are not the
reference's views (the reference's own views are not reproducible across worker counts); the
parameter distributions are.  torchvision / torchaudio are absent here, so the match to their
pixel output is "parity unpinned"; the kernel's pixel maths is pinned by oracle/augment.py.
"""
import math

import collections

import numpy as np
import torch

from . import ops

KIND_ORDER = {"crop": 0, "time_warp": 1, "frequency_mask": 2, "time_mask": 2, "rotation": 3,
              "affine": 4, "erasing": 5, "gaussian_noise": 6, "grouped_masking": 7}
REC = ops.AUG_REC
F_CROP, F_AFF, F_ROT, F_TW = 1, 2, 4, 8


def default_chains():
    """The reference's default chains (get_data.py:122-193) as (kind, kwargs, p) lists."""
    img_g = [("crop", dict(scale=(0.75, 1.0)), 1.0), ("rotation", dict(degrees=5), 1.0),
             ("affine", dict(translate=(0.1, 0.1)), 1.0)]
    img_l = [("crop", dict(scale=(0.3, 0.75)), 1.0), ("rotation", dict(degrees=15), 1.0),
             ("affine", dict(translate=(0.2, 0.2), scale=(0.8, 1.2)), 1.0),
             ("erasing", dict(scale=(0.02, 0.15)), 0.3)]
    aud_g = [("crop", dict(scale=(0.8, 1.0)), 0.5),
             ("time_warp", dict(min_factor=0.9, max_factor=1.1), 0.3),
             ("frequency_mask", dict(freq_mask_param=15), 0.3),
             ("time_mask", dict(time_mask_param=15), 0.3),
             ("affine", dict(translate=(0, 0.1), scale=(0.9, 1.1)), 0.5),
             ("grouped_masking", dict(mask_ratio=0.15), 0.5)]
    aud_l = [("crop", dict(scale=(0.5, 0.9)), 0.7),
             ("time_warp", dict(min_factor=0.7, max_factor=1.3), 0.7),
             ("frequency_mask", dict(freq_mask_param=25), 0.7),
             ("time_mask", dict(time_mask_param=25), 0.7),
             ("affine", dict(translate=(0, 0.2), scale=(0.7, 1.3)), 0.7),
             ("gaussian_noise", dict(std=0.1), 0.7),
             ("grouped_masking", dict(mask_ratio=0.6), 0.9)]
    return {"global": {"image": img_g, "audio": aud_g}, "local": {"image": img_l, "audio": aud_l}}


_CUSTOM = {"time_warp": "time_warp", "frequency_mask": "frequency_mask", "time_mask": "time_mask",
           "grouped_masking": "grouped_masking", "gaussian_noise": "gaussian_noise",
           "random_affine": "affine", "random_resized_crop": "crop"}


def custom_audio_chain(augmentations, probabilities):
    """`augment_values` audio chains (get_data.py:195-231): {name: kwargs}, {name: p}."""
    chain = []
    for name, kw in augmentations.items():
        if name not in _CUSTOM:
            raise KeyError(name)
        kw = {k: tuple(v) if isinstance(v, list) else v for k, v in kw.items()}
        chain.append((_CUSTOM[name], kw, float(probabilities[name])))
    return chain


def validate_chain(chain):
    """Every stage a known transform, each at most once (a record has one parameter slot per
    transform kind).  Any order: transforms.Compose order is kept (avd_augment_views_seq)."""
    seen = set()
    for kind, _, _ in chain:
        if kind not in KIND_ORDER or kind in seen:
            raise NotImplementedError(f"transform chain not supported on device: {chain}")
        seen.add(kind)


def fixed_order(chain):
    """True when the chain is a sub-sequence of the gather kernel's order (avd_augment_views:
    crop -> time stretch -> masks -> rotation -> affine -> erasing -> noise -> groups), so the
    one-pass gather kernel applies it; other orders run stage by stage (avd_augment_views_seq)."""
    last = -1
    for kind, _, _ in chain:
        if KIND_ORDER[kind] < last:
            return False
        last = KIND_ORDER[kind]
    return True


def chain_kinds(chain):
    """The chain's stage kinds in application order (avd_augment_records numbering)."""
    return [_SK[kind] for kind, _, _ in chain]


# ----------------------------------------------------------------------------- parameter draws

def _rrc(rng, n, H, W, scale, ratio=(3.0 / 4.0, 4.0 / 3.0)):
    """torchvision RandomResizedCrop.get_params, vectorised over n draws."""
    area = H * W
    ta = area * rng.uniform(scale[0], scale[1], (n, 10))
    ar = np.exp(rng.uniform(math.log(ratio[0]), math.log(ratio[1]), (n, 10)))
    w = np.round(np.sqrt(ta * ar)).astype(np.int64)
    h = np.round(np.sqrt(ta / ar)).astype(np.int64)
    ok = (w > 0) & (w <= W) & (h > 0) & (h <= H)
    first = ok.argmax(1)
    has = ok.any(1)
    r = np.arange(n)
    h, w = h[r, first], w[r, first]
    in_ratio = W / H  # fallback: centre crop at the nearest admissible aspect
    if in_ratio < min(ratio):
        fw, fh = W, int(round(W / min(ratio)))
    elif in_ratio > max(ratio):
        fh, fw = H, int(round(H * max(ratio)))
    else:
        fw, fh = W, H
    h, w = np.where(has, h, fh), np.where(has, w, fw)
    i = np.where(has, rng.integers(0, H - h + 1), (H - fh) // 2)
    j = np.where(has, rng.integers(0, W - w + 1), (W - fw) // 2)
    return i, j, h, w


def _inverse_affine(angle_deg, tx, ty, s):
    """torchvision _get_inverse_affine_matrix with centre (0, 0) and no shear."""
    rot = np.radians(angle_deg)
    c, sn = np.cos(rot), np.sin(rot)
    m = np.stack([c, sn, np.zeros_like(c), -sn, c, np.zeros_like(c)], 1) / s[:, None]
    m[:, 2] += m[:, 0] * (-tx) + m[:, 1] * (-ty)
    m[:, 5] += m[:, 3] * (-tx) + m[:, 4] * (-ty)
    return m


def _erasing(rng, n, H, W, scale, ratio=(0.3, 3.3)):
    """torchvision RandomErasing.get_params (value 0), 10 attempts, else no erase."""
    area = H * W
    ea = area * rng.uniform(scale[0], scale[1], (n, 10))
    ar = np.exp(rng.uniform(math.log(ratio[0]), math.log(ratio[1]), (n, 10)))
    h = np.round(np.sqrt(ea * ar)).astype(np.int64)
    w = np.round(np.sqrt(ea / ar)).astype(np.int64)
    ok = (h < H) & (w < W)
    first = ok.argmax(1)
    has = ok.any(1)
    r = np.arange(n)
    h, w = np.where(has, h[r, first], 0), np.where(has, w[r, first], 0)
    i = np.where(has, rng.integers(0, H - h + 1), 0)
    j = np.where(has, rng.integers(0, W - w + 1), 0)
    return i, j, h, w


def _mask_band(rng, n, size, param):
    """torchaudio mask_along_axis: [floor(min_value), floor(min_value) + floor(value))."""
    value = rng.random(n) * param
    min_value = rng.random(n) * (size - value)
    start = np.floor(min_value).astype(np.int64)
    return start, start + np.floor(value).astype(np.int64)


def _group_bits(rng, n, ng, k):
    """n rows of exactly k distinct set bits out of ng (GroupedMasking's randperm[:k])."""
    words = (ng + 31) // 32
    bits = np.zeros((n, words * 32), np.uint64)
    if k > 0:
        pick = np.argpartition(rng.random((n, ng)), k - 1, axis=1)[:, :k]
        bits[np.arange(n)[:, None], pick] = 1
    weights = np.left_shift(np.uint64(1), np.arange(32, dtype=np.uint64))
    return (bits.reshape(n, words, 32) * weights).sum(2).astype(np.uint32)


def sample_records(rng, chain, n, H, W, group=4):
    """Draw one view's parameters for n samples: (rec [n, REC] f32, gm bitmask rows or None)."""
    validate_chain(chain)
    rec = np.zeros((n, REC), np.float32)
    rec[:, 22] = -1
    flags = np.zeros(n, np.int64)
    gm = None
    for kind, kw, p in chain:
        on = rng.random(n) < p
        if kind == "crop":
            i, j, h, w = _rrc(rng, n, H, W, kw.get("scale", (0.08, 1.0)),
                              kw.get("ratio", (3.0 / 4.0, 4.0 / 3.0)))
            rec[on, 0:4] = np.stack([i, j, h, w], 1)[on]
            flags[on] |= F_CROP
        elif kind == "rotation":
            d = kw["degrees"]
            m = _inverse_affine(-rng.uniform(-d, d, n), np.zeros(n), np.zeros(n), np.ones(n))
            rec[on, 10:16] = m[on]
            flags[on] |= F_ROT
        elif kind == "affine":
            d = kw.get("degrees", 0)
            ang = rng.uniform(-d, d, n)
            tr = kw.get("translate")
            tx = np.round(rng.uniform(-tr[0] * W, tr[0] * W, n)) if tr else np.zeros(n)
            ty = np.round(rng.uniform(-tr[1] * H, tr[1] * H, n)) if tr else np.zeros(n)
            sc = kw.get("scale")
            s = rng.uniform(sc[0], sc[1], n) if sc else np.ones(n)
            rec[on, 4:10] = _inverse_affine(ang, tx, ty, s)[on]
            flags[on] |= F_AFF
        elif kind == "time_warp":
            rec[on, 16] = rng.uniform(kw.get("min_factor", 0.8), kw.get("max_factor", 1.2), n)[on]
            flags[on] |= F_TW
        elif kind == "frequency_mask":
            a, b = _mask_band(rng, n, H, kw["freq_mask_param"])
            rec[on, 17], rec[on, 18] = a[on], b[on]
        elif kind == "time_mask":
            a, b = _mask_band(rng, n, W, kw["time_mask_param"])
            rec[on, 19], rec[on, 20] = a[on], b[on]
        elif kind == "erasing":
            i, j, h, w = _erasing(rng, n, H, W, kw.get("scale", (0.02, 0.33)),
                                  kw.get("ratio", (0.3, 3.3)))
            rec[on, 24:28] = np.stack([i, j, h, w], 1)[on]
        elif kind == "gaussian_noise":
            rec[on, 21] = kw.get("std", 0.1)
        elif kind == "grouped_masking":
            g = kw.get("group_size", 4)
            if g != group or H % g or W % g:
                raise ValueError("grouped masking needs H, W divisible by the group size")
            ng = (H // g) * (W // g)
            gm = _group_bits(rng, n, ng, int(kw.get("mask_ratio", 0.5) * ng))
            rec[on, 22] = np.arange(n)[on]
    rec[:, 23] = flags
    return rec, gm


# ----------------------------------------------------------------------------- device draws
_SK = {"crop": 0, "time_warp": 1, "frequency_mask": 2, "time_mask": 3, "rotation": 4,
       "affine": 5, "erasing": 6, "gaussian_noise": 7, "grouped_masking": 8}


def chain_stages(chain, group=4):
    """A chain as avd_augment_records' host stage table [S, 8] f32: {kind, p, params...}
    (include/avdino.h)."""
    validate_chain(chain)
    st = np.zeros((len(chain), ops.AUG_STAGE_F), np.float32)
    for i, (kind, kw, pr) in enumerate(chain):
        q = st[i, 2:]
        st[i, 0], st[i, 1] = _SK[kind], pr
        if kind == "crop":
            q[0:2] = kw.get("scale", (0.08, 1.0))
            q[2:4] = kw.get("ratio", (3.0 / 4.0, 4.0 / 3.0))
        elif kind == "erasing":
            q[0:2] = kw.get("scale", (0.02, 0.33))
            q[2:4] = kw.get("ratio", (0.3, 3.3))
        elif kind == "time_warp":
            q[0], q[1] = kw.get("min_factor", 0.8), kw.get("max_factor", 1.2)
        elif kind == "frequency_mask":
            q[0] = kw["freq_mask_param"]
        elif kind == "time_mask":
            q[0] = kw["time_mask_param"]
        elif kind == "rotation":
            q[0] = kw["degrees"]
        elif kind == "affine":
            q[0] = kw.get("degrees", 0)
            tr, sc = kw.get("translate"), kw.get("scale")
            q[1], q[2] = tr if tr else (-1.0, -1.0)
            q[3], q[4] = sc if sc else (0.0, 0.0)
        elif kind == "gaussian_noise":
            q[0] = kw.get("std", 0.1)
        elif kind == "grouped_masking":
            if kw.get("group_size", 4) != group:
                raise ValueError("grouped masking group size must match the kernel's group")
            q[0] = kw.get("mask_ratio", 0.5)
    return st


# ----------------------------------------------------------------------------- the device op

class ViewAugmenter:
    """One modality's device view builder over a dataset resident in HBM.

    ``src_u8`` [N, H*W] uint8 on the device, ``lut`` [256] f32 (the dataset's normalisation).
    ``__call__(idx, chain, n_views)`` -> f32 [B, n_views, 1, H, W] on the device."""

    def __init__(self, src_u8, lut, H, W, seed=0, device_params=True, sequential=False):
        self.src, self.lut, self.H, self.W = src_u8, lut, H, W
        # sequential=True: every chain through the stage-by-stage kernel (tests compare the two)
        self.sequential = sequential
        self.rng = np.random.default_rng(seed)
        self.seed = seed
        self.calls = 0
        # parameters drawn by avd_augment_records (default) or by numpy on the host
        self.device_params = device_params
        self._stage_cache = {}
        self._pinned = collections.deque(maxlen=64)    # host ids of in-flight transfers

    def records_dev(self, chain, B, n_views, group=4):
        """(rec [B*n_views, REC], gm [B*n_views, words] or None) drawn on the device."""
        key = id(chain)
        st = self._stage_cache.get(key)
        if st is None or st[0] is not chain:
            st = (chain, chain_stages(chain, group))
            self._stage_cache[key] = st
        stages = st[1]
        n = B * n_views
        dev = self.src.device
        rec = torch.empty(n, REC, dtype=torch.float32, device=dev)
        gm = None
        if any(k == "grouped_masking" for k, _, _ in chain):
            words = ((self.H // group) * (self.W // group) + 31) // 32
            gm = torch.empty(n, words, dtype=torch.int32, device=dev)
        self.calls += 1
        rseed = (self.seed * 0xD1B54A32D192ED03 + 0x5EED * self.calls) & (2**64 - 1)
        ops.augment_records(stages, n, self.H, self.W, group, rseed, rec, gm)
        return rec, gm

    def records(self, chain, B, n_views):
        rec = np.zeros((B, n_views, REC), np.float32)
        gms, rows = [], 0
        for v in range(n_views):
            r, gm = sample_records(self.rng, chain, B, self.H, self.W)
            if gm is not None:
                r[r[:, 22] >= 0, 22] += rows
                gms.append(gm)
                rows += gm.shape[0]
            rec[:, v] = r
        return rec.reshape(B * n_views, REC), (np.concatenate(gms) if gms else None)

    def __call__(self, idx, chain, n_views, out=None, order=0):
        idx = np.asarray(idx, np.int64)
        if self.device_params:
            rec, gm = self.records_dev(chain, idx.shape[0], n_views)
        else:
            rec, gm = self.records(chain, idx.shape[0], n_views)
        kinds = chain_kinds(chain) if (self.sequential or not fixed_order(chain)) else None
        return self.apply(idx, rec, gm, n_views, out, order, kinds)

    def apply(self, idx, rec, gm, n_views, out=None, order=0, kinds=None):
        """kinds: the stage kinds in application order for avd_augment_views_seq (None: the
        fixed-order gather kernel)."""
        idx = np.asarray(idx, np.int64)
        if idx.size == 0 or idx.min() < 0 or idx.max() >= self.src.shape[0]:
            raise IndexError("sample id outside the dataset")
        on_dev = isinstance(rec, torch.Tensor)   # avd_augment_records: gm row r for record r
        if not on_dev and gm is not None and rec[:, 22].max() >= gm.shape[0]:
            raise IndexError("grouped-mask row outside the bitmask table")
        dev = self.src.device
        B = idx.shape[0]
        shape = (B, n_views, 1, self.H, self.W) if order == 0 else (n_views, B, 1, self.H, self.W)
        if out is None:
            out = torch.empty(shape, dtype=torch.float32, device=dev)
        # pinned + non-blocking: a data-stream prefetch must not block the host on that stream.
        # The pinned copy of the ids is also held here for a while: a prefetch's transfer runs
        # only once its data stream's wait is over, possibly after this call has returned
        idx_t = torch.from_numpy(idx)
        if dev.type == "cuda":
            pin = idx_t.pin_memory()
            self._pinned.append(pin)
            idx_d = pin.to(dev, non_blocking=True)
        else:
            idx_d = idx_t.to(dev)
        if on_dev:
            rec_d, gm_d = rec, gm
        else:
            rec_d = torch.from_numpy(np.ascontiguousarray(rec, np.float32)).to(dev)
            gm_d = None if gm is None else torch.from_numpy(gm.view(np.int32)).to(dev)
        self.calls += 1
        seed = (self.seed * 0x9E3779B97F4A7C15 + self.calls) & (2**64 - 1)
        ops.augment_views(self.src, idx_d, self.lut, rec_d, gm_d, 4, seed, n_views, self.H,
                          self.W, out, order, kinds)
        return out

    def identity(self, idx, out=None):
        """Un-augmented normalised rows [B, 1, H, W] (the dataset's `_process_image_audio`)."""
        rec = np.zeros((len(idx), REC), np.float32)
        rec[:, 22] = -1
        return self.apply(idx, rec, None, 1, out).view(len(idx), 1, self.H, self.W)


class MultiModalAugmentation:
    """Device counterpart of get_data.py:110-257 for a batch of dataset rows.

    Same constructor; after ``bind(image_augmenter, audio_augmenter)``, ``__call__(idx)`` returns
    the collated views ``(g_img [B,G,1,28,28], g_aud [B,G,1,112,112], l_img, l_aud)``."""

    def __init__(self, n_global_views=2, n_local_views=4, global_spec_size=112,
                 local_spec_size=112, augment_values=None):
        if global_spec_size != 112 or local_spec_size != 112:
            raise NotImplementedError("device crops resize to the stored 112x112 spectrogram")
        self.n_global_views, self.n_local_views = n_global_views, n_local_views
        self.global_spec_size, self.local_spec_size = global_spec_size, local_spec_size
        ch = default_chains()
        self.global_transforms = dict(ch["global"])
        self.local_transforms = dict(ch["local"])
        if augment_values is not None:
            aug, pr = augment_values["augmentations"], augment_values["augmentation_probabilities"]
            self.global_transforms["audio"] = custom_audio_chain(aug["global_views"],
                                                                 pr["global_views"])
            self.local_transforms["audio"] = custom_audio_chain(aug["local_views"],
                                                                pr["local_views"])
        for t in (self.global_transforms, self.local_transforms):
            for c in t.values():
                validate_chain(c)
        self.image = self.audio = None

    def bind(self, image_aug, audio_aug):
        self.image, self.audio = image_aug, audio_aug
        return self

    def __call__(self, idx):
        G, L = self.n_global_views, self.n_local_views
        gi = self.image(idx, self.global_transforms["image"], G)
        ga = self.audio(idx, self.global_transforms["audio"], G)
        li = self.image(idx, self.local_transforms["image"], L) if L else None
        la = self.audio(idx, self.local_transforms["audio"], L) if L else None
        return gi, ga, li, la

    def stage(self, idx, x_img, x_aud, with_orig):
        """Build the views straight into the engine's staged view-major inputs (bf16 or f32
        [(G + L [+1]) * B, H, W]): global views rows [0, G*B), local views [G*B, (G+L)*B), the
        un-augmented originals (the Extended dataset's image / audio) the last B rows -- the
        layout avd_stage_views would produce from the collated f32 views, without them."""
        idx = np.asarray(idx, np.int64)
        B, G, L = idx.shape[0], self.n_global_views, self.n_local_views
        for aug, x, hw in ((self.image, x_img, 784), (self.audio, x_aud, 12544)):
            key = "image" if aug is self.image else "audio"
            nv = G + L + (1 if with_orig else 0)
            xv = x.view(nv, B * hw)
            aug(idx, self.global_transforms[key], G, out=xv[:G].view(-1), order=1)
            if L:
                aug(idx, self.local_transforms[key], L, out=xv[G:G + L].view(-1), order=1)
            if with_orig:
                aug.identity(idx, out=xv[G + L].view(-1))


def process_augment_config(config, trial=None, is_hyperparameter_search=False):
    """process_augment_config's final-training branch (hyperparameter_tuning/
    objective_augment.py:68-96): the config's ``best_augments`` split into
    {"augmentations": kwargs without p, "augmentation_probabilities": p} per view setting.
    The Optuna search branch is out of scope."""
    if is_hyperparameter_search:
        raise NotImplementedError("Optuna augmentation search is outside the MI355X hot path")
    if "best_augments" not in config:
        raise ValueError("best_augments not found in config for final training")
    augmentations = {"global_views": {}, "local_views": {}}
    probabilities = {"global_views": {}, "local_views": {}}
    for view in ("global_views", "local_views"):
        for aug, params in config["best_augments"][view].items():
            kw = {k: v for k, v in params.items() if k != "p"}
            if kw:
                augmentations[view][aug] = kw
            if "p" in params:
                probabilities[view][aug] = params["p"]
    return {"augmentations": augmentations, "augmentation_probabilities": probabilities}
