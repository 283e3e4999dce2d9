"""AVMNIST on-disk loader with the dataset resident in HBM.

Reference: ``BaseAVMNISTDataset`` / ``AVMNISTDataset`` / ``AVMNISTSSLDataset(Extended)`` and the
data modules in AVMNIST_Experiments/utils/get_data.py:412-672, ``MemmapWrapper`` 745-764.

File contract (unchanged, so an existing AVMNIST directory drops in):

* ``f"{data_dir}image/{split}_data.npy"`` -- npy, (N, 28, 28) or (N, 784), byte-valued pixels
  (uint8, or a float array holding integers 0..255); opened with ``np.load(mmap_mode="r")``
  (never unpickled);
* ``f"{data_dir}audio/{split}_data_augmented_{type}.npy"`` -- a *raw* uint8 memmap (N, 112, 112)
  without an npy header (written by ``np.memmap(mode="w+")``, audio_gen.ipynb);
* ``f"{data_dir}{split}_labels.npy"`` -- (N,) integer labels.

``data_dir`` is concatenated as in the reference (it must end with "/").

MI355X-first layout: the whole split is copied to the device once as bytes (55,000 x (784 +
12,544) B = 733 MB of 288 GB HBM), so a step moves only its sample ids and augmentation records
over PCIe; normalisation (``_process_image_audio``, get_data.py:456-472) is the 256-entry byte
table applied inside the gather kernel.  ``random_split`` (606-609) is ``torch.randperm`` on the
given generator; batches follow ``DataLoader(shuffle=True, drop_last=False)`` order, and a
``DistributedSampler``-style rank stride when ``world > 1``.
"""
import os

import numpy as np
import torch

from .augment import MultiModalAugmentation, ViewAugmenter

IMG_HW, AUD_HW = (28, 28), (112, 112)


def avmnist_paths(data_dir, type="burst_noise"):
    """Paths of BaseAVMNISTDataModule.__init__ (get_data.py:545-551)."""
    return {
        "train": (f"{data_dir}image/train_data.npy", f"{data_dir}audio/train_data_augmented_{type}.npy",
                  f"{data_dir}train_labels.npy"),
        "test": (f"{data_dir}image/test_data.npy", f"{data_dir}audio/test_data_augmented_{type}.npy",
                 f"{data_dir}test_labels.npy"),
    }


def prepare_data(data_dir, type="burst_noise"):
    """BaseAVMNISTDataModule.prepare_data (get_data.py:553-558)."""
    for split in avmnist_paths(data_dir, type).values():
        for path in split:
            if not os.path.exists(path):
                raise FileNotFoundError(f"Data file not found: {path}")


def _as_bytes(arr, what):
    a = np.asarray(arr)
    if a.dtype == np.uint8:
        return a
    if not np.issubdtype(a.dtype, np.number) or a.size and (
            a.min() < 0 or a.max() > 255 or not np.array_equal(a, np.round(a))):
        raise ValueError(f"{what}: pixels must be byte values 0..255 for the device path")
    return a.astype(np.uint8)


class AVMNISTArrays:
    """One split: memory-mapped files (BaseAVMNISTDataset.__init__, get_data.py:412-442)."""

    def __init__(self, image_path, audio_path, labels_path, normalize_image=True,
                 normalize_audio=True, compute_stats=False):
        self.labels = np.load(labels_path).astype(int)
        self.image_data = np.load(image_path, mmap_mode="r")
        n = len(self.labels)
        self.audio_data = np.memmap(audio_path, mode="r", dtype=np.uint8, shape=(n, *AUD_HW))
        if self.image_data.shape[0] != n:
            raise ValueError("image and label counts differ")
        self.normalize_image, self.normalize_audio = normalize_image, normalize_audio
        if compute_stats and normalize_audio:
            a = np.asarray(self.audio_data, np.float64).reshape(n, -1) / 255.0
            self.audio_mean, self.audio_std = float(a.mean(1).mean()), float(a.std(1).mean())
        else:
            self.audio_mean, self.audio_std = 0.0, 1.0

    def __len__(self):
        return len(self.labels)

    def luts(self):
        """Byte -> f32 normalisation tables (get_data.py:464-467, float64 then float32)."""
        u = np.arange(256, dtype=np.float64)
        img = u / 255.0 if self.normalize_image else u
        aud = (u / 255.0 - self.audio_mean) / self.audio_std if self.normalize_audio else u
        return img.astype(np.float32), aud.astype(np.float32)

    def to_device(self, device):
        """The split's bytes, labels and tables as device tensors (one upload)."""
        n = len(self)
        img = _as_bytes(self.image_data, "image").reshape(n, -1)
        aud = np.asarray(self.audio_data).reshape(n, -1)
        li, la = self.luts()
        t = lambda a: torch.from_numpy(np.array(a, order="C")).to(device)  # noqa: E731
        return dict(image=t(img), audio=t(aud), labels=t(self.labels.astype(np.int64)),
                    lut_image=t(li), lut_audio=t(la))


def random_split_indices(n, lengths, generator=None):
    """torch.utils.data.random_split's index partition (randperm over the generator)."""
    if sum(lengths) != n:
        raise ValueError("Sum of input lengths does not equal the length of the input dataset!")
    perm = torch.randperm(n, generator=generator).numpy()
    out, off = [], 0
    for k in lengths:
        out.append(perm[off:off + k])
        off += k
    return out


class AVMNISTDinoLoader:
    """Batches of the DINO data modules on the device.

    ``multimodal_mode`` None/"default" yields ``(g_img, g_aud, l_img, l_aud)`` like
    ``AVMNISTSSLDataset`` (get_data.py:480-490); any other mode yields
    ``(image, audio, label, views)`` like ``AVMNISTSSLDatasetExtended`` (492-509).  The views
    come from the device ``MultiModalAugmentation`` (augment.py)."""

    def __init__(self, data_dir, batch_size=32, n_global_views=2, n_local_views=4,
                 type="burst_noise", augmentations=None, device="cuda", split="train",
                 train_size=55000, val_size=5000, seed=0, multimodal_mode="mse", shuffle=True,
                 rank=0, world=1, staged=False):
        self.paths = avmnist_paths(data_dir, type)
        for path in self.paths[split]:
            if not os.path.exists(path):
                raise FileNotFoundError(f"Data file not found: {path}")
        arrays = AVMNISTArrays(*self.paths[split])
        self.dev = arrays.to_device(device)
        n = len(arrays)
        self.seed = seed
        gen = torch.Generator().manual_seed(seed)
        if split == "train":   # random_split raises on a size mismatch (get_data.py:606-609)
            self.train_idx, self.val_idx = random_split_indices(n, [train_size, val_size], gen)
        else:
            self.train_idx, self.val_idx = np.arange(n), np.arange(0)
        self.batch_size, self.shuffle, self.rank, self.world = batch_size, shuffle, rank, world
        self.mode = multimodal_mode
        # staged=True: iterate staged_batch dicts (the multimodal engines build the views in
        # place and can prefetch them under the previous step) instead of collated views
        self.staged = staged
        self.aug = augmentations or MultiModalAugmentation(n_global_views, n_local_views)
        # augmentation streams differ per rank (each rank's worker RNGs do in the reference);
        # the shuffle order (seed) stays shared so the rank strides partition one permutation
        aseed = seed + 2 * rank
        self.aug.bind(ViewAugmenter(self.dev["image"], self.dev["lut_image"], *IMG_HW, seed=aseed),
                      ViewAugmenter(self.dev["audio"], self.dev["lut_audio"], *AUD_HW,
                                    seed=aseed + 1))
        self.epoch = 0

    def _order(self):
        idx = self.train_idx
        if self.shuffle:
            g = torch.Generator().manual_seed(self.seed + 1000003 * (self.epoch + 1))
            idx = idx[torch.randperm(len(idx), generator=g).numpy()]
        if self.world > 1:  # DistributedSampler: pad to a multiple of world, then stride
            total = -(-len(idx) // self.world) * self.world
            idx = np.concatenate([idx, idx[:total - len(idx)]])[self.rank::self.world]
        return idx

    def __len__(self):
        per_rank = -(-len(self.train_idx) // self.world)
        return -(-per_rank // self.batch_size)

    def batch(self, idx):
        views = self.aug(idx)
        if self.mode in (None, "default"):
            return views
        img = self.aug.image.identity(idx)
        aud = self.aug.audio.identity(idx)
        lab = self.dev["labels"][torch.from_numpy(np.asarray(idx, np.int64)).to(img.device)]
        return img, aud, lab, views

    def staged_batch(self, idx):
        """Engine fast path: {"aug", "idx", "label"} -- MultiCentralEngine.stage builds the views
        straight into its staged bf16 inputs (no collated f32 views)."""
        lab = self.dev["labels"][torch.from_numpy(np.asarray(idx, np.int64)).to(self.dev["labels"].device)]
        return {"aug": self.aug, "idx": np.asarray(idx, np.int64), "label": lab}

    def __iter__(self):
        if self.staged:
            yield from self.iter_staged()
            return
        order = self._order()
        self.epoch += 1
        for s in range(0, len(order), self.batch_size):
            yield self.batch(order[s:s + self.batch_size])

    def iter_staged(self):
        """One epoch of engine fast-path batches (staged_batch)."""
        order = self._order()
        self.epoch += 1
        for s in range(0, len(order), self.batch_size):
            yield self.staged_batch(order[s:s + self.batch_size])


class AVMNISTLabelledLoader:
    """``AVMNISTDataModule``'s loaders (get_data.py:592-620, batch 128): (images [B,1,28,28],
    audios [B,1,112,112], labels [B]) device batches, un-augmented and normalised by the byte
    tables.  split "train"/"val" = the two parts of random_split(55000, 5000) of the train
    files, "test" = the test files (the reference's random_split(test, [10000, 0]) only
    permutes them, and its test loader does not shuffle); the train split shuffles per epoch."""

    def __init__(self, data_dir, batch_size=128, type="burst_noise", device="cuda", split="train",
                 train_size=55000, val_size=5000, seed=0, shuffle=None):
        paths = avmnist_paths(data_dir, type)["test" if split == "test" else "train"]
        for path in paths:
            if not os.path.exists(path):
                raise FileNotFoundError(f"Data file not found: {path}")
        arrays = AVMNISTArrays(*paths)
        self.dev = arrays.to_device(device)
        n = len(arrays)
        if split == "test":
            self.idx = np.arange(n)
        else:
            tr, va = random_split_indices(n, [train_size, val_size], torch.Generator().manual_seed(seed))
            self.idx = tr if split == "train" else va
        self.batch_size, self.seed, self.epoch = batch_size, seed, 0
        self.shuffle = (split == "train") if shuffle is None else shuffle
        self.image = ViewAugmenter(self.dev["image"], self.dev["lut_image"], *IMG_HW, seed=seed)
        self.audio = ViewAugmenter(self.dev["audio"], self.dev["lut_audio"], *AUD_HW, seed=seed)

    def __len__(self):
        return -(-len(self.idx) // self.batch_size)

    def __iter__(self):
        idx = self.idx
        if self.shuffle:
            g = torch.Generator().manual_seed(self.seed + 1000003 * (self.epoch + 1))
            idx = idx[torch.randperm(len(idx), generator=g).numpy()]
        self.epoch += 1
        for s in range(0, len(idx), self.batch_size):
            b = idx[s:s + self.batch_size]
            lab = self.dev["labels"][torch.from_numpy(np.asarray(b, np.int64)).to(self.dev["labels"].device)]
            yield self.image.identity(b), self.audio.identity(b), lab
