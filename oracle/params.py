"""Deterministic parameter / input generators shared by the golden-vector script,
the oracle and the parity tests.  TEST INFRASTRUCTURE ONLY (see oracle/spec.py).

Values are a pure function of (seed, state-dict key, shape), so the reference
(imported only in this container by tests/golden/gen_golden.py), the oracle and
the HIP path all start from bit-identical fp32 tensors without shipping them.

Distributions follow PyTorch's defaults for the reference's layers
(Linear/Conv2d: U(-1/sqrt(fan_in), 1/sqrt(fan_in))), except that BatchNorm
affine parameters and the DINO center are perturbed away from their trivial
init (1 / 0 / 0) so the fixtures exercise them.
"""
import zlib

import numpy as np


def _rng(seed, key):
    return np.random.Generator(np.random.PCG64([seed, zlib.crc32(key.encode())]))


def make_tensor(seed, key, shape, kind):
    shape = tuple(shape)
    g = _rng(seed, key)
    if kind == "dense_w":
        fan_in = int(np.prod(shape[1:]))
        b = 1.0 / np.sqrt(fan_in)
        return g.uniform(-b, b, size=shape).astype(np.float32)
    if kind == "dense_b":
        return g.uniform(-0.1, 0.1, size=shape).astype(np.float32)
    if kind == "bn_w":
        return (1.0 + g.uniform(-0.2, 0.2, size=shape)).astype(np.float32)
    if kind == "bn_b":
        return g.uniform(-0.2, 0.2, size=shape).astype(np.float32)
    if kind == "rm":
        return np.zeros(shape, np.float32)
    if kind == "rv":
        return np.ones(shape, np.float32)
    if kind == "nbt":
        return np.zeros(shape, np.int64)
    if kind == "center":
        return g.uniform(-0.05, 0.05, size=shape).astype(np.float32)
    raise ValueError(kind)


def make_state(spec, seed):
    """spec: OrderedDict key -> (shape, kind)  ->  OrderedDict key -> ndarray."""
    return {k: make_tensor(seed, k, shp, kind) for k, (shp, kind) in spec.items()}


def make_multimodal_batch(B, G, L, seed, with_originals=True):
    """Synthetic AVMNIST batch in the reference's collated layout.

    image [B,1,28,28], audio [B,1,112,112], label [B] int64,
    views = (g_img [B,G,1,28,28], g_aud [B,G,1,112,112], l_img [B,L,...], l_aud [B,L,...]),
    pixel values randint(0,256)/255 in fp32, as get_data.py:456-467 produces.
    """
    g = np.random.Generator(np.random.PCG64([seed, 7]))

    def px(*shape):
        return (g.integers(0, 256, size=shape).astype(np.float32) / np.float32(255.0))

    out = {}
    out["g_img"] = px(B, G, 1, 28, 28)
    out["g_aud"] = px(B, G, 1, 112, 112)
    out["l_img"] = px(B, L, 1, 28, 28)
    out["l_aud"] = px(B, L, 1, 112, 112)
    if with_originals:
        out["image"] = px(B, 1, 28, 28)
        out["audio"] = px(B, 1, 112, 112)
        out["label"] = g.integers(0, 10, size=(B,)).astype(np.int64)
    return out


def make_simclr_batch(B, seed):
    g = np.random.Generator(np.random.PCG64([seed, 11]))

    def px(*shape):
        return (g.integers(0, 256, size=shape).astype(np.float32) / np.float32(255.0))

    return {"img1": px(B, 1, 28, 28), "spec1": px(B, 1, 112, 112),
            "img2": px(B, 1, 28, 28), "spec2": px(B, 1, 112, 112)}
