"""Helpers to compare results against the golden fixtures in tests/golden/.

A fixture stores each tensor either fully (key) or as size-independent
properties (key@sum, key@norm, key@idx, key@val) -- see tests/golden/gen_golden.py.
"""
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    return dict(np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False))


def has(fx, key):
    return key in fx or (key + "@norm") in fx


def rel_err(a, b):
    a = np.asarray(a, np.float64).reshape(-1)
    b = np.asarray(b, np.float64).reshape(-1)
    nb = np.linalg.norm(b)
    return np.linalg.norm(a - b) / max(nb, 1e-30)


def compare(fx, key, value, rel=1e-4, abs_floor=0.0):
    """Return (ok, message).  rel = bound on relative L2 error (full tensors) or on the
    relative error of the norm and of the sampled entries (summarised tensors).
    abs_floor > 0 marks a tensor that is mathematically zero (e.g. a conv bias feeding
    BN): then only |value| <= abs_floor is required, whatever noise the fixture holds."""
    v = np.asarray(value, np.float64)
    if abs_floor > 0:
        nv = np.linalg.norm(v)
        return nv <= abs_floor, f"{key}: |v|={nv:.3g} (zero-gradient tensor, floor {abs_floor:g})"
    if key in fx:
        ref = np.asarray(fx[key], np.float64)
        if ref.shape != v.shape:
            return False, f"{key}: shape {v.shape} vs {ref.shape}"
        nref = np.linalg.norm(ref)
        if nref <= abs_floor:
            ok = np.linalg.norm(v) <= 10 * abs_floor
            return ok, f"{key}: |v|={np.linalg.norm(v):.3g} (ref {nref:.3g}, zero-gradient tensor)"
        e = rel_err(v, ref)
        return e <= rel, f"{key}: rel_err={e:.3g}"
    if key + "@norm" not in fx:
        return False, f"{key}: not in fixture"
    flat = v.reshape(-1)
    nref = float(fx[key + "@norm"])
    if nref <= abs_floor:
        ok = np.linalg.norm(flat) <= 10 * abs_floor
        return ok, f"{key}: |v|={np.linalg.norm(flat):.3g} (zero-gradient tensor)"
    en = abs(np.linalg.norm(flat) - nref) / nref
    idx = fx[key + "@idx"]
    es = rel_err(flat[idx], fx[key + "@val"])
    n = flat.size
    esum = abs(flat.sum() - float(fx[key + "@sum"])) / (nref * np.sqrt(n))
    ok = en <= rel and es <= 10 * rel and esum <= rel
    return ok, f"{key}: norm_err={en:.3g} sample_err={es:.3g} sum_err={esum:.3g}"


def zero_grad_keys(fx64, prefix="grad/"):
    """Gradient tensors that are mathematically zero: biases of layers whose output
    only reaches the loss through a train-mode BatchNorm (via linear maps), e.g. conv
    biases before BN2d, fusion.3 / projection Linear biases before BN1d.  Read from the
    float64 reference run, where they are rounding noise (< 1e-9); the fp32 reference
    holds noise up to ~1e-5 there (hard part (ii))."""
    out = set()
    for k in fx64:
        if not k.startswith(prefix) and ("/" + prefix) not in k:
            continue
        if k.endswith("@norm"):
            if float(fx64[k]) < 1e-9:
                out.add(k[:-5])
        elif "@" not in k and np.linalg.norm(np.asarray(fx64[k], np.float64)) < 1e-9:
            out.add(k)
    return out
