"""Deterministic synthetic weights / inputs shared by the golden generator and the tests.

TEST INFRASTRUCTURE (oracle). Every tensor is drawn from numpy PCG64 seeded by
(seed, crc32(name)), so any module exposing the reference's state_dict keys
 receives bit-identical values on any machine.

Distributions (own choice, documented in DESIGN.md §Oracle):
  Linear / conv weight       U(-1,1)/sqrt(fan_in)
  biases                     U(-0.1,0.1)
  LayerNorm / BN weight      1 + U(-0.1,0.1)
  layer_scale_*              U(0.5,1.0)  (the reference's 1e-6 init hides the branches)
  BN running_mean / var      U(-0.1,0.1) / U(0.5,1.5)
Inputs follow the reference's normalisation conventions
(rgb: (U{0..255}/255 - mean)/std, NYUDepthv2.py:72-73; depth: (U/255-0.48)/0.28, dataloader.py:56-58).
"""
import zlib

import numpy as np

RGB_MEAN = np.array([0.485, 0.456, 0.406])
RGB_STD = np.array([0.229, 0.224, 0.225])


def rng(seed, name):
    return np.random.Generator(np.random.PCG64([seed, zlib.crc32(name.encode())]))


def param_value(name, shape, seed=1234):
    g = rng(seed, name)
    leaf = name.split(".")[-1]
    shape = tuple(shape)
    if leaf == "num_batches_tracked":
        return np.zeros(shape, dtype=np.int64)
    if "layer_scale" in leaf:
        return g.uniform(0.5, 1.0, shape)
    if leaf == "running_mean":
        return g.uniform(-0.1, 0.1, shape)
    if leaf == "running_var":
        return g.uniform(0.5, 1.5, shape)
    if leaf == "bias":
        return g.uniform(-0.1, 0.1, shape)
    if leaf == "weight":
        if len(shape) == 1:  # LN / BN affine
            return 1.0 + g.uniform(-0.1, 0.1, shape)
        fan_in = int(np.prod(shape[1:]))
        return g.uniform(-1.0, 1.0, shape) / np.sqrt(fan_in)
    raise KeyError(name)


def state_dict_values(named_shapes, seed=1234):
    """named_shapes: iterable of (name, shape). Returns {name: float64/int64 ndarray}."""
    return {n: param_value(n, s, seed) for n, s in named_shapes}


def rgb_depth(B, H, W, seed=8964):
    g = rng(seed, "inputs")
    rgb = g.integers(0, 256, (B, 3, H, W)) / 255.0
    rgb = (rgb - RGB_MEAN[None, :, None, None]) / RGB_STD[None, :, None, None]
    dep = g.integers(0, 256, (B, 1, H, W)) / 255.0
    dep = (dep - 0.48) / 0.28
    return rgb, dep


def labels(B, H, W, ncls=40, seed=8964, ignore_frac=0.1):
    g = rng(seed, "labels")
    lab = g.integers(0, ncls, (B, H, W))
    lab[g.random((B, H, W)) < ignore_frac] = 255
    return lab


def normal(name, shape, seed=77, scale=1.0):
    return rng(seed, name).standard_normal(tuple(shape)) * scale


def uniform(name, shape, lo=0.0, hi=1.0, seed=77):
    return rng(seed, name).uniform(lo, hi, tuple(shape))


def nmf_bases(B, D, R, seed=4242, name="nmf_bases"):
    """Injected NMF bases: F.normalize(U[0,1), dim=1) exactly like ham_head.py:109-117."""
    b = rng(seed, name).random((B, D, R))
    return b / np.maximum(np.sqrt((b * b).sum(axis=1, keepdims=True)), 1e-12)


def fingerprint(a, nsamp=64):
    """Size-independent statistic vector of an array: sum, abs-sum, l2, strided samples."""
    f = np.asarray(a, dtype=np.float64).ravel()
    idx = np.linspace(0, f.size - 1, min(nsamp, f.size)).astype(np.int64)
    return np.concatenate([[f.sum(), np.abs(f).sum(), np.sqrt((f * f).sum())], f[idx]])
