"""Library-independent deterministic weights (TEST INFRASTRUCTURE).

Every state_dict key gets a splitmix64 counter stream seeded by crc32(key); values are
uniform in [-1, 1) times a per-key scale (so fixtures never depend on torch's RNG draw
order or version).  numpy-only so the GPU box regenerates identical fp32 tensors.
"""
from __future__ import annotations

import zlib

import numpy as np

_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)
_G = np.uint64(0x9E3779B97F4A7C15)


def splitmix_uniform(seed: int, n: int) -> np.ndarray:
    """n uniforms in [-1, 1) from a splitmix64 counter stream."""
    with np.errstate(over="ignore"):
        idx = np.arange(1, n + 1, dtype=np.uint64)
        z = np.uint64(seed) + idx * _G
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        z = z ^ (z >> np.uint64(31))
    u = (z >> np.uint64(40)).astype(np.float64) / float(1 << 24)  # [0, 1)
    return (2.0 * u - 1.0).astype(np.float32)


def key_seed(key: str, salt: int = 0) -> int:
    return (zlib.crc32(key.encode()) * 2654435761 + salt) & 0xFFFFFFFFFFFF


def scale_for(key: str, shape) -> float:
    """Magnitudes roughly matching the reference inits (std ~0.02 linears, LN ~1)."""
    if key.endswith("cross_gate"):
        return 0.5  # non-zero so the gated cross-attention path is exercised
    if ".ln" in key or key.startswith("ln") or "ln_" in key or key.endswith(("ln1.weight",)):
        if key.endswith("weight"):
            return -1.0  # marker: 1 + 0.1*u
        return 0.05
    if key.endswith("query_tokens"):
        return 1.0
    if key.endswith("bias") or key.endswith("in_proj_bias"):
        return 0.02
    return 0.035


def make_tensor(key: str, shape, salt: int = 0) -> np.ndarray:
    n = int(np.prod(shape)) if len(shape) else 1
    u = splitmix_uniform(key_seed(key, salt), n).reshape(shape)
    s = scale_for(key, shape)
    if s < 0:
        return np.asarray(1.0 + 0.1 * u, dtype=np.float32).reshape(shape)
    return np.asarray(s * u, dtype=np.float32).reshape(shape)


def make_state(keys_shapes, salt: int = 0, tied=(("lm_head.weight", "transformer.wte.weight"),)):
    """{key: np.float32 array} for [(key, shape)]; tied keys share the first key's values."""
    out = {}
    for k, shp in keys_shapes:
        out[k] = make_tensor(k, tuple(shp), salt)
    for a, b in tied:
        for k in list(out):
            if k.endswith(a):
                kb = k[: -len(a)] + b
                if kb in out:
                    out[kb] = out[k]
    return out


def make_ids(n: int, vocab: int, seed: int) -> np.ndarray:
    u = splitmix_uniform(seed, n)
    return np.minimum(((u + 1.0) * 0.5 * vocab).astype(np.int64), vocab - 1)


def make_normal_like(n: int, seed: int) -> np.ndarray:
    """Deterministic ~N(0,1) values (Box-Muller on two splitmix streams)."""
    u1 = (splitmix_uniform(seed, n).astype(np.float64) + 1.0) * 0.5
    u2 = (splitmix_uniform(seed + 1, n).astype(np.float64) + 1.0) * 0.5
    u1 = np.clip(u1, 1e-7, 1.0)
    return (np.sqrt(-2.0 * np.log(u1)) * np.cos(2 * np.pi * u2)).astype(np.float32)
