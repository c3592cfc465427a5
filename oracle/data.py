"""DataLoaderLite restated (TEST INFRASTRUCTURE): source/gpt2/train_gpt2.py:148-187, literally,
on numpy token arrays (no torch, no mmap) — the checker for gvl.data.DataLoaderLite."""
from __future__ import annotations

import os

import numpy as np


def windows(data_root, split, B, T, rank, world, n_batches):
    """The first n_batches (x, y) pairs rank `rank` draws (train_gpt2.py:171-187)."""
    shards = sorted(s for s in os.listdir(data_root) if split in s)
    shards = [os.path.join(data_root, s) for s in shards]
    cur = 0
    tokens = np.load(shards[cur]).astype(np.int32).astype(np.int64)
    pos = B * T * rank
    out = []
    for _ in range(n_batches):
        buf = tokens[pos:pos + B * T + 1]
        out.append((buf[:-1].reshape(B, T), buf[1:].reshape(B, T)))
        pos += B * T * world
        if pos + (B * T * world + 1) > len(tokens):
            cur = (cur + 1) % len(shards)
            tokens = np.load(shards[cur]).astype(np.int32).astype(np.int64)
            pos = B * T * rank
    return out
