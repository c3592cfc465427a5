"""Precomputed CLIP feature shards — the on-disk format the reference's caption trainers read
(source/gpt2_linear/data.py:16-62 `CocoClipFullTokensDataset`,
:92-107 `evaluate_cider`):

    tokens_dir/index.json    [{"shard": "<file>", "row": r}, ...]   one entry per sample
    tokens_dir/<file>        torch.save'd tensor [rows, L, D] (L = 257 CLIP ViT-L/14 tokens)

Reader: the same per-sample lookup (load the entry's shard, cache it while consecutive
samples stay in it, return row r), with `torch.load(weights_only=True)` and an optional
memory map, plus a batched gather and a pinned, one-batch-ahead device copy for the GPU
step.  Writer: the CLIP stage's output (gvl.clip.CLIPFeatureStage.tokens, or any [B, L, D]
tensors) into shards + index in that format, so features made here feed the reference's
own dataset and vice versa.  Caption tokenisation (tiktoken) is out of scope:
the dataset takes token ids, or an `encode(text) -> ids` callable.
"""
from __future__ import annotations

import json
import os
import random

import torch

INDEX = "index.json"


def encode_caption(ids, max_len: int, eot: int):
    """(x, y, mask) of one caption — gpt2_linear/data.py:35-49: ids[:max_len-1] + [eot],
    padded with eot to max_len; x = ids[:-1], y = ids[1:], mask[:max(L-1, 1)] = True."""
    ids = list(ids)
    if len(ids) == 0:
        ids = [eot]
    ids = ids[: max_len - 1] + [eot]
    L = len(ids)
    if L < max_len:
        ids = ids + [eot] * (max_len - L)
    t = torch.tensor(ids, dtype=torch.long)
    x, y = t[:-1], t[1:]
    mask = torch.zeros_like(y, dtype=torch.bool)
    mask[: max(L - 1, 1)] = True
    return x, y, mask


class FeatureShardWriter:
    """Append [B, L, D] feature batches; every `rows_per_shard` rows become one
    torch.save'd shard `prefix_{k:05d}.pt`; close() writes index.json."""

    def __init__(self, tokens_dir, rows_per_shard: int = 1024, prefix: str = "clip_tokens",
                 dtype=torch.float16):
        self.dir, self.rows, self.prefix, self.dtype = tokens_dir, int(rows_per_shard), prefix, dtype
        os.makedirs(tokens_dir, exist_ok=True)
        self.index, self.buf, self.nbuf, self.k = [], [], 0, 0

    def add(self, feats: torch.Tensor):
        feats = feats.detach().to("cpu", self.dtype)
        while feats.shape[0]:
            take = min(self.rows - self.nbuf, feats.shape[0])
            self.buf.append(feats[:take])
            self.nbuf += take
            feats = feats[take:]
            if self.nbuf == self.rows:
                self._flush()

    def _flush(self):
        if not self.nbuf:
            return
        name = f"{self.prefix}_{self.k:05d}.pt"
        shard = torch.cat(self.buf, 0).contiguous()
        tmp = os.path.join(self.dir, name + ".tmp")
        torch.save(shard, tmp)
        os.replace(tmp, os.path.join(self.dir, name))
        self.index += [{"shard": name, "row": r} for r in range(shard.shape[0])]
        self.buf, self.nbuf, self.k = [], 0, self.k + 1

    def close(self):
        self._flush()
        tmp = os.path.join(self.dir, INDEX + ".tmp")
        with open(tmp, "w") as f:
            json.dump(self.index, f)
        os.replace(tmp, os.path.join(self.dir, INDEX))
        return len(self.index)


class FeatureShards:
    """Per-sample reader of a tokens_dir (the lookup of gpt2_linear/data.py:55-62):
    z = shard(index[i]["shard"])[index[i]["row"]], with the current shard cached."""

    def __init__(self, tokens_dir, mmap: bool = True):
        self.dir = tokens_dir
        with open(os.path.join(tokens_dir, INDEX)) as f:
            self.index = json.load(f)
        self.mmap = mmap
        self._name, self._tensor = None, None

    def __len__(self):
        return len(self.index)

    def _shard(self, name):
        if name != self._name:
            path = os.path.join(self.dir, name)
            try:
                t = torch.load(path, map_location="cpu", weights_only=True, mmap=self.mmap)
            except RuntimeError:  # legacy (non-zip) serialisation cannot be memory-mapped
                t = torch.load(path, map_location="cpu", weights_only=True)
            if not torch.is_tensor(t):
                raise TypeError(f"{path}: expected a tensor shard, got {type(t).__name__}")
            self._name, self._tensor = name, t
        return self._tensor

    def __getitem__(self, idx):
        e = self.index[idx]
        return self._shard(e["shard"])[e["row"]]

    def gather(self, indices, out=None):
        """[len(indices), L, D] rows (grouped by shard, so each shard is opened once)."""
        indices = list(indices)
        first = self[indices[0]]
        if out is None:
            out = torch.empty((len(indices),) + tuple(first.shape), dtype=first.dtype)
        order = sorted(range(len(indices)), key=lambda j: (self.index[indices[j]]["shard"], j))
        for j in order:
            out[j].copy_(self[indices[j]])
        return out


class CaptionFeatureDataset(torch.utils.data.Dataset):
    """CocoClipFullTokensDataset without the COCO image decode: item i = (x, y, mask, z)
    with z from the feature shards and a caption drawn at random from captions[i]
    (token-id lists, or strings with `encode`)."""

    def __init__(self, tokens_dir, captions, max_len: int = 32, eot: int = 50256, encode=None,
                 seed=None):
        self.shards = FeatureShards(tokens_dir)
        self.captions, self.max_len, self.eot, self.encode = captions, max_len, eot, encode
        assert len(self.shards) == len(captions), "index.json length mismatch with captions"
        self.rng = random.Random(seed)

    def __len__(self):
        return len(self.shards)

    def __getitem__(self, idx):
        cap = self.rng.choice(self.captions[idx])
        ids = self.encode(cap) if isinstance(cap, str) else cap
        x, y, m = encode_caption(ids, self.max_len, self.eot)
        return x, y, m, self.shards[idx]


class CaptionFeatureLoader:
    """Batches of a CaptionFeatureDataset on the GPU: rows gathered into a pinned host
    buffer, copied on a side stream one batch ahead, CLIP tokens pooled to 33 on the device
    (gvl.caption.pool_clip_197_to_33_avg_with_cls) — yields (z33, x, y, mask, labels), the
    inputs of gvl.train's caption loss (labels = y.masked_fill(~mask, -100))."""

    def __init__(self, dataset, batch_size, device="cuda", shuffle=True, seed=0, drop_last=True,
                 pool=True):
        self.ds, self.B, self.dev, self.pool = dataset, int(batch_size), torch.device(device), pool
        self.shuffle, self.seed, self.drop_last = shuffle, seed, drop_last
        self.stream = torch.cuda.Stream(self.dev) if self.dev.type == "cuda" else None

    def _host(self, idx):
        items = [self.ds[i] for i in idx]
        x = torch.stack([t[0] for t in items])
        y = torch.stack([t[1] for t in items])
        m = torch.stack([t[2] for t in items])
        z = torch.stack([t[3] for t in items])
        if self.stream is not None:
            x, y, m, z = (t.pin_memory() for t in (x, y, m, z))
        return x, y, m, z

    def _to_dev(self, host):
        if self.stream is None:
            return host
        with torch.cuda.stream(self.stream):
            out = tuple(t.to(self.dev, non_blocking=True) for t in host)
        return out

    def __iter__(self):
        from .caption import pool_clip_197_to_33_avg_with_cls
        n = len(self.ds)
        order = list(range(n))
        if self.shuffle:
            random.Random(self.seed).shuffle(order)
        stop = n - n % self.B if self.drop_last else n
        batches = [order[i:i + self.B] for i in range(0, stop, self.B)]
        nxt = self._to_dev(self._host(batches[0])) if batches else None
        for k in range(len(batches)):
            cur = nxt
            if self.stream is not None:
                torch.cuda.current_stream(self.dev).wait_stream(self.stream)
                for t in cur:
                    t.record_stream(torch.cuda.current_stream(self.dev))
            nxt = self._to_dev(self._host(batches[k + 1])) if k + 1 < len(batches) else None
            x, y, m, z = cur
            if self.pool and z.shape[1] != 33:
                z = pool_clip_197_to_33_avg_with_cls(z)
            yield z, x, y, m, y.masked_fill(~m, -100)
