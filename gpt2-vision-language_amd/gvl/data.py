"""FineWeb token-shard loader, validation loss and the HellaSwag scorer.

Semantics restated from source/gpt2/train_gpt2.py:148-202:
  * shards: every file in the data root whose name contains the split, sorted; a shard is a
    .npy of token ids (load_tokens: int32 -> int64);
  * DataLoaderLite windows: rank r starts at B*T*r; a batch is buf = tokens[pos : pos+B*T+1],
    x = buf[:-1].view(B, T), y = buf[1:].view(B, T); pos += B*T*world; when the next window
    would run past the shard (pos + B*T*world + 1 > len), move to the next shard (cyclic)
    and restart at B*T*r;
  * val loss: mean of `steps` batch losses after reset(), AVG-all-reduced (train_gpt2.py:
    338-354);
  * get_most_likely_row: per-ending masked mean CE of the shifted tokens, argmin (:190-202).

MI355X side: shards are memory-mapped (a 100M-token shard is not read whole), a batch is
copied into a pinned host buffer and moved to the device on a side stream one batch ahead,
so the copy of batch i+1 overlaps the step that consumes batch i.
"""
from __future__ import annotations

import os

import numpy as np
import torch


def load_tokens(filename, mmap=True):
    """train_gpt2.py:148-151 (int32 -> int64); memory-mapped when mmap."""
    npt = np.load(filename, mmap_mode="r" if mmap else None)
    return npt


def list_shards(data_root, split):
    assert split in {"train", "val"}
    shards = sorted(s for s in os.listdir(data_root) if split in s)
    assert len(shards) > 0, f"no shards found for split {split}"
    return [os.path.join(data_root, s) for s in shards]


class DataLoaderLite:
    """Drop-in for train_gpt2.py:154-187 (same constructor, reset(), next_batch()).

    device=None returns int64 CPU tensors like the reference; device='cuda' returns device
    tensors, prefetched one batch ahead through pinned memory on a side stream."""

    def __init__(self, B, T, process_rank, num_processes, split, data_root=None, device=None,
                 verbose=False):
        self.B, self.T = B, T
        self.process_rank = process_rank
        self.num_processes = num_processes
        root = data_root or os.environ.get("FW_OUT_DIR", "edu_fineweb10B")
        self.shards = list_shards(root, split)
        if verbose:
            print(f"found {len(self.shards)} shards for split {split}")
        self.device = torch.device(device) if device is not None else None
        self._stream = None
        self._pinned = None
        self._ahead = None
        self.reset()

    # -------------------------------------------------------------- host windows
    def reset(self):
        self.current_shard = 0
        self.tokens = load_tokens(self.shards[self.current_shard])
        self.current_position = self.B * self.T * self.process_rank
        self._ahead = None

    def _next_window(self):
        B, T = self.B, self.T
        p = self.current_position
        buf = np.asarray(self.tokens[p:p + B * T + 1]).astype(np.int64)
        self.current_position += B * T * self.num_processes
        if self.current_position + (B * T * self.num_processes + 1) > len(self.tokens):
            self.current_shard = (self.current_shard + 1) % len(self.shards)
            self.tokens = load_tokens(self.shards[self.current_shard])
            self.current_position = B * T * self.process_rank
        return buf

    # ------------------------------------------------------------ device prefetch
    def _stage(self):
        """Copy the next window into a pinned slot and launch its H2D copy on the side
        stream; returns (x, y, event) on the device."""
        buf = self._next_window()
        n = buf.shape[0]
        if self._pinned is None:
            self._pinned = [torch.empty(n, dtype=torch.int64).pin_memory() for _ in range(2)]
            self._copied = [None, None]
            self._slot = 0
            self._stream = torch.cuda.Stream(device=self.device)
        slot = self._slot
        self._slot ^= 1
        if self._copied[slot] is not None:
            self._copied[slot].synchronize()  # the slot's previous H2D copy has read it
        host = self._pinned[slot]
        host.copy_(torch.from_numpy(buf))
        with torch.cuda.stream(self._stream):
            dev = host.to(self.device, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self._stream)
        self._copied[slot] = ev
        B, T = self.B, self.T
        return dev[:-1].view(B, T), dev[1:].view(B, T), ev, dev

    def next_batch(self):
        if self.device is None or self.device.type != "cuda":
            buf = torch.from_numpy(self._next_window())
            return buf[:-1].view(self.B, self.T), buf[1:].view(self.B, self.T)
        cur = self._ahead if self._ahead is not None else self._stage()
        self._ahead = self._stage()  # the next copy overlaps this batch's step
        x, y, ev, dev = cur
        torch.cuda.current_stream(self.device).wait_event(ev)
        dev.record_stream(torch.cuda.current_stream(self.device))
        return x, y


@torch.no_grad()
def evaluate_val_loss(model, loader, steps=20, process_group=None):
    """train_gpt2.py:338-354: reset, mean of `steps` batch losses, AVG over ranks."""
    from .dist import all_reduce_mean_
    was_training = model.training
    model.eval()
    loader.reset()
    acc = None
    for _ in range(steps):
        x, y = loader.next_batch()
        _, loss = model(x, y)
        loss = loss.detach().float() / steps
        acc = loss if acc is None else acc + loss
    all_reduce_mean_(acc, process_group)
    model.train(was_training)
    return acc


def get_most_likely_row(tokens, mask, logits):
    """train_gpt2.py:190-202: index of the ending with the lowest masked mean CE of the
    shifted tokens.  tokens/mask [E, T], logits [E, T, V]."""
    import torch.nn.functional as F
    shift_logits = logits[..., :-1, :].contiguous().float()
    shift_tokens = tokens[..., 1:].contiguous()
    losses = F.cross_entropy(shift_logits.view(-1, shift_logits.size(-1)), shift_tokens.view(-1),
                             reduction="none").view(tokens.size(0), -1)
    shift_mask = mask[..., 1:].contiguous()
    avg = (losses * shift_mask).sum(dim=1) / shift_mask.sum(dim=1)
    return int(avg.argmin().item())
