"""Data-parallel gradient exchange for the DP training loop (replaces the reference's
DDP wrapper, train_gpt2.py:270 / gpt2_linear/train.py:122, and its loss all-reduce :471).

Design (MI355X, one process per GPU, RCCL over xGMI via torch.distributed "nccl"):
  * gradients live in the optimizer's flat bf16 grad arena (gvl.optim.AdamW), so a
    bucket is a plain contiguous slice: no flatten/unflatten copies;
  * buckets are cut from the END of the arena (last layers first, matching the order in
    which backward produces gradients), ~bucket_mb each;
  * a post-accumulate-grad hook (or, for gradients the fused Functions accumulate in
    place, gvl.functional's grad-ready hook) marks parameters ready; on the sync micro-step the
    bucket's all-reduce (AVG) is launched as soon as its last parameter is ready, so it
    overlaps the remaining backward on RCCL's own stream;
  * wait() joins every outstanding bucket into the current stream before clip + AdamW;
  * only trainable parameters are in the arena: frozen caption decoders never move bytes.
On a gloo group (CPU tests) AVG is emulated as SUM then divide, synchronously.
"""
from __future__ import annotations

import torch.distributed as dist

from . import functional as F


def _is_nccl(pg):
    try:
        return dist.get_backend(pg) == "nccl"
    except Exception:
        return False


def _avg(t, pg, async_op):
    if _is_nccl(pg):
        return dist.all_reduce(t, op=dist.ReduceOp.AVG, group=pg, async_op=async_op)
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=pg)
    t.div_(dist.get_world_size(pg))
    return None


class GradBuckets:
    def __init__(self, optimizer, process_group=None, bucket_mb: float = 16.0):
        self.opt = optimizer
        self.pg = process_group
        self.world = dist.get_world_size(process_group) if dist.is_initialized() else 1
        layout = optimizer.arena_layout()  # builds the arenas
        arena = optimizer.grad_arena
        limit = max(1, int(bucket_mb * 1024 * 1024 / arena.element_size()))
        self.buckets = []  # (start, end, params) — contiguous arena slices, last layers first
        end, cur = arena.numel(), []
        for p, off, _ in reversed(layout):
            cur.append(p)
            if end - off >= limit or off == 0:
                self.buckets.append((off, end, cur))
                end, cur = off, []
        self._bucket_of = {p: bi for bi, (_, _, ps) in enumerate(self.buckets) for p in ps}
        self._pending = [len(ps) for _, _, ps in self.buckets]
        self._handles = []
        self.sync = True
        self._hooks = [p.register_post_accumulate_grad_hook(self._on_grad) for p, _, _ in layout]
        self._hooks.append(F.register_grad_ready_hook(self._on_fused))

    def _launch(self, bi):
        s, e, _ = self.buckets[bi]
        h = _avg(self.opt.grad_arena[s:e], self.pg, async_op=True)
        if h is not None:
            self._handles.append(h)
        self._pending[bi] = -1

    def _on_grad(self, p):
        if not self.sync or self.world == 1:
            return
        bi = self._bucket_of[p]
        self._pending[bi] -= 1
        if self._pending[bi] == 0:
            self._launch(bi)

    def _on_fused(self, p):
        if p in self._bucket_of:
            self._on_grad(p)

    def set_sync(self, flag: bool):
        """Enable the all-reduce for the coming backward (the last micro-step)."""
        self.sync = flag
        self._pending = [len(ps) for _, _, ps in self.buckets]

    def wait(self):
        """Join outstanding buckets; buckets whose hooks did not all fire (unused params)
        are reduced here so every rank ends with identical gradients."""
        if self.world == 1:
            return
        if self.sync:
            for bi, left in enumerate(self._pending):
                if left >= 0:
                    self._launch(bi)
        for h in self._handles:
            h.wait()
        self._handles = []

    def remove(self):
        for h in self._hooks:
            h.remove()


def all_reduce_mean_(t, group=None):
    """The per-step scalar loss all-reduce (C3)."""
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        _avg(t, group, async_op=False)
    return t
