"""Data-parallel gradient exchange for the DP training loop (replaces the reference's
DDP wrapper, train_gpt2.py:270 / gpt2_linear/train.py:122, and its loss all-reduce :471).

Design (MI355X, one process per GPU, RCCL over xGMI via torch.distributed "nccl"):
  * gradients live in the optimizer's flat bf16 grad arena (gvl.optim.AdamW), so a
    bucket is a short list of contiguous arena slices (the decay and no-decay parts of the
    same layers): no flatten/unflatten copies;
  * buckets follow the order in which backward finalises gradients — the reverse of the
    module order (last block first), ~bucket_mb each — NOT the arena order (which is
    grouped by weight decay, so a bucket cut from the arena end would hold every layer's
    biases and could only fire at the very end of backward);
  * a post-accumulate-grad hook (or, for gradients the fused Functions accumulate in
    place, gvl.functional's grad-ready hook) marks parameters ready; on the sync micro-step
    the bucket's all-reduce (AVG) is launched on RCCL's own stream as soon as its last
    parameter is ready, so it overlaps the remaining backward.  For the deferred, batched
    block weight gradients this needs them flushed during backward, not once at its end:
    set_sync(True) turns gvl.functional.set_overlap_blocks on for that micro-step;
  * parameters that receive gradient from more than one place (the tied wte: lm_head and
    embedding) are final only at the end of backward: their bucket waits for wait();
  * wait() joins every outstanding bucket into the current stream before clip + AdamW;
  * only trainable parameters are in the arena: frozen caption decoders never move bytes.
A captured step (gvl.graph, world > 1) cannot hold collectives; it replays the backward in
segments (BackwardSegments) and launches the buckets each segment finalised between the
segment graphs (GradBuckets.capture_log / launch_logged).
On a gloo group (CPU tests) AVG is emulated as SUM then divide, synchronously.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

from . import functional as F

# GPT-2 blocks per in-backward flush of the deferred weight gradients on the sync micro-step
OVERLAP_BLOCKS = int(os.environ.get("GVL_DP_OVERLAP_BLOCKS", "4"))
# GVL_TRACE_BUCKETS=1: a roctx marker per bucket issue (rocprofv3 --marker-trace shows where
# each all-reduce enters the stream relative to the backward kernels)
TRACE = os.environ.get("GVL_TRACE_BUCKETS") == "1"


def _mark(name):
    if TRACE:
        torch.cuda.nvtx.mark(name)


def _is_nccl(pg):
    try:
        return dist.get_backend(pg) == "nccl"
    except Exception:
        return False


def _avg(t, pg, async_op):
    if _is_nccl(pg):
        return dist.all_reduce(t, op=dist.ReduceOp.AVG, group=pg, async_op=async_op)
    # gloo (CPU tests; GPU tensors in the two-ranks-on-one-GPU tests): its host-staged copy
    # of a device tensor is not reliably ordered behind kernels queued on the caller's stream
    # (measured: deferred weight gradients reduced before they were written), so the device
    # is drained around it — gloo is never the production path (RCCL is)
    if t.is_cuda:
        torch.cuda.synchronize(t.device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=pg)
    t.div_(dist.get_world_size(pg))
    if t.is_cuda:
        torch.cuda.synchronize(t.device)
    return None


def _runs(entries, align_end):
    """Merge (offset, numel) arena entries into maximal contiguous [start, end) slices
    (segments are padded to 8 elements; the pad is zero and rides along)."""
    out = []
    for off, n in sorted(entries):
        end = align_end(off, n)
        if out and out[-1][1] == off:
            out[-1][1] = end
        else:
            out.append([off, end])
    return [tuple(r) for r in out]


def tied_parameters(model):
    """Parameters registered under more than one name (the tied wte / lm_head)."""
    seen, tied = {}, set()
    for _, p in model.named_parameters(remove_duplicate=False):
        if id(p) in seen:
            tied.add(id(p))
        seen[id(p)] = p
    return tied


class GradBuckets:
    def __init__(self, optimizer, process_group=None, bucket_mb: float = 16.0, model=None,
                 force: bool = False, overlap_blocks: int = None):
        """`model` (optional) names the parameters whose gradient is final only at the end
        of backward (tied_parameters).  `force` runs the collectives even at world size 1
        (profiling the overlap on one GPU)."""
        from .optim import _pad
        self.opt = optimizer
        self.pg = process_group
        self.world = dist.get_world_size(process_group) if dist.is_initialized() else 1
        self.active = self.world > 1 or force
        self.overlap_blocks = OVERLAP_BLOCKS if overlap_blocks is None else overlap_blocks
        layout = optimizer.arena_layout()  # builds the arenas
        arena = optimizer.grad_arena
        limit = max(1, int(bucket_mb * 1024 * 1024 / arena.element_size()))
        late = tied_parameters(model) if model is not None else set()
        self.late = {p for p, _, _ in layout if id(p) in late or getattr(p, "_gvl_tied", False)}
        # backward finalises parameters in the reverse of the module order; the arena lists
        # them group by group, so without the model the (grouped) arena order is the proxy
        rank = ({id(p): i for i, p in enumerate(model.parameters())} if model is not None
                else {id(p): i for i, (p, _, _) in enumerate(layout)})
        order = sorted((e for e in layout if e[0] not in self.late),
                       key=lambda e: -rank.get(id(e[0]), -1))
        self.buckets = []  # (runs, params), first-ready first
        cur, size = [], 0
        for p, off, n in order:
            cur.append((p, off, n))
            size += n
            if size >= limit:
                self._add(cur, _pad)
                cur, size = [], 0
        if cur:
            self._add(cur, _pad)
        if self.late:
            self._add([(p, o, n) for p, o, n in layout if p in self.late], _pad)
        self._bucket_of = {p: bi for bi, (_, ps) in enumerate(self.buckets) for p in ps}
        self._pending = [len(ps) for _, ps in self.buckets]
        self._handles = []
        self.sync = True
        self.capture_log = None  # list: record bucket launches instead of issuing them
        self.launch_log = []     # bucket indices in launch order (tests / diagnostics)
        self._hooks = [p.register_post_accumulate_grad_hook(self._on_acc) for p, _, _ in layout]
        self._hooks.append(F.register_grad_ready_hook(self._on_fused))

    def _add(self, entries, pad):
        runs = _runs([(o, n) for _, o, n in entries], lambda o, n: o + pad(n))
        self.buckets.append((runs, [p for p, _, _ in entries]))

    def _launch(self, bi):
        self._pending[bi] = -1
        if self.capture_log is not None:
            self.capture_log.append(bi)
            return
        self.launch_log.append(bi)
        _mark(f"gvl.bucket{bi}")
        for s, e in self.buckets[bi][0]:
            h = _avg(self.opt.grad_arena[s:e], self.pg, async_op=True)
            if h is not None:
                self._handles.append(h)

    def launch_logged(self, indices):
        """Issue the all-reduces of buckets recorded during a capture (gvl.graph replay)."""
        for bi in indices:
            self.launch_log.append(bi)
            _mark(f"gvl.bucket{bi}")
            for s, e in self.buckets[bi][0]:
                h = _avg(self.opt.grad_arena[s:e], self.pg, async_op=True)
                if h is not None:
                    self._handles.append(h)

    def _on_grad(self, p):
        if not self.sync or not self.active or p in self.late:
            return
        bi = self._bucket_of.get(p)
        if bi is None or self._pending[bi] < 0:
            return
        self._pending[bi] -= 1
        if self._pending[bi] == 0:
            self._launch(bi)

    def _on_acc(self, p):
        # AccumulateGrad also runs (gradient-less) for parameters a fused unit sank in place:
        # those are counted by the unit's own ready notification (_on_fused) only
        if F.sunk_in_this_backward(p):
            return
        self._on_grad(p)

    def _on_fused(self, p):
        if p in self._bucket_of:
            self._on_grad(p)

    def set_sync(self, flag: bool):
        """Enable the all-reduce for the coming backward (the last micro-step)."""
        self.sync = flag
        self._pending = [len(ps) for _, ps in self.buckets]
        F.set_overlap_blocks(self.overlap_blocks if (flag and self.active) else 0)

    def pending_buckets(self):
        return [bi for bi, left in enumerate(self._pending) if left >= 0]

    def wait(self):
        """Join outstanding buckets; buckets whose hooks did not all fire (tied or unused
        params) are reduced here so every rank ends with identical gradients."""
        F.set_overlap_blocks(0)
        if not self.active:
            return
        if self.sync:
            for bi in self.pending_buckets():
                self._launch(bi)
        if self.capture_log is not None:
            return
        self.join()

    def join(self):
        """Make the current stream wait for every issued bucket."""
        for h in self._handles:
            h.wait()
        self._handles = []

    def remove(self):
        for h in self._hooks:
            h.remove()


class BackwardSegments:
    """Backward in segments for a captured data-parallel step.

    Forward pre-hooks on the `cuts` modules replace each one's first input by a detached
    leaf while armed (arm()); backward(loss) then runs loss.backward() (head + the top
    segment) and one x.backward(leaf.grad) per cut, top to bottom, calling between(j) after
    segment j.  Each segment's deferred weight gradients flush at its own end (the engine's
    final callback), so the buckets it completes are known between segments — a hipGraph per
    segment can be replayed with their all-reduces launched in between (gvl.graph)."""

    def __init__(self, cuts):
        self.cuts = list(cuts)
        self.armed = False
        self._saved = []
        self._hooks = [m.register_forward_pre_hook(self._pre) for m in self.cuts]

    def _pre(self, mod, args):
        if not self.armed or not torch.is_grad_enabled():
            return None
        pairs, new, leaf_of = [], [], {}
        for a in args:  # every differentiable input of the cut (the Q-Former layer's queries
            #             AND the projected image tokens both layers read)
            if torch.is_tensor(a) and a.requires_grad:
                if id(a) not in leaf_of:
                    leaf_of[id(a)] = a.detach().requires_grad_(True)
                    pairs.append((a, leaf_of[id(a)]))
                a = leaf_of[id(a)]
            new.append(a)
        if not pairs:
            return None
        self._saved.append(pairs)
        return tuple(new)

    def arm(self, flag=True):
        self.armed = flag
        if flag:
            self._saved = []

    def backward(self, loss, between=None):
        """loss.backward() then the segments below each cut, top to bottom; returns the
        number of segments.  A cut module must consume its inputs entirely (no residual
        around it): GPT-2 blocks and Q-Former layers add their residuals inside."""
        saved, self._saved = self._saved, []
        self.armed = False
        loss.backward()
        # An input read by several cuts (the projected image tokens every Q-Former layer reads)
        # is back-propagated once, from the lowest cut that reads it, with the gradients of
        # every cut above summed into it: back-propagating it per segment would run its
        # producer's backward (vis_proj) in two graph tasks, so its bucket would count as final
        # (and be all-reduced) before the second partial gradient landed.
        lowest = {}
        for j, pairs in enumerate(saved):
            for x, _ in pairs:
                lowest.setdefault(id(x), j)
        carry = {}
        for j in range(len(saved) - 1, -1, -1):
            if between is not None:
                between(len(saved) - 1 - j)
            outs = []
            for x, leaf in saved[j]:
                g = leaf.grad
                if id(x) in carry:
                    c = carry.pop(id(x))
                    g = c if g is None else g + c
                if g is None:
                    continue
                if lowest[id(x)] < j:
                    carry[id(x)] = g
                else:
                    outs.append((x, g))
            if outs:
                torch.autograd.backward([x for x, _ in outs], [g for _, g in outs])
        return len(saved) + 1

    def remove(self):
        for h in self._hooks:
            h.remove()


def segment_cuts(model, blocks_per_segment: int = None):
    """Default cut modules for BackwardSegments: every `blocks_per_segment`-th GPT-2 block
    of a trainable decoder (LM), the Q-Former layers after the first (Q-Former bridge);
    none for models whose trainable gradients all finalise at the end of backward."""
    g = OVERLAP_BLOCKS if blocks_per_segment is None else blocks_per_segment
    tr = getattr(model, "transformer", None)
    if tr is not None and hasattr(tr, "h") and not hasattr(tr.h[0], "xattn"):
        if any(p.requires_grad for p in tr.h.parameters()) and g > 0:
            n = len(tr.h)
            return [tr.h[i] for i in range(n - g, 0, -g)][::-1]
        return []
    bridge = getattr(model, "bridge", None)
    if bridge is not None and hasattr(bridge, "layers"):
        return list(bridge.layers)[1:]
    return []


def close_graphed_steps(group=None):
    """Close every live gvl.graph.GraphedStep (all of them, or those bound to `group`)."""
    from .graph import live_steps
    for st in live_steps():
        if group is None or st.pg is group or st.pg is None:
            st.close()


def destroy_process_group(group=None):
    """The reference scripts' teardown (train_gpt2.py:523, gpt2_linear/train.py:372,
    gpt2_cross-att/train.py:348) with gvl's captured steps released first.

    Order: close every live GraphedStep (joins its last replay's bucket work, drains the
    device, resets its graphs and memory pool), drain the device, then destroy the
    communicator.  Nothing of a captured step outlives the process group it was replayed
    against, whatever the caller's garbage-collection order."""
    close_graphed_steps(group)
    if torch.cuda.is_available() and torch.cuda.is_initialized():
        torch.cuda.synchronize()
    if dist.is_initialized():
        dist.destroy_process_group(group)


def all_reduce_mean_(t, group=None):
    """The per-step scalar loss all-reduce (C3)."""
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        _avg(t, group, async_op=False)
    return t
