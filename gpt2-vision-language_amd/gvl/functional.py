"""Autograd Functions over the libgvl kernels — the fused units the drop-in modules call.

Granularity follows the MI355X design: one Function per GPT-2 block (so
DDP-style gradient buckets become ready block by block during backward), fused
MHA / MLP / gated cross-attention units for the bridges, and a fused lm_head +
cross-entropy.  Frozen parameters (requires_grad=False, the caption setting) skip their
weight-gradient GEMMs entirely via ctx.needs_input_grad.
"""
from __future__ import annotations

import math
import os

import torch

from . import kernels as K

BF16 = torch.bfloat16
ATT_SCALE = 1.0 / math.sqrt(64.0)


def bf(t):
    """Parameters are bf16 on the GPU path (the reference runs model.to(bfloat16));
    fp32 parameters are cast per call, as autocast would."""
    if t is None:
        return None
    return t if t.dtype == BF16 else t.to(BF16)


def new_seed():
    return int(torch.randint(1, 2**62, (1,)).item())


def _off(t, p):
    """Device dropout step offset (gvl.kernels.seed_offset) for a dropout site, else None."""
    return K.seed_offset(t.device) if p > 0 else None


def _need(ctx, i):
    return ctx.needs_input_grad[i]


# ------------------------------------------------------------------- index checks
# nn.Embedding and F.cross_entropy raise on an id / class index outside the table
# (train_gpt2.py:114-124).  The kernels never read outside their rows whatever the ids
# (include/gvl.h ABI v3), and this host-side check raises like torch does.  It reads one
# device scalar (a sync), so it is skipped inside a hipGraph capture (gvl.graph) and can be
# turned off with GVL_CHECK_IDS=0.
CHECK_IDS = os.environ.get("GVL_CHECK_IDS", "1") != "0"
# The first SYNC_CHECKS checks of a process block on the result (an error raises at the op,
# like torch).  Later ones stay asynchronous: the device-side verdict is copied into pinned
# host memory behind an event, and every later call polls the completed verdicts without
# synchronising, so a bad id raises IndexError one or a few calls after the op that read it
# (the kernels never read outside their rows meanwhile).  GVL_CHECK_IDS=2: always synchronous.
SYNC_CHECKS = 1 << 60 if os.environ.get("GVL_CHECK_IDS") == "2" else 16
_ID_CHECKS = [0]
_ID_INFLIGHT = []  # (pinned bool, event, what, n)


def _poll_id_checks():
    while _ID_INFLIGHT and _ID_INFLIGHT[0][1].query():
        flag, _, what, n = _ID_INFLIGHT.pop(0)
        if bool(flag[0]):
            _ID_INFLIGHT.clear()
            raise IndexError(f"gvl: {what} out of range [0, {n}) (detected asynchronously)")


def check_index_range(t, n, what, ignore_index=None):
    if not CHECK_IDS or t.numel() == 0 or (t.is_cuda and torch.cuda.is_current_stream_capturing()):
        return
    bad = (t < 0) | (t >= n)
    if ignore_index is not None:
        bad &= t != ignore_index
    _ID_CHECKS[0] += 1
    if not t.is_cuda or _ID_CHECKS[0] <= SYNC_CHECKS:
        if bool(bad.any()):
            lo, hi = int(t.min()), int(t.max())
            raise IndexError(f"gvl: {what} out of range [0, {n}) (min {lo}, max {hi})")
        return
    _poll_id_checks()
    flag = torch.empty(1, dtype=torch.bool, pin_memory=True)
    flag.copy_(bad.any().view(1), non_blocking=True)
    ev = torch.cuda.Event()
    ev.record()
    _ID_INFLIGHT.append((flag, ev, what, n))


def pad_vocab(w):
    """(weight padded with zero rows to a multiple of 8, true vocab).  GPTConfig()'s default
    vocab of 50257 (train_gpt2.py:79) is not a multiple of the GEMM's 8-column store; the
    logits GEMM runs on the padded table and the CE kernel masks the pad columns.  The
    reference trains with 50304, where this is the identity."""
    V = w.shape[0]
    if V % 8 == 0:
        return w, V
    return torch.cat([w, w.new_zeros((8 - V % 8, w.shape[1]))], 0), V


# ------------------------------------------------------- fused gradient accumulation
# With gradient accumulation the reference lets autograd add every micro-step's weight
# gradient into .grad (one extra read-modify-write pass per parameter per micro-step).
# Here a parameter whose .grad is a view of a gvl.optim.AdamW arena (bf16, its shape) is a
# "sink": the weight-gradient GEMM adds into it in its epilogue (C = dY^T X + C), bias and
# LayerNorm gradients use their kernels' accumulate flag, and the Function returns None for
# that input.  AccumulateGrad then never runs for it, so _ready() notifies the
# data-parallel bucketing (gvl.dist) in its place.  The tied wte (embedding + lm_head) sinks
# both uses into its one arena gradient (LMHeadLossFn's GEMM epilogue, EmbedFn's row update).
FUSE_GRAD_ACC = True
# MLP GELU: the forward epilogue stores gelu'(x) instead of x (GEMM act 3/4) and the backward
# multiplies by it (dact 3), so the dX epilogue runs no transcendentals.  0 (GVL_GELU_DERIV=0)
# stores x and recomputes gelu'(x) in the dX epilogue (act 1/2, dact 1/2).
GELU_DERIV = 0 if os.environ.get("GVL_GELU_DERIV", "1") == "0" else 2
_READY_HOOKS = []
# Deferred weight gradients: a sunk nn.Linear weight gradient (dY^T X added into .grad) and
# bias gradient (column sums of dY) are queued instead of launched, and at the end of the backward pass (an autograd engine final
# callback) the queue runs as one batched persistent GEMM per shape (gvl_gemm_batched): the
# 12 GPT-2 blocks' c_attn / attn.c_proj / c_fc / mlp.c_proj weight gradients (K = the
# micro-step's 16k tokens) are 9-36 output tiles each — alone they need a K split with fp32
# slabs and a reduce kernel to fill the chip, batched they fill it with whole-K tiles; the 48
# bias column sums (96 small launches) become 4 launch pairs (gvl_colsum_batched).
# The per-block units repeated 12 times defer (GPTBlockFn, CrossAttnFn) and are flushed as
# batched launches per shape.  The bridge units (MLPFn, MHAFn's out_proj, LinearFn) defer too
# (GVL_DEFER_BRIDGE, round 4): their few problems of different shapes are flushed as ONE grouped
# launch (gvl_gemm_grouped) with the bias sums fused, instead of one split-K launch + reduce +
# column-sum pair each (round 2 measured plain deferral of the bridge 0.5 % slower: per-shape
# batches of 2 problems underfill the chip).  GVL_DEFER_WGRAD=0 launches each one in place.
DEFER_WGRAD = os.environ.get("GVL_DEFER_WGRAD", "1") != "0"
DEFER_BRIDGE = os.environ.get("GVL_DEFER_BRIDGE", "1") != "0"
DEFER_INPROJ = os.environ.get("GVL_DEFER_INPROJ", "1") != "0"  # MHAFn's packed in_proj slices too
# The tied lm_head's weight gradient (dlogits^T x, scaled by the device scalar dloss / count) is
# queued too (round 5), so the LM flush can group it with the blocks' (_flush_grouped)
DEFER_LMHEAD = os.environ.get("GVL_DEFER_LMHEAD", "1") != "0"
# LayerNorm weight / bias gradients (round 5, ABI v12): the backward leaves its per-block column
# partials in a workspace and the flush reduces all of them in one launch
# (gvl_layernorm_bwd_finalize_batched) instead of one finalize launch per LayerNorm
DEFER_LN = os.environ.get("GVL_DEFER_LN", "1") != "0"
# The cross-att tanh gate's gradient added into its bf16 grad by the gate kernel itself (ABI v13)
# instead of an fp32 zero-fill + kernel + cast + autograd add per block (GVL_GATE_SINK=0: A/B)
GATE_SINK = os.environ.get("GVL_GATE_SINK", "1") != "0"
# Grouped flush (gvl_gemm_grouped) of the queued weight gradients of one stream over <= 8192
# tokens: 2 (default) up to 48 problems (the cross-att decoder's 12 blocks' flush: +1.9 % on its
# step, profiles/r4/grouped48_r4g48.txt), 1 up to 16 (the Q-Former bridge's), 0 off.  The LM's
# K = 16384 flushes stay per-shape batches: all 48 of them as one grouped launch measured 3070
# vs 2942 us and the LM step 924k vs 933.6k tokens/s (same box).
GROUPED_WGRAD = int(os.environ.get("GVL_GROUPED_WGRAD", "2"))
GROUPED_MAX = 48
# Queue entries are tagged with the autograd graph task that produced them, and every task
# that defers queues its OWN end-of-backward flush, which runs only that task's entries: two
# backward passes (two models, two threads, a nested reentrant backward) never consume each
# other's gradients, and a backward that raises (its final callbacks never run) cannot
# switch deferral off for later passes.  Its stale entries are dropped by discard_pending(),
# which gvl.optim.AdamW.zero_grad calls.  Peak memory: the queued (dY, X) operands stay alive
# until the flush.
_PENDING = []          # (task, param, grad sink, dy2, x2, stream, alpha_ptr or None)
_PENDING_B = []        # (task, param, grad sink, dy2, stream): bias gradients = column sums of dy2
_PENDING_LN = []       # (task, w, b, grad sink w or None, grad sink b or None, workspace, blocks, cols, stream)
_QUEUED = set()        # graph tasks with a flush callback queued
# Data-parallel overlap (gvl.dist.GradBuckets sets it for the synchronising micro-step):
# with OVERLAP_BLOCKS[0] = G > 0 every G-th GPT-2 block backward flushes its task's queue in
# place, so the gradients of the top blocks become final — and their all-reduce buckets
# launch — while the lower blocks' backward is still running (train_gpt2.py:468-469, DDP's
# bucketed reducer).  0: one flush at the end of backward (largest batched launches).
OVERLAP_BLOCKS = [0]
_BLOCKS_SEEN = {}      # task -> GPT-2 blocks deferred since that task's last flush


def _task():
    return torch._C._current_graph_task_id()


def set_overlap_blocks(g: int):
    """Flush deferred weight gradients every `g` GPT-2 blocks during backward (0: at the end)."""
    OVERLAP_BLOCKS[0] = max(0, int(g))


def discard_pending():
    """Drop every queued deferred gradient (left behind by a backward that raised)."""
    _PENDING.clear()
    _PENDING_B.clear()
    _PENDING_LN.clear()
    _QUEUED.clear()
    _BLOCKS_SEEN.clear()


def _take(lst, task):
    if task is None:
        out = list(lst)
        lst.clear()
        return out
    out = [e for e in lst if e[0] == task]
    if out:
        lst[:] = [e for e in lst if e[0] != task]
    return out


def _dkey(d):
    return (d.data_ptr(), tuple(d.shape), d.stride(0))


def flush_wgrads(task=None):
    """Run the queued weight gradients of graph task `task` (every task when None) batched by
    shape, then notify the grad-ready hooks.  Runs by itself at the end of every backward pass
    that queued any; harmless when empty."""
    pend = [e[1:] for e in _take(_PENDING, task)]
    pend_b = [e[1:] for e in _take(_PENDING_B, task)]
    pend_ln = [e[1:] for e in _take(_PENDING_LN, task)]
    _BLOCKS_SEEN.pop(task, None)
    # a parameter may have several queued entries (the packed in_proj's row slices): its
    # grad-ready hook runs once, after the last of them is launched
    left = {}
    for e in pend + pend_b:
        left[id(e[0])] = left.get(id(e[0]), 0) + 1
    for w, b, gw, gb, *_ in pend_ln:
        for p, g in ((w, gw), (b, gb)):
            if g is not None:
                left[id(p)] = left.get(id(p), 0) + 1

    def _done(p):
        left[id(p)] -= 1
        if left[id(p)] == 0:
            _ready(p)

    if pend_ln:
        lgroups = {}
        for w, b, gw, gb, ws, nblk, cols, st in pend_ln:
            lgroups.setdefault((cols, st), []).append((w, b, gw, gb, ws, nblk))
        for (cols, st), its in lgroups.items():
            with torch.cuda.stream(st):
                K.layernorm_finalize_batched([(ws, nblk, gw, gb) for _, _, gw, gb, ws, nblk in its],
                                             cols, accumulate=True)
            for w, b, gw, gb, _, _ in its:
                if gw is not None:
                    _done(w)
                if gb is not None:
                    _done(b)

    # a bias gradient over the same dY as a queued weight gradient rides in that batched GEMM
    # (gvl_gemm_batched_dbias: row sums of dY^T from the same operand tiles); each bias pairs
    # with ONE weight gradient (popped when used), so a dY shared by two weight gradients
    # never gets its bias fused twice
    paired = {}
    rest_b = []
    if pend_b and pend:
        wkeys = {_dkey(d) for _, _, d, _, _, _ in pend}
        for p, g, dy2, st in pend_b:
            k = _dkey(dy2)
            if k in wkeys and k not in paired:
                paired[k] = (p, g)
            else:
                rest_b.append((p, g, dy2, st))
    else:
        rest_b = pend_b
    groups = {}
    for p, g, dy2, x2, st, ap in pend:
        # key[-2]: the device scale of the problem (the tied lm_head's, else None), key[-1]: stream
        key = (tuple(dy2.shape), dy2.stride(0), tuple(x2.shape), x2.stride(0), g.stride(0),
               dy2.device, ap, st)
        groups.setdefault(key, []).append((p, g, dy2, x2))
    if GROUPED_WGRAD and len(groups) >= 2:
        groups = _flush_grouped(groups, paired, _done)
    order = list(groups.items())
    ready = []
    for key, items in order:
        with torch.cuda.stream(key[-1]):
            if key[-2] is not None:  # scaled by a device scalar: one launch each
                for p, g, dy2, x2 in items:
                    K.gemm(dy2, x2, a_mn=True, b_mn=True, alpha_ptr=key[-2], out=g, residual=g)
                    ready.append(p)
                items = []
            for i in range(0, len(items), 16):
                chunk = items[i:i + 16]
                bias = [paired.pop(_dkey(d), None) for _, _, d, _ in chunk]
                fused = all(b is not None for b in bias) and K.gemm_batched(
                    [(dy2, x2, g, True) for _, g, dy2, x2 in chunk], a_mn=True, b_mn=True,
                    dbias=[b[1] for b in bias])
                if not fused:
                    K.gemm_batched([(dy2, x2, g, True) for _, g, dy2, x2 in chunk], a_mn=True,
                                   b_mn=True)
                    for (_, _, d, _), b in zip(chunk, bias):
                        if b is not None:
                            rest_b.append((b[0], b[1], d, key[-1]))
                ready += [p for p, *_ in chunk]
                if fused:
                    ready += [b[0] for b in bias]
        for p in ready:
            _done(p)
        ready = []
    for k, (p, g) in paired.items():  # (unreachable unless a weight entry vanished)
        raise RuntimeError(f"gvl: unpaired deferred bias gradient {k}")
    if rest_b:
        bgroups = {}
        for p, g, dy2, st in rest_b:
            bgroups.setdefault((tuple(dy2.shape), dy2.stride(0), dy2.device, st), []).append((p, g, dy2))
        for key, items in bgroups.items():
            with torch.cuda.stream(key[-1]):
                for i in range(0, len(items), 16):
                    chunk = items[i:i + 16]
                    K.colsum_batched([d for _, _, d in chunk], [g for _, g, _ in chunk],
                                     accumulate=True)
                    for p, *_ in chunk:
                        _done(p)


_CUS = {}


def _num_cus(dev):
    if dev not in _CUS:
        _CUS[dev] = torch.cuda.get_device_properties(dev).multi_processor_count
    return _CUS[dev]


def _tiles256(its):
    """256 x 256 output tiles of one problem of a shape group (dW [M, N] = dY^T X)."""
    _, _, dy2, x2 = its[0]
    return -(-dy2.shape[1] // 256) * -(-x2.shape[1] // 256)


def _flush_grouped(groups, paired, done):
    """Queued weight gradients of one stream as one grouped launch (gvl_gemm_grouped); returns
    the groups left to the per-shape path.
    * Flushes over <= 8192 tokens (the caption steps): all of them, at most GROUPED_MAX
      (GROUPED_WGRAD 1: 16).
    * Larger ones (the LM's 16k-token micro-step, GROUPED_WGRAD 2): the shapes of >= 16 tiles per
      problem (c_attn, c_fc, mlp.c_proj and the tied lm_head's dW, scaled by its device scalar),
      when one launch over all their tiles takes fewer whole rounds of CUs than the per-shape
      launches (each a whole number of rounds; under one round they split K), counting the
      grouped launch's tiles 10 % slower (profiles/r5/lm_wgrad_grouped_r5k.txt: 3713 vs 3966 us
      for the 37 problems).  The small attn.c_proj problems keep their split-K batch."""
    if len({key[-1] for key in groups}) != 1:
        return groups
    items = [it for its in groups.values() for it in its]
    if all(it[2].shape[0] <= 8192 for it in items):
        if len(items) > (GROUPED_MAX if GROUPED_WGRAD >= 2 else 16):
            return groups
        sel = groups
    else:
        if GROUPED_WGRAD < 2:
            return groups
        sel = {k: its for k, its in groups.items() if _tiles256(its) >= 16}
        n = sum(len(its) for its in sel.values())
        if len(sel) < 2 or n > GROUPED_MAX:
            return groups
        cus = _num_cus(items[0][2].device)
        sep = 0.0
        for its in sel.values():
            t = _tiles256(its) * len(its)
            sep += t / cus if t < cus else -(-t // cus)
        tot = -(-sum(_tiles256(its) * len(its) for its in sel.values()) // cus)
        if tot * 1.1 >= sep:
            return groups
    entries = [(it, key[-2]) for key, its in sel.items() for it in its]
    bias = [paired.pop(_dkey(it[2]), None) for it, _ in entries]
    with torch.cuda.stream(next(iter(groups))[-1]):
        ok = K.gemm_grouped([(dy2, x2, g, ap) for (_, g, dy2, x2), ap in entries],
                            dbias=[b[1] if b is not None else None for b in bias])
    if not ok:
        for (it, _), b in zip(entries, bias):
            if b is not None:
                paired[_dkey(it[2])] = b
        return groups
    for ((p, _, _, _), _), b in zip(entries, bias):
        done(p)
        if b is not None:
            done(b[0])
    return {k: its for k, its in groups.items() if k not in sel}


def _final_flush(task):
    _QUEUED.discard(task)
    flush_wgrads(task)


def _queue_flush(task):
    if task not in _QUEUED:
        _QUEUED.add(task)
        torch.autograd.Variable._execution_engine.queue_callback(lambda: _final_flush(task))


def _defer_wgrad(p, g, dy2, x2, alpha_ptr=None):
    task = _task()
    p._gvl_sunk_task = task
    if x2 is None:  # bias gradient
        _PENDING_B.append((task, p, g, dy2, torch.cuda.current_stream(dy2.device)))
    else:
        _PENDING.append((task, p, g, dy2, x2, torch.cuda.current_stream(dy2.device), alpha_ptr))
    _queue_flush(task)


def _block_done():
    """End of one GPT-2 block's backward: with data-parallel overlap on, flush this task's
    queue every OVERLAP_BLOCKS blocks."""
    G = OVERLAP_BLOCKS[0]
    if G <= 0 or not DEFER_WGRAD:
        return
    task = _task()
    n = _BLOCKS_SEEN.get(task, 0) + 1
    if n >= G:
        flush_wgrads(task)
    else:
        _BLOCKS_SEEN[task] = n


def register_grad_ready_hook(fn):
    """fn(param) runs when a fused Function has finished accumulating param.grad."""
    _READY_HOOKS.append(fn)

    class _Handle:
        @staticmethod
        def remove():
            if fn in _READY_HOOKS:
                _READY_HOOKS.remove(fn)
    return _Handle()


def _ddp_forward_active():
    """True while torch DDP runs its wrapped module's forward (DDP._inside_ddp_forward).
    DDP's reducer all-reduces from AccumulateGrad hooks (train_gpt2.py:270,468), so a
    Function built under it must hand its gradients to autograd instead of sinking them."""
    ddp = torch.nn.parallel.DistributedDataParallel
    return getattr(ddp, "_active_ddp_module", None) is not None


def _mark(ctx):
    """Forward-time decision whether this node may accumulate into arena grads in place."""
    ctx.sink_ok = FUSE_GRAD_ACC and not _ddp_forward_active()


def _sink(p, ctx=None):
    # only gradients that live in a gvl.optim.AdamW arena: their consumers (the fused
    # optimizer, gvl.dist.GradBuckets) do not rely on AccumulateGrad hooks, which torch DDP
    # and plain torch optimizers' users may
    if not FUSE_GRAD_ACC or not getattr(p, "_gvl_grad_sink", False):
        return None
    if ctx is not None and not getattr(ctx, "sink_ok", True):
        return None
    g = p.grad
    if g is None or g.dtype != BF16 or g.shape != p.shape or not g.is_contiguous() or not g.is_cuda:
        return None
    return g


def _ready(p):
    # The engine still runs p's AccumulateGrad node (and its post-accumulate-grad hooks)
    # when the Function returned None for p; the mark tells gvl.dist.GradBuckets that this
    # backward's gradient of p arrives through this path instead.
    p._gvl_sunk_task = _task()
    for fn in _READY_HOOKS:
        fn(p)


def sunk_in_this_backward(p):
    """True when a fused unit accumulates p's gradient in place during the current backward
    (its AccumulateGrad hook then carries no gradient)."""
    return getattr(p, "_gvl_sunk_task", None) == _task()


def _wgrad(ctx, i, p, dy2, x2, defer=False):
    """nn.Linear weight gradient dy2^T x2 of input i (accumulated in place when p sinks)."""
    if not _need(ctx, i):
        return None
    g = _sink(p, ctx)
    if g is None:
        return K.linear_dw(dy2, x2)
    if defer and DEFER_WGRAD:  # dy2 and x2 must stay unmodified until the end of backward
        _defer_wgrad(p, g, dy2, x2)
        return None
    K.linear_dw(dy2, x2, out=g, residual=g)
    _ready(p)
    return None


def _bgrad(ctx, i, p, dy2, defer=False):
    """Bias gradient (column sum of dy2) of input i."""
    if not _need(ctx, i):
        return None
    g = _sink(p, ctx)
    if g is None:
        return K.colsum(dy2)
    if defer and DEFER_WGRAD and dy2.shape[0] > 0 and dy2.stride(1) == 1:
        _defer_wgrad(p, g.view(-1), dy2, None)
        return None
    K.colsum(dy2, out=g, accumulate=True)
    _ready(p)
    return None


def _ln_bwd(ctx, iw, ib, w, b, dy2, x2, mean, rstd, dx, accumulate_dx, residual=None):
    """LayerNorm backward writing/accumulating dx (or dx = residual + ..., no copy of the
    residual gradient); returns the (dw, db) autograd outputs."""
    nw, nb = _need(ctx, iw), _need(ctx, ib)
    gw = _sink(w, ctx) if nw else None
    gb = _sink(b, ctx) if nb else None
    if (nw or nb) and (gw is not None or not nw) and (gb is not None or not nb):
        if DEFER_WGRAD and DEFER_LN and x2.shape[0] > 0:  # partials flushed at the end of backward
            _, (ws, nblk) = K.layernorm_bwd(dy2, x2, w, mean, rstd, dx=dx, accumulate_dx=accumulate_dx,
                                            residual=residual, defer_wb=True)
            task = _task()
            for p, n in ((w, nw), (b, nb)):
                if n:
                    p._gvl_sunk_task = task
            _PENDING_LN.append((task, w, b, gw, gb, ws, nblk, x2.shape[1],
                                torch.cuda.current_stream(x2.device)))
            _queue_flush(task)
            return None, None
        K.layernorm_bwd(dy2, x2, w, mean, rstd, dx=dx, accumulate_dx=accumulate_dx, dw=gw, db=gb,
                        accumulate_wb=True, residual=residual)
        for p, n in ((w, nw), (b, nb)):
            if n:
                _ready(p)
        return None, None
    C = x2.shape[1]
    dw = torch.empty(C, dtype=BF16, device=x2.device) if nw else None
    db = torch.empty(C, dtype=BF16, device=x2.device) if nb else None
    K.layernorm_bwd(dy2, x2, w, mean, rstd, dx=dx, accumulate_dx=accumulate_dx, dw=dw, db=db,
                    residual=residual)
    return dw, db


# ------------------------------------------------------------------------ GPT-2 block
class GPTBlockFn(torch.autograd.Function):
    """x + attn(ln_1 x); then + mlp(ln_2 .) — source/gpt2/train_gpt2.py:62-74.

    Forward: LN -> c_attn GEMM(+bias) -> causal attention straight out of the packed qkv
    -> c_proj GEMM(+bias, +residual) -> LN -> c_fc GEMM(+bias, GELU-tanh, saves the
    pre-activation) -> c_proj GEMM(+bias, +residual).
    """

    @staticmethod
    def forward(ctx, x, ln1_w, ln1_b, attn_w, attn_b, aproj_w, aproj_b, ln2_w, ln2_b, fc_w,
                fc_b, mproj_w, mproj_b, n_head: int, causal: bool = True):
        B, T, C = x.shape
        x2 = x.reshape(B * T, C)
        if not x2.is_contiguous():
            x2 = x2.contiguous()
        xn1, m1, r1 = K.layernorm_fwd(x2, ln1_w, ln1_b)
        qkv = K.linear(xn1, attn_w, attn_b)
        q3 = qkv.view(B, T, 3 * C)
        y, lse = K.attn_fwd(q3[:, :, :C], q3[:, :, C:2 * C], q3[:, :, 2 * C:], n_head, causal)
        y2 = y.view(B * T, C)
        xm = K.linear(y2, aproj_w, aproj_b, residual=x2)
        xn2, m2, r2 = K.layernorm_fwd(xm, ln2_w, ln2_b)
        # the c_fc epilogue stores gelu'(x) (act 3) for the backward's dGELU multiply
        hpre = torch.empty(B * T, fc_w.shape[0], dtype=BF16, device=x.device)
        h = K.linear(xn2, fc_w, fc_b, act=1 + GELU_DERIV, pre_out=hpre)
        out = K.linear(h, mproj_w, mproj_b, residual=xm)
        if any(ctx.needs_input_grad):  # (grad mode is off inside forward)
            ctx.save_for_backward(x2, xn1, m1, r1, qkv, y, lse, xm, xn2, m2, r2, hpre, h, ln1_w,
                                  attn_w, aproj_w, ln2_w, fc_w, mproj_w)
            ctx.shape = (B, T, C, n_head, causal)
            ctx.params = (None, ln1_w, ln1_b, attn_w, attn_b, aproj_w, aproj_b, ln2_w, ln2_b,
                          fc_w, fc_b, mproj_w, mproj_b)
            _mark(ctx)
        return out.view(B, T, C)

    @staticmethod
    def backward(ctx, dout):
        (x2, xn1, m1, r1, qkv, y, lse, xm, xn2, m2, r2, hpre, h, ln1_w, attn_w, aproj_w, ln2_w,
         fc_w, mproj_w) = ctx.saved_tensors
        B, T, C, H, causal = ctx.shape
        g = [None] * 15
        d2 = dout.reshape(B * T, C)
        if d2.dtype != BF16:
            d2 = d2.to(BF16)
        d2 = d2.contiguous()
        P = ctx.params
        # MLP c_proj
        g[11] = _wgrad(ctx, 11, P[11], d2, h, defer=True)
        g[12] = _bgrad(ctx, 12, P[12], d2, defer=True)
        dpre = K.linear_dx(d2, mproj_w, dact=3 if GELU_DERIV else 1, pre_in=hpre)
        g[9] = _wgrad(ctx, 9, P[9], dpre, xn2, defer=True)
        g[10] = _bgrad(ctx, 10, P[10], dpre, defer=True)
        dxn2 = K.linear_dx(dpre, fc_w)
        dxm = torch.empty_like(d2)  # = d2 + LN_2 backward (the residual read from d2, no copy)
        g[7], g[8] = _ln_bwd(ctx, 7, 8, P[7], P[8], dxn2, xm, m2, r2, dxm, True, residual=d2)
        # attention c_proj
        g[5] = _wgrad(ctx, 5, P[5], dxm, y.view(B * T, C), defer=True)
        g[6] = _bgrad(ctx, 6, P[6], dxm, defer=True)
        dy = K.linear_dx(dxm, aproj_w)
        dqkv = torch.empty(B * T, 3 * C, dtype=BF16, device=d2.device)
        q3 = qkv.view(B, T, 3 * C)
        dq3 = dqkv.view(B, T, 3 * C)
        K.attn_bwd(dy.view(B, T, C), q3[:, :, :C], q3[:, :, C:2 * C], q3[:, :, 2 * C:], y, lse, H,
                   causal, dq3[:, :, :C], dq3[:, :, C:2 * C], dq3[:, :, 2 * C:])
        g[3] = _wgrad(ctx, 3, P[3], dqkv, xn1, defer=True)
        g[4] = _bgrad(ctx, 4, P[4], dqkv, defer=True)
        dxn1 = K.linear_dx(dqkv, attn_w)
        dx = torch.empty_like(dxm)  # dxm stays intact: the (deferred) c_proj dW reads it
        g[1], g[2] = _ln_bwd(ctx, 1, 2, P[1], P[2], dxn1, x2, m1, r1, dx, True, residual=dxm)
        g[0] = dx.view(B, T, C) if _need(ctx, 0) else None
        _block_done()
        return tuple(g)


# ------------------------------------------------------------------------- LayerNorm
class ResTape:
    """Pre-LN residual stream x -> x + f(LN(x)) outside one fused unit (the Q-Former layers):
    autograd would sum x's two gradients (the residual path's and LN's) with a separate add
    kernel.  Instead the unit gets x detached as its residual, ResTapFn on its output hands
    d(output) to this tape, and LayerNormFn(x, ..., tape) returns dx = d(output) + LN'(dy) from
    one LayerNorm-backward launch (gvl_layernorm_bwd_res)."""
    __slots__ = ("d",)

    def __init__(self):
        self.d = None


class ResTapFn(torch.autograd.Function):
    """Identity on a residual unit's output; its backward stores the output gradient in the
    tape (the gradient of the unit's detached residual input) and passes it on unchanged."""

    @staticmethod
    def forward(ctx, y, tape):
        ctx.tape = tape
        return y.view_as(y)

    @staticmethod
    def backward(ctx, dy):
        ctx.tape.d = dy
        return dy, None


class LayerNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, eps: float = 1e-5, tape: ResTape = None):
        shp = x.shape
        x2 = x.reshape(-1, shp[-1])
        if x2.dtype != BF16:
            x2 = x2.to(BF16)
        x2 = x2.contiguous()
        y, mean, rstd = K.layernorm_fwd(x2, w, b, eps)
        if any(ctx.needs_input_grad):  # (grad mode is off inside forward)
            ctx.save_for_backward(x2, w, mean, rstd)
            ctx.shp = shp
            ctx.params = (w, b)
            ctx.tape = tape
            _mark(ctx)
        return y.view(shp)

    @staticmethod
    def backward(ctx, dy):
        x2, w, mean, rstd = ctx.saved_tensors
        C = x2.shape[1]
        d2 = dy.reshape(-1, C).to(BF16).contiguous()
        dx = torch.empty(x2.shape[0], C, dtype=BF16, device=x2.device)
        res = None
        if ctx.tape is not None and ctx.tape.d is not None:  # the stream's residual gradient
            res = ctx.tape.d.reshape(-1, C).to(BF16).contiguous()
            ctx.tape.d = None
        if _need(ctx, 1) or _need(ctx, 2):
            dw, db = _ln_bwd(ctx, 1, 2, ctx.params[0], ctx.params[1], d2, x2, mean, rstd, dx,
                             False, residual=res)
        else:
            dw = db = None
            K.layernorm_bwd(d2, x2, w, mean, rstd, dx=dx, residual=res)
        return (dx.view(ctx.shp) if _need(ctx, 0) else None), dw, db, None, None


# ---------------------------------------------------------------------------- Linear
class LinearFn(torch.autograd.Function):
    """y = [residual +] [tanh(gate) *] dropout(x W^T + b)."""

    @staticmethod
    def forward(ctx, x, w, b, residual=None, gate=None, drop_p: float = 0.0, seed: int = 0):
        shp = x.shape
        x2 = x.reshape(-1, shp[-1])
        if x2.dtype != BF16:
            x2 = x2.to(BF16)
        x2 = x2.contiguous()
        N = w.shape[0]
        r2 = None
        if residual is not None:
            r2 = residual.reshape(-1, N)
            if r2.dtype != BF16:
                r2 = r2.to(BF16)
            r2 = r2.contiguous()
        ybr = None
        if gate is not None:
            ybr = torch.empty(x2.shape[0], N, dtype=BF16, device=x.device)
        y = K.linear(x2, w, b, residual=r2, gate=gate, pre_out=ybr, drop_p=drop_p, seed=seed,
                     seed_ptr=_off(x2, drop_p))
        if any(ctx.needs_input_grad):  # (grad mode is off inside forward)
            ctx.save_for_backward(x2, w, gate, ybr)
            ctx.cfg = (shp, N, drop_p, seed, residual is not None)
            ctx.params = (w, b)
            _mark(ctx)
        return y.view(*shp[:-1], N)

    @staticmethod
    def backward(ctx, dy):
        x2, w, gate, ybr = ctx.saved_tensors
        shp, N, drop_p, seed, has_res = ctx.cfg
        d2 = dy.reshape(-1, N)
        if d2.dtype != BF16:
            d2 = d2.to(BF16)
        d2 = d2.contiguous()
        dres = dy if (has_res and _need(ctx, 3)) else None
        dgate = None
        dbr = d2
        if gate is not None:
            gacc = torch.zeros(1, dtype=torch.float32, device=d2.device)
            dbr = K.gate_bwd(d2, ybr, gate, gacc)
            if _need(ctx, 4):
                dgate = gacc.to(gate.dtype).view_as(gate)
        if drop_p > 0:
            dbr = K.dropout_mask_apply(dbr, drop_p, seed, seed_ptr=_off(dbr, drop_p))
        dx = K.linear_dx(dbr, w).view(shp) if _need(ctx, 0) else None
        dw = _wgrad(ctx, 1, ctx.params[0], dbr, x2, defer=DEFER_BRIDGE)
        db = _bgrad(ctx, 2, ctx.params[1], dbr, defer=DEFER_BRIDGE)
        return dx, dw, db, dres, dgate, None, None


class MLPFn(torch.autograd.Function):
    """y = [residual +] dropout(act(x W1^T + b1) W2^T + b2); act: 1 gelu-tanh, 2 gelu-erf."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, residual=None, act: int = 1, drop_p: float = 0.0,
                seed: int = 0):
        shp = x.shape
        x2 = x.reshape(-1, shp[-1]).to(BF16).contiguous()
        hpre = torch.empty(x2.shape[0], w1.shape[0], dtype=BF16, device=x.device)
        h = K.linear(x2, w1, b1, act=act + GELU_DERIV, pre_out=hpre)  # pre_out <- gelu'(x)
        r2 = residual.reshape(-1, w2.shape[0]).to(BF16).contiguous() if residual is not None else None
        y = K.linear(h, w2, b2, residual=r2, drop_p=drop_p, seed=seed, seed_ptr=_off(h, drop_p))
        if any(ctx.needs_input_grad):  # (grad mode is off inside forward)
            ctx.save_for_backward(x2, w1, w2, hpre, h)
            ctx.cfg = (shp, act, drop_p, seed, residual is not None)
            ctx.params = (None, w1, b1, w2, b2)
            _mark(ctx)
        return y.view(*shp[:-1], w2.shape[0])

    @staticmethod
    def backward(ctx, dy):
        x2, w1, w2, hpre, h = ctx.saved_tensors
        shp, act, drop_p, seed, has_res = ctx.cfg
        d2 = dy.reshape(-1, w2.shape[0]).to(BF16).contiguous()
        dres = dy if (has_res and _need(ctx, 5)) else None
        if drop_p > 0:
            d2 = K.dropout_mask_apply(d2, drop_p, seed, seed_ptr=_off(d2, drop_p))
        P = ctx.params
        dw2 = _wgrad(ctx, 3, P[3], d2, h, defer=DEFER_BRIDGE)
        db2 = _bgrad(ctx, 4, P[4], d2, defer=DEFER_BRIDGE)
        dpre = K.linear_dx(d2, w2, dact=3 if GELU_DERIV else act, pre_in=hpre)
        dw1 = _wgrad(ctx, 1, P[1], dpre, x2, defer=DEFER_BRIDGE)
        db1 = _bgrad(ctx, 2, P[2], dpre, defer=DEFER_BRIDGE)
        dx = K.linear_dx(dpre, w1).view(shp) if _need(ctx, 0) else None
        return dx, dw1, db1, dw2, db2, dres, None, None, None


# ------------------------------------------------------------------ attention units
class MHAFn(torch.autograd.Function):
    """nn.MultiheadAttention(batch_first) core + out_proj + dropout + residual
    (gpt2_q_former/model.py:119-141): out = residual + drop(out_proj(attn(...))).

    self_attn: q_in is also the key/value input and the packed in_proj runs as ONE GEMM
    (N = 3C); otherwise q rows [0,C) of in_proj act on q_in and rows [C,3C) on kv_in.
    Attention-probability dropout p_attn uses the in-kernel counter mask.
    """

    @staticmethod
    def forward(ctx, q_in, kv_in, in_w, in_b, out_w, out_b, residual, n_head: int,
                self_attn: bool, p_attn: float, p_out: float, seed: int):
        B, Tq, C = q_in.shape
        Tk = kv_in.shape[1]
        q2 = q_in.reshape(B * Tq, C).to(BF16).contiguous()
        if self_attn:
            qkv = K.linear(q2, in_w, in_b)
            p3 = qkv.view(B, Tq, 3 * C)
            qv, kv_, vv = p3[:, :, :C], p3[:, :, C:2 * C], p3[:, :, 2 * C:]
            kv2 = None
            qp = kvp = None
        else:
            kv2 = kv_in.reshape(B * Tk, C).to(BF16).contiguous()
            qp = K.linear(q2, in_w[:C], in_b[:C])
            kvp = K.linear(kv2, in_w[C:], in_b[C:])
            q3 = qp.view(B, Tq, C)
            k3 = kvp.view(B, Tk, 2 * C)
            qv, kv_, vv = q3, k3[:, :, :C], k3[:, :, C:]
            qkv = None
        sa = seed ^ 0x5A5A5A5A
        o, lse = K.attn_fwd(qv, kv_, vv, n_head, False, drop_p=p_attn, seed=sa,
                            seed_ptr=_off(qv, p_attn))
        r2 = residual.reshape(B * Tq, C).to(BF16).contiguous()
        out = K.linear(o.view(B * Tq, C), out_w, out_b, residual=r2, drop_p=p_out, seed=seed,
                       seed_ptr=_off(o, p_out))
        if any(ctx.needs_input_grad):  # (grad mode is off inside forward)
            ctx.save_for_backward(q2, kv2, in_w, out_w, qkv, qp, kvp, o, lse)
            ctx.cfg = (B, Tq, Tk, C, n_head, self_attn, p_attn, p_out, seed, sa)
            ctx.params = (in_w, in_b, out_w, out_b)
            _mark(ctx)
        return out.view(B, Tq, C)

    @staticmethod
    def backward(ctx, dout):
        q2, kv2, in_w, out_w, qkv, qp, kvp, o, lse = ctx.saved_tensors
        B, Tq, Tk, C, H, self_attn, p_attn, p_out, seed, sa = ctx.cfg
        d2 = dout.reshape(B * Tq, C).to(BF16).contiguous()
        dres = dout if _need(ctx, 6) else None
        dbr = (K.dropout_mask_apply(d2, p_out, seed, seed_ptr=_off(d2, p_out)) if p_out > 0
               else d2)
        P_in_w, P_in_b, P_out_w, P_out_b = ctx.params
        d_out_w = _wgrad(ctx, 4, P_out_w, dbr, o.view(B * Tq, C), defer=DEFER_BRIDGE)
        d_out_b = _bgrad(ctx, 5, P_out_b, dbr, defer=DEFER_BRIDGE)
        do = K.linear_dx(dbr, out_w).view(B, Tq, C)
        # packed in_proj gradients: written into the sinks (accumulate) or fresh buffers
        sw = _sink(P_in_w, ctx) if _need(ctx, 2) else None
        sb = _sink(P_in_b, ctx) if _need(ctx, 3) else None
        din_w = torch.empty_like(in_w) if (_need(ctx, 2) and sw is None) else None
        din_b = (torch.empty(3 * C, dtype=BF16, device=d2.device)
                 if (_need(ctx, 3) and sb is None) else None)
        tw = sw if sw is not None else din_w
        tb = sb if sb is not None else din_b

        # into the arena sinks the row slices are deferred like the other bridge gradients
        # (one grouped launch at the end of backward; the grad-ready hook after the last slice)
        dfw = sw is not None and DEFER_BRIDGE and DEFER_INPROJ and DEFER_WGRAD
        dfb = sb is not None and DEFER_BRIDGE and DEFER_INPROJ and DEFER_WGRAD
        b_deferred = [False]  # some slice went to the queue: its flush fires the grad-ready hook

        def wg(dy_, x_, rows):
            if dfw:
                _defer_wgrad(P_in_w, tw[rows], dy_, x_)
            elif tw is not None:
                K.linear_dw(dy_, x_, out=tw[rows], residual=tw[rows] if sw is not None else None)

        def bg(dy_, rows):
            # deferred under the same guard as _bgrad (rows present, unit column stride); today
            # dqkv / dqp / dkvp are fresh contiguous buffers, so the guard only protects callers
            if dfb and dy_.shape[0] > 0 and dy_.stride(1) == 1:
                _defer_wgrad(P_in_b, tb[rows], dy_, None)
                b_deferred[0] = True
            elif tb is not None:
                K.colsum(dy_, out=tb[rows], accumulate=sb is not None)

        dq_in = dkv_in = None
        if self_attn:
            p3 = qkv.view(B, Tq, 3 * C)
            dqkv = torch.empty(B * Tq, 3 * C, dtype=BF16, device=d2.device)
            dp3 = dqkv.view(B, Tq, 3 * C)
            K.attn_bwd(do, p3[:, :, :C], p3[:, :, C:2 * C], p3[:, :, 2 * C:], o, lse, H, False,
                       dp3[:, :, :C], dp3[:, :, C:2 * C], dp3[:, :, 2 * C:], drop_p=p_attn,
                       seed=sa, seed_ptr=_off(do, p_attn))
            wg(dqkv, q2, slice(None))
            bg(dqkv, slice(None))
            if _need(ctx, 0):
                dq_in = K.linear_dx(dqkv, in_w).view(B, Tq, C)
        else:
            q3 = qp.view(B, Tq, C)
            k3 = kvp.view(B, Tk, 2 * C)
            dqp = torch.empty(B * Tq, C, dtype=BF16, device=d2.device)
            dkvp = torch.empty(B * Tk, 2 * C, dtype=BF16, device=d2.device)
            dk3 = dkvp.view(B, Tk, 2 * C)
            K.attn_bwd(do, q3, k3[:, :, :C], k3[:, :, C:], o, lse, H, False, dqp.view(B, Tq, C),
                       dk3[:, :, :C], dk3[:, :, C:], drop_p=p_attn, seed=sa,
                       seed_ptr=_off(do, p_attn))
            wg(dqp, q2, slice(0, C))
            wg(dkvp, kv2, slice(C, None))
            bg(dqp, slice(0, C))
            bg(dkvp, slice(C, None))
            if _need(ctx, 0):
                dq_in = K.linear_dx(dqp, in_w[:C]).view(B, Tq, C)
            if _need(ctx, 1):
                dkv_in = K.linear_dx(dkvp, in_w[C:]).view(B, Tk, C)
        if sw is not None and not dfw:
            _ready(P_in_w)
        if sb is not None and not b_deferred[0]:
            _ready(P_in_b)
        return dq_in, dkv_in, din_w, din_b, d_out_w, d_out_b, dres, None, None, None, None, None


class CrossAttnFn(torch.autograd.Function):
    """Gated cross-attention residual of the cross-att bridge (gpt2_cross-att/model.py:46-58,
    :99-101): x + tanh(g) * c_proj(SDPA(q_proj(ln_x x), kv_proj(z)))."""

    @staticmethod
    def forward(ctx, x, z, ln_w, ln_b, q_w, q_b, kv_w, kv_b, c_w, c_b, gate, n_head: int):
        S = z.shape[1]
        z2 = z.reshape(z.shape[0] * S, z.shape[2]).to(BF16).contiguous()
        kvp = K.linear(z2, kv_w, kv_b)
        out = _xattn_fwd(ctx, x, kvp.view(z.shape[0], S, kvp.shape[1]), 0, ln_w, ln_b, q_w, q_b,
                         c_w, c_b, gate, n_head)
        if any(ctx.needs_input_grad):
            ctx.z2, ctx.kv_w = z2, kv_w
            ctx.params = (None, None, ln_w, ln_b, q_w, q_b, kv_w, kv_b, c_w, c_b, gate)
            ctx.idx = (0, 2, 3, 4, 5, 8, 9, 10)
        return out

    @staticmethod
    def backward(ctx, dout):
        g = [None] * 12
        C = ctx.cfg[3]
        dkvp = torch.empty(ctx.z2.shape[0], 2 * C, dtype=BF16, device=dout.device)
        _xattn_bwd(ctx, dout, dkvp.view(ctx.cfg[0], ctx.cfg[2], 2 * C), g)
        P = ctx.params
        g[6] = _wgrad(ctx, 6, P[6], dkvp, ctx.z2, defer=True)
        g[7] = _bgrad(ctx, 7, P[7], dkvp, defer=True)
        if _need(ctx, 1):
            g[1] = K.linear_dx(dkvp, ctx.kv_w).view(ctx.cfg[0], ctx.cfg[2], C)
        return tuple(g)


def _xattn_fwd(ctx, x, kv, off, ln_w, ln_b, q_w, q_b, c_w, c_b, gate, n_head):
    """Everything of the gated cross-attention but kv_proj: K = kv[..., off:off+C],
    V = kv[..., off+C:off+2C] (strided views of the packed projection)."""
    B, T, C = x.shape
    S = kv.shape[1]
    x2 = x.reshape(B * T, C).contiguous()
    xn, mean, rstd = K.layernorm_fwd(x2, ln_w, ln_b)
    qp = K.linear(xn, q_w, q_b)
    o, lse = K.attn_fwd(qp.view(B, T, C), kv[:, :, off:off + C], kv[:, :, off + C:off + 2 * C],
                        n_head, False)
    ybr = torch.empty(B * T, C, dtype=BF16, device=x.device)
    out = K.linear(o.view(B * T, C), c_w, c_b, residual=x2, gate=gate, pre_out=ybr)
    if any(ctx.needs_input_grad):  # (grad mode is off inside forward)
        ctx.save_for_backward(x2, xn, mean, rstd, qp, kv, o, lse, ybr, ln_w, q_w, c_w, gate)
        ctx.cfg = (B, T, S, C, n_head, off)
        _mark(ctx)
    return out.view(B, T, C)


def _xattn_bwd(ctx, dout, dkv, g):
    """Backward of _xattn_fwd: writes dK / dV into dkv[..., off:off+2C] and fills g at the
    positions ctx.idx = (x, ln_w, ln_b, q_w, q_b, c_w, c_b, gate) of the caller's inputs."""
    x2, xn, mean, rstd, qp, kv, o, lse, ybr, ln_w, q_w, c_w, gate = ctx.saved_tensors
    B, T, S, C, H, off = ctx.cfg
    ix, iln_w, iln_b, iq_w, iq_b, ic_w, ic_b, igate = ctx.idx
    P = ctx.params
    d2 = dout.reshape(B * T, C).to(BF16).contiguous()
    gsink = _sink(P[igate], ctx) if _need(ctx, igate) and GATE_SINK else None
    if gsink is not None:  # added into the gate's bf16 grad in the finish kernel
        dbr = K.gate_bwd(d2, ybr, gate, grad_bf16=gsink)
        _ready(P[igate])
    else:
        gacc = torch.zeros(1, dtype=torch.float32, device=d2.device)
        dbr = K.gate_bwd(d2, ybr, gate, gacc)
        if _need(ctx, igate):
            g[igate] = gacc.to(gate.dtype).view_as(gate)
    g[ic_w] = _wgrad(ctx, ic_w, P[ic_w], dbr, o.view(B * T, C), defer=True)
    g[ic_b] = _bgrad(ctx, ic_b, P[ic_b], dbr, defer=True)
    do = K.linear_dx(dbr, c_w).view(B, T, C)
    dqp = torch.empty(B * T, C, dtype=BF16, device=d2.device)
    K.attn_bwd(do, qp.view(B, T, C), kv[:, :, off:off + C], kv[:, :, off + C:off + 2 * C], o, lse,
               H, False, dqp.view(B, T, C), dkv[:, :, off:off + C], dkv[:, :, off + C:off + 2 * C])
    g[iq_w] = _wgrad(ctx, iq_w, P[iq_w], dqp, xn, defer=True)
    g[iq_b] = _bgrad(ctx, iq_b, P[iq_b], dqp, defer=True)
    dxn = K.linear_dx(dqp, q_w)
    dx = torch.empty_like(d2)  # = d2 + LN backward (residual read from d2, no copy)
    g[iln_w], g[iln_b] = _ln_bwd(ctx, iln_w, iln_b, P[iln_w], P[iln_b], dxn, x2, mean, rstd, dx,
                                 True, residual=d2)
    g[ix] = dx.view(B, T, C) if _need(ctx, ix) else None


class KVGradSlab:
    """The [B, S, L*2C] gradient of CrossKVFn's packed output, shared by the L blocks: each
    block's backward writes its dK / dV columns in place, and the last one to run hands the
    whole slab to autograd (the others return None), so CrossKVFn.backward — which the engine
    runs only after all L consumers — sees every column written and no [B, S, L*2C] zeros or
    slice-gradient adds are ever materialised."""

    def __init__(self, layers):
        self.layers, self.left, self.buf, self.task = layers, layers, None, None

    def take(self, like):
        # re-armed per autograd graph task: a backward that stopped part-way (raised, or
        # torch.autograd.grad to an intermediate output) leaves no half-counted state for the
        # next backward over the same (retained) graph
        task = _task()
        if self.task != task:
            self.task, self.left, self.buf = task, self.layers, None
        if self.buf is None:
            self.buf = torch.empty(like.shape, dtype=BF16, device=like.device)
        return self.buf

    def release(self):
        self.left -= 1
        if self.left > 0:
            return None
        buf, self.buf, self.left, self.task = self.buf, None, self.layers, None
        return buf


def _stacked(ts):
    """torch.cat(ts, 0) — or, when the tensors already sit back to back in one storage (the gvl
    AdamW arena places parameters tagged with one `_gvl_stack_key` consecutively), a view of
    that storage with no copy."""
    t0 = ts[0]
    n, es = t0.numel(), t0.element_size()
    if all(t.is_contiguous() and t.dtype == t0.dtype and t.shape == t0.shape and
           t.untyped_storage().data_ptr() == t0.untyped_storage().data_ptr() and
           t.data_ptr() == t0.data_ptr() + i * n * es for i, t in enumerate(ts)):
        return t0.as_strided((len(ts) * t0.shape[0],) + tuple(t0.shape[1:]),
                             (t0.stride(0),) + tuple(t0.stride()[1:]))
    return torch.cat(ts, 0)


class CrossKVFn(torch.autograd.Function):
    """kv_proj of ALL cross-attention blocks (gpt2_cross-att/model.py:49-50 in each Block)
    over the same projected CLIP tokens as one GEMM against the stacked weights
    [L*2C, C] -> packed [B, S, L*2C]; backward: dz as one GEMM (K = L*2C) instead of L
    dX GEMMs plus L-1 gradient adds, the L weight/bias gradients as deferred problems of
    the batched launch.  forward(z, slab, w_0, b_0, ..., w_{L-1}, b_{L-1})."""

    @staticmethod
    def forward(ctx, z, slab, *wb):
        L = len(wb) // 2
        B, S, C = z.shape
        z2 = z.reshape(B * S, C).to(BF16).contiguous()
        w_all = _stacked(wb[0::2])
        kv = K.linear(z2, w_all, _stacked(wb[1::2]))
        if any(ctx.needs_input_grad):
            ctx.save_for_backward(z2, w_all)
            ctx.cfg = (B, S, C, L)
            ctx.params = (None, None) + tuple(wb)
            _mark(ctx)
        return kv.view(B, S, w_all.shape[0])

    @staticmethod
    def backward(ctx, dkv):
        z2, w_all = ctx.saved_tensors
        B, S, C, L = ctx.cfg
        d2 = dkv.reshape(B * S, 2 * C * L)
        if d2.dtype != BF16 or d2.stride(1) != 1:
            d2 = d2.to(BF16).contiguous()
        g = [None] * (2 + 2 * L)
        P = ctx.params
        for layer in range(L):
            sl = d2[:, 2 * C * layer:2 * C * (layer + 1)]
            g[2 + 2 * layer] = _wgrad(ctx, 2 + 2 * layer, P[2 + 2 * layer], sl, z2, defer=True)
            g[3 + 2 * layer] = _bgrad(ctx, 3 + 2 * layer, P[3 + 2 * layer], sl, defer=True)
        if _need(ctx, 0):
            g[0] = K.linear_dx(d2, w_all).view(B, S, C)
        return tuple(g)


class CrossAttnKVFn(torch.autograd.Function):
    """CrossAttnFn of block `layer` over the packed projection of CrossKVFn (no kv_proj of
    its own); dK / dV go straight into the shared KVGradSlab."""

    @staticmethod
    def forward(ctx, x, kv, layer: int, slab, ln_w, ln_b, q_w, q_b, c_w, c_b, gate, n_head: int):
        C = x.shape[2]
        out = _xattn_fwd(ctx, x, kv, 2 * C * layer, ln_w, ln_b, q_w, q_b, c_w, c_b, gate, n_head)
        if any(ctx.needs_input_grad):
            ctx.slab = slab
            ctx.params = (None, None, None, None, ln_w, ln_b, q_w, q_b, c_w, c_b, gate)
            ctx.idx = (0, 4, 5, 6, 7, 8, 9, 10)
        return out

    @staticmethod
    def backward(ctx, dout):
        g = [None] * 12
        kv = ctx.saved_tensors[5]
        buf = ctx.slab.take(kv)
        _xattn_bwd(ctx, dout, buf, g)
        g[1] = ctx.slab.release() if _need(ctx, 1) else None
        return tuple(g)


# ------------------------------------------------------------------------ embeddings
class EmbedFn(torch.autograd.Function):
    """wte(idx) + wpe(arange(T)) written at row offset `off` of a [B, S, C] buffer whose
    first `off` rows per sequence are `prefix` (the caption image tokens; may be None).

    Backward: the deterministic per-id / per-position sums (gvl_embedding_bwd_det, no
    atomics) accumulate straight into arena-sink gradients; the tied wte therefore gets the
    lm_head weight gradient (LMHeadLossFn, GEMM epilogue C += dl^T x) and this row update in
    ONE bf16 buffer, with no [V, C] temporary, cast or autograd add per micro-step."""

    @staticmethod
    def forward(ctx, idx, wte, wpe, prefix=None):
        B, T = idx.shape
        C = wte.shape[1]
        check_index_range(idx, wte.shape[0], "token id")
        M = 0 if prefix is None else prefix.shape[1]
        S = M + T
        out = torch.empty(B, S, C, dtype=BF16, device=idx.device)
        if prefix is not None:  # the image tokens in front (torch.cat, model.py:191)
            pre = prefix if prefix.dtype == BF16 else prefix.to(BF16)
            pre = pre.contiguous()
            K.copy_rows(pre.view(B * M, C), out.view(B * S, C), M, B, M, 0, S, 0)
        K.embedding_fwd(idx, wte, wpe, out, T, S, M)
        if any(ctx.needs_input_grad):  # (grad mode is off inside forward)
            ctx.save_for_backward(idx)
            ctx.cfg = (B, T, C, M, S, wte.shape[0], wpe.shape[0], wte.dtype, wpe.dtype)
            ctx.params = (None, wte, wpe)
            _mark(ctx)
        return out

    @staticmethod
    def backward(ctx, dout):
        (idx,) = ctx.saved_tensors
        B, T, C, M, S, V, P, dt_te, dt_pe = ctx.cfg
        dout = dout.to(BF16).contiguous()
        dwte = dwpe = dprefix = None
        if _need(ctx, 1) or _need(ctx, 2):
            wte, wpe = ctx.params[1], ctx.params[2]
            gte = _sink(wte, ctx) if _need(ctx, 1) else None
            gpe = _sink(wpe, ctx) if _need(ctx, 2) else None
            tte = gte if gte is not None else (
                torch.zeros(V, C, dtype=BF16, device=dout.device) if _need(ctx, 1) else None)
            tpe = gpe if gpe is not None else (
                torch.zeros(P, C, dtype=BF16, device=dout.device) if _need(ctx, 2) else None)
            K.embedding_bwd_det(idx, dout, tte, tpe, T, S, M, C, V)
            if gte is not None:
                _ready(wte)
            elif tte is not None:
                dwte = tte if dt_te == BF16 else tte.to(dt_te)
            if gpe is not None:
                _ready(wpe)
            elif tpe is not None:
                dwpe = tpe if dt_pe == BF16 else tpe.to(dt_pe)
        if M > 0 and _need(ctx, 3):
            dprefix = dout[:, :M]
        return None, dwte, dwpe, dprefix


# -------------------------------------------------------------- lm_head + cross-entropy
class LMHeadLossFn(torch.autograd.Function):
    """logits = x W^T (tied wte), loss = CE(logits[:, off:off+T], targets) in one unit.

    The CE kernel reads the loss rows of the logits in place and emits
    dlogits = softmax - onehot at forward time; backward is two GEMMs scaled on the
    device by grad_loss / count (no host sync).  Logits are returned non-differentiable.
    """

    @staticmethod
    def forward(ctx, x, w, targets, row_offset: int, mask=None, mask_mode: bool = False,
                vocab: int = None):
        B, S, C = x.shape
        T = targets.shape[1]
        x2 = x.reshape(B * S, C).to(BF16).contiguous()
        logits = K.linear(x2, w)
        V = w.shape[0]
        vocab = V if vocab is None else vocab
        check_index_range(targets, vocab, "target", ignore_index=-100)
        need = ctx.needs_input_grad[0] or ctx.needs_input_grad[1]
        if need:
            ctx.params = (None, w)
            _mark(ctx)
        out, dl = K.cross_entropy(logits, targets, rows_per_group=T, group_stride=S,
                                  row_offset=row_offset, mask=mask, mask_mode=mask_mode,
                                  want_grad=need, vocab=vocab)
        loss = out[0].clone()
        logits = logits.view(B, S, V)
        ctx.mark_non_differentiable(logits)
        ctx.set_materialize_grads(False)  # no zero-filled [rows, V] grad for the logits
        if need:
            ctx.save_for_backward(x2, w, dl, out)
            ctx.cfg = (B, S, T, C, row_offset)
        return logits, loss

    @staticmethod
    def backward(ctx, _dlogits, dloss):
        x2, w, dl, out = ctx.saved_tensors
        B, S, T, C, off = ctx.cfg
        if dloss is None:
            return None, None, None, None, None, None, None
        scale = (dloss.float().reshape(1) * out[1:2]).contiguous()
        dx = dw = None
        if ctx.needs_input_grad[0]:
            dxt = K.gemm(dl, w, b_mn=True, alpha_ptr=scale)
            if off == 0 and T == S:
                dx = dxt.view(B, S, C)
            else:  # text rows at their offset, the image rows' gradient is zero
                dx = torch.empty(B, S, C, dtype=BF16, device=dl.device)
                K.copy_rows(dxt, dx.view(B * S, C), T, B, T, 0, S, off, zero_rest=True)
        if ctx.needs_input_grad[1]:
            if off == 0 and T == S:
                xt = x2
            else:
                xt = x2.view(B, S, C)[:, off:off + T].reshape(B * T, C).contiguous()
            g = _sink(ctx.params[1], ctx)  # the tied wte's arena gradient: C += dl^T x
            if g is not None and DEFER_WGRAD and DEFER_LMHEAD:
                # queued: the end-of-backward flush can run it in one grouped launch with the
                # blocks' weight gradients (dl and xt stay alive in the queue until then)
                _defer_wgrad(ctx.params[1], g, dl, xt, alpha_ptr=scale)
            elif g is not None:
                K.gemm(dl, xt, a_mn=True, b_mn=True, alpha_ptr=scale, out=g, residual=g)
                _ready(ctx.params[1])
            else:
                dw = K.gemm(dl, xt, a_mn=True, b_mn=True, alpha_ptr=scale)
        return dx, dw, None, None, None, None, None


class QueryExpandFn(torch.autograd.Function):
    """query_tokens.unsqueeze(0).expand(B, -1, -1) materialised once as a contiguous [B, Q, C]
    bf16 tensor (gpt2_q_former/model.py:160-161); backward: the batch sum as one column-sum
    kernel over [B, Q*C] (into the arena gradient when it sinks) instead of ATen's reduce."""

    @staticmethod
    def forward(ctx, q, B: int):
        Q, C = q.shape
        qb = q if q.dtype == BF16 else q.to(BF16)
        out = torch.empty(B, Q, C, dtype=BF16, device=q.device)
        K.copy_rows(qb.contiguous(), out.view(B * Q, C), Q, B, 0, 0, Q, 0)
        if ctx.needs_input_grad[0]:
            ctx.params = (q,)
            ctx.shape = (B, Q, C, q.dtype)
            _mark(ctx)
        return out

    @staticmethod
    def backward(ctx, dout):
        B, Q, C, dt = ctx.shape
        d2 = dout.to(BF16).contiguous().view(B, Q * C)
        p = ctx.params[0]
        g = _sink(p, ctx)
        if g is not None:
            K.colsum(d2, out=g.view(-1), accumulate=True)
            _ready(p)
            return None, None
        dq = K.colsum(d2).view(Q, C)
        return (dq if dt == BF16 else dq.to(dt)), None


def lm_head_loss(x, w, targets, row_offset=0, mask=None, mask_mode=False):
    """(logits, loss) of the tied lm_head + CE for any vocab size (pads V to 8 if needed)."""
    wp, V = pad_vocab(w)
    logits, loss = LMHeadLossFn.apply(x, wp, targets, row_offset, mask, mask_mode, V)
    if wp is not w:
        logits = logits[..., :V].contiguous()
    return logits, loss


def lm_logits(x, w):
    """logits = x w^T for the lm_head (any vocab size)."""
    wp, V = pad_vocab(w)
    logits = LinearFn.apply(x, wp, None)
    return logits if wp is w else logits[..., :V].contiguous()


def pool_clip(tokens):
    """pool_clip_197_to_33_avg_with_cls on the GPU (gpt2_linear/model.py:240-254)."""
    return K.pool_clip(tokens)
