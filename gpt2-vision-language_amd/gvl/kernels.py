"""Typed Python wrappers over the libgvl C-ABI (one function per entry point of include/gvl.h).

Every wrapper takes torch tensors that already live on the current ROCm device, checks
dtype/layout on the host, and launches on torch.cuda.current_stream().  There is no CPU
path: a CPU tensor is rejected with a clear error.
"""
from __future__ import annotations

import ctypes as C
import math

import os

import torch

from . import _lib
from ._lib import AttnBwdDesc, AttnDesc, GemmDesc

BF16 = torch.bfloat16
F32 = torch.float32


def _L():
    return _lib.lib()


def _stream():
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


def _p(t):
    return None if t is None else t.data_ptr()


def _dev(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise RuntimeError(
                "gvl: the HIP kernel path needs tensors on a ROCm GPU (got a CPU tensor); "
                "there is no CPU fallback in the product path")


def _rowmajor(t, name):
    if t.dim() != 2 or t.stride(1) != 1:
        raise ValueError(f"gvl: {name} must be a 2-D row-major view (got shape {tuple(t.shape)}, "
                         f"strides {t.stride()})")


# ------------------------------------------------------------------ live kernel timing
class KernelTimer:
    """Times every GEMM launch with a pair of HIP events (bench.py's roofline line).

    dispatch=True (default): the events are bound to the GEMM kernel's own dispatch
    (gvl_set_launch_events -> hipExtLaunchKernelGGL), so each interval is the kernel's
    execution as its dispatch records it — the quantity rocprofv3's kernel trace reports.
    dispatch=False: two stream markers around the launch (includes dispatch latency)."""

    def __init__(self, dispatch: bool = True):
        self.records = []
        self.dispatch = dispatch

    def summary(self):
        torch.cuda.synchronize()
        out = {}
        for name, e0, e1, flops in self.records:
            s = out.setdefault(name, {"launches": 0, "ms": 0.0, "flops": 0.0})
            s["launches"] += 1
            s["ms"] += e0.elapsed_time(e1)
            s["flops"] += flops
        return out


_timer = None


def set_kernel_timer(t):
    global _timer
    _timer = t


GEMM_NAMES = {(0, 0): "gemm_bf16_kernel<false,false>", (0, 1): "gemm_bf16_kernel<false,true>",
              (1, 0): "gemm_bf16_kernel<true,false>", (1, 1): "gemm_bf16_kernel<true,true>"}


_WS = {}
GEMM_WORKSPACE_MB = 64


def _gemm_workspace(device):
    """Per-device fp32 split-K scratch, allocated once (stream-ordered reuse; allocate it
    before any hipGraph capture — bench/train warm up eagerly first)."""
    key = device.index if device.index is not None else torch.cuda.current_device()
    ws = _WS.get(key)
    if ws is None:
        ws = torch.empty(GEMM_WORKSPACE_MB * 1024 * 1024 // 4, dtype=F32, device=device)
        _WS[key] = ws
    return ws


_TK = {}
GEMM_TICKETS = 1 << 16
# Arrival tickets (gvl.h ABI v5) go with every gvl_gemm call; the persistent kernel's in-launch
# two-way combine that uses them stays off unless GVL_PP3_COMBINE=1 (checked in C, gemm_plan.hip).
# Batched weight gradients may use it (gvl_gemm_batched decides; GVL_BATCHED_SPLIT=0: never).
BATCHED_SPLIT = os.environ.get("GVL_BATCHED_SPLIT", "1") != "0"


def _gemm_tickets(device):
    """Per-device arrival tickets of the in-launch two-way split-K combine (gvl.h ABI v5):
    zero-filled once; every GEMM call leaves them zero again."""
    key = device.index if device.index is not None else torch.cuda.current_device()
    t = _TK.get(key)
    if t is None:
        t = torch.zeros(GEMM_TICKETS, dtype=torch.int32, device=device)
        _TK[key] = t
    return t


# ------------------------------------------------------------- device dropout offset
_SEED_OFF = {}


def seed_offset(device):
    """Per-device int64 step offset that re-keys every dropout seed on the device
    (include/gvl.h: seed_eff).  It stays 0 in eager use; gvl.graph advances it once per
    replay of a captured step so frozen host seeds still draw fresh masks."""
    key = device.index if device.index is not None else torch.cuda.current_device()
    t = _SEED_OFF.get(key)
    if t is None:
        t = torch.zeros(1, dtype=torch.int64, device=device)
        _SEED_OFF[key] = t
    return t


# ------------------------------------------------------------------------------- GEMM
def gemm(a, b, *, a_mn=False, b_mn=False, out=None, alpha=1.0, alpha_ptr=None, bias=None,
         act=0, dact=0, pre_out=None, pre_in=None, residual=None, gate=None, drop_p=0.0,
         seed=0, seed_ptr=None, out_dtype=BF16):
    """C = epi(alpha * opA @ opB).  a: [M,K] (a_mn=False) or [K,M]; b: [N,K] (b_mn=False,
    nn.Linear weight) or [K,N].  Returns C [M,N]."""
    _dev(a, b)
    _rowmajor(a, "A")
    _rowmajor(b, "B")
    if a.dtype != BF16 or b.dtype != BF16:
        raise TypeError("gvl.gemm: operands must be bf16")
    M, K = (a.shape[1], a.shape[0]) if a_mn else (a.shape[0], a.shape[1])
    N, Kb = (b.shape[1], b.shape[0]) if b_mn else (b.shape[0], b.shape[1])
    if K != Kb:
        raise ValueError(f"gvl.gemm: inner dims differ ({K} vs {Kb})")
    if out is None:
        out = torch.empty(M, N, dtype=out_dtype, device=a.device)
    _rowmajor(out, "C")
    d = GemmDesc()
    d.a, d.b, d.c = a.data_ptr(), b.data_ptr(), out.data_ptr()
    d.m, d.n, d.k = M, N, K
    d.lda, d.ldb, d.ldc = a.stride(0), b.stride(0), out.stride(0)
    d.a_mn, d.b_mn = int(a_mn), int(b_mn)
    d.alpha = float(alpha)
    d.alpha_ptr = _p(alpha_ptr)
    d.bias = _p(bias)
    d.act, d.dact = int(act), int(dact)
    d.pre_out = _p(pre_out)
    d.pre_in = _p(pre_in)
    pre = pre_out if pre_out is not None else pre_in
    d.ldp = pre.stride(0) if pre is not None else 0
    d.residual = _p(residual)
    d.ldr = residual.stride(0) if residual is not None else 0
    d.gate = _p(gate)
    d.drop_p = float(drop_p)
    d.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    d.seed_ptr = _p(seed_ptr)
    d.c_fp32 = int(out.dtype == F32)
    ws = _gemm_workspace(a.device)
    d.workspace, d.workspace_bytes = ws.data_ptr(), ws.numel() * 4
    tk = _gemm_tickets(a.device)
    d.tickets, d.ticket_count = tk.data_ptr(), tk.numel()
    if _timer is not None:
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        if _timer.dispatch:
            e0.record()  # materialise both hipEvents; the launch re-records them
            e1.record()
            _L().gvl_set_launch_events(C.c_void_p(e0.cuda_event), C.c_void_p(e1.cuda_event))
            try:
                _lib.check(_L().gvl_gemm(C.byref(d), _stream()), "gvl_gemm")
            finally:
                _L().gvl_set_launch_events(None, None)
        else:
            e0.record()
            _lib.check(_L().gvl_gemm(C.byref(d), _stream()), "gvl_gemm")
            e1.record()
        buf = C.create_string_buffer(128)
        _L().gvl_gemm_kernel_name(C.byref(d), buf, 128)
        _timer.records.append((buf.value.decode(), e0, e1, 2.0 * M * N * K))
        return out
    _lib.check(_L().gvl_gemm(C.byref(d), _stream()), "gvl_gemm")
    return out


def linear(x2, w, bias=None, **kw):
    """y = x2 @ w.T (+bias) — nn.Linear forward on a [rows, in] view."""
    return gemm(x2, w, bias=bias, **kw)


def linear_dx(dy2, w, **kw):
    """dx = dy2 @ w — nn.Linear input gradient (w stored [out, in] is MN-major here)."""
    return gemm(dy2, w, b_mn=True, **kw)


def linear_dw(dy2, x2, **kw):
    """dW = dy2.T @ x2 — nn.Linear weight gradient ([out, in])."""
    return gemm(dy2, x2, a_mn=True, b_mn=True, **kw)


def gemm_batched(items, *, a_mn=False, b_mn=False, dbias=None):
    """items: [(a, b, out, accumulate)] of one shape and layout: out (+)= op(a) @ op(b) for
    every item as ONE persistent launch (gvl_gemm_batched; falls back to one launch each
    when the library cannot batch them).  dbias (weight gradients only: a_mn = b_mn, every
    item accumulating): bf16 [M] bias grads, dbias[i] += column sums of items[i]'s dY, fused
    into the same launch (gvl_gemm_batched_dbias); returns False (nothing launched) when the
    batch cannot run fused."""
    n = len(items)
    if n == 0:
        return
    arr = (GemmDesc * n)()
    ws = None
    for i, (a, b, out, acc) in enumerate(items):
        _dev(a, b)
        _rowmajor(a, "A")
        _rowmajor(b, "B")
        _rowmajor(out, "C")
        if a.dtype != BF16 or b.dtype != BF16 or out.dtype != BF16:
            raise TypeError("gvl.gemm_batched: operands must be bf16")
        M, K_ = (a.shape[1], a.shape[0]) if a_mn else (a.shape[0], a.shape[1])
        N, Kb = (b.shape[1], b.shape[0]) if b_mn else (b.shape[0], b.shape[1])
        if K_ != Kb or tuple(out.shape) != (M, N):
            raise ValueError("gvl.gemm_batched: shape mismatch")
        d = arr[i]
        d.a, d.b, d.c = a.data_ptr(), b.data_ptr(), out.data_ptr()
        d.m, d.n, d.k = M, N, K_
        d.lda, d.ldb, d.ldc = a.stride(0), b.stride(0), out.stride(0)
        d.a_mn, d.b_mn = int(a_mn), int(b_mn)
        d.alpha = 1.0
        if acc:
            d.residual, d.ldr = out.data_ptr(), out.stride(0)
        if ws is None:
            ws = _gemm_workspace(a.device)
            tk = _gemm_tickets(a.device) if BATCHED_SPLIT else None
        d.workspace, d.workspace_bytes = ws.data_ptr(), ws.numel() * 4
        if tk is not None:  # the library may split a batch that underfills the chip in two
            d.tickets, d.ticket_count = tk.data_ptr(), tk.numel()
    ev = None
    if _timer is not None and _timer.dispatch:  # bound to the batched kernel's own dispatch
        ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        ev[0].record()
        ev[1].record()
        _L().gvl_set_launch_events(C.c_void_p(ev[0].cuda_event), C.c_void_p(ev[1].cuda_event))
    try:
        if dbias is not None:
            for t in dbias:
                if t.dtype != BF16 or not t.is_contiguous():
                    raise ValueError("gvl.gemm_batched: dbias must be contiguous bf16")
            da = (C.c_void_p * n)(*[t.data_ptr() for t in dbias])
            rc = _L().gvl_gemm_batched_dbias(arr, da, n, _stream())
            if rc not in (0, -1):  # -1: nothing launched, the caller runs the unfused pair
                _lib.check(rc, "gvl_gemm_batched_dbias")
            ok = rc == 0
        else:
            _lib.check(_L().gvl_gemm_batched(arr, n, _stream()), "gvl_gemm_batched")
            ok = True
    finally:
        if ev is not None:
            _L().gvl_set_launch_events(None, None)
    if ev is not None and ok:
        buf = C.create_string_buffer(128)
        _L().gvl_gemm_batched_kernel_name(buf, 128)
        if buf.value:  # one batched launch (not the per-problem fallback)
            flops = sum(2.0 * arr[i].m * arr[i].n * arr[i].k for i in range(n))
            _timer.records.append((buf.value.decode(), ev[0], ev[1], flops))
    return ok


def gemm_grouped(items, dbias=None):
    """Weight gradients of different shapes as ONE launch (gvl_gemm_grouped): items =
    [(dy, x, out)], out += dy^T @ x (dy [K_i, M_i], x [K_i, N_i], out [M_i, N_i], bf16,
    MN-contiguous operands); an item may carry a 4th element, an fp32 device scalar (or None)
    its product is scaled by (ABI v11: one such tensor per call); dbias: None or a list with a
    bf16 [M_i] bias grad or None per item, += column sums of dy_i.  Returns False when nothing
    was launched (the caller runs the problems another way)."""
    n = len(items)
    if n == 0:
        return True
    arr = (GemmDesc * n)()
    for i, it in enumerate(items):
        a, b, out = it[:3]
        ap = it[3] if len(it) > 3 else None
        if ap is not None and (ap.dtype != torch.float32 or not ap.is_cuda):
            raise TypeError("gvl.gemm_grouped: alpha_ptr must be an fp32 device tensor")
        _dev(a, b)
        _rowmajor(a, "A")
        _rowmajor(b, "B")
        _rowmajor(out, "C")
        if a.dtype != BF16 or b.dtype != BF16 or out.dtype != BF16:
            raise TypeError("gvl.gemm_grouped: operands must be bf16")
        if a.shape[0] != b.shape[0] or tuple(out.shape) != (a.shape[1], b.shape[1]):
            raise ValueError("gvl.gemm_grouped: shape mismatch")
        d = arr[i]
        d.a, d.b, d.c = a.data_ptr(), b.data_ptr(), out.data_ptr()
        d.m, d.n, d.k = a.shape[1], b.shape[1], a.shape[0]
        d.lda, d.ldb, d.ldc = a.stride(0), b.stride(0), out.stride(0)
        d.a_mn, d.b_mn = 1, 1
        d.alpha = 1.0
        d.alpha_ptr = _p(ap)
        d.residual, d.ldr = out.data_ptr(), out.stride(0)
    da = None
    if dbias is not None:
        for t in dbias:
            if t is not None and (t.dtype != BF16 or not t.is_contiguous()):
                raise ValueError("gvl.gemm_grouped: dbias must be contiguous bf16")
        da = (C.c_void_p * n)(*[(t.data_ptr() if t is not None else None) for t in dbias])
    ev = None
    if _timer is not None and _timer.dispatch:
        ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        ev[0].record()
        ev[1].record()
        _L().gvl_set_launch_events(C.c_void_p(ev[0].cuda_event), C.c_void_p(ev[1].cuda_event))
    try:
        rc = _L().gvl_gemm_grouped(arr, da, n, _stream())
        if rc not in (0, -1):
            _lib.check(rc, "gvl_gemm_grouped")
    finally:
        if ev is not None:
            _L().gvl_set_launch_events(None, None)
    if rc == 0 and ev is not None:
        buf = C.create_string_buffer(128)
        _L().gvl_gemm_batched_kernel_name(buf, 128)
        flops = sum(2.0 * arr[i].m * arr[i].n * arr[i].k for i in range(n))
        _timer.records.append((buf.value.decode(), ev[0], ev[1], flops))
    return rc == 0


# ------------------------------------------------------------------------- LayerNorm
def layernorm_fwd(x2, w, b, eps=1e-5, out=None, stats=True):
    _dev(x2)
    _rowmajor(x2, "x")
    rows, cols = x2.shape
    if out is None:
        out = torch.empty(rows, cols, dtype=BF16, device=x2.device)
    mean = torch.empty(rows, dtype=F32, device=x2.device) if stats else None
    rstd = torch.empty(rows, dtype=F32, device=x2.device) if stats else None
    _lib.check(_L().gvl_layernorm_fwd(x2.data_ptr(), x2.stride(0), w.data_ptr(), b.data_ptr(),
                                      out.data_ptr(), out.stride(0), _p(mean), _p(rstd), rows, cols,
                                      float(eps), _stream()), "gvl_layernorm_fwd")
    return out, mean, rstd


def layernorm_bwd(dy2, x2, w, mean, rstd, dx=None, accumulate_dx=False, dw=None, db=None,
                  accumulate_wb=False, residual=None, defer_wb=False):
    """dx [= dx | residual] + LayerNorm backward; `residual` (a [rows, cols] bf16 operand read
    instead of dx, gvl_layernorm_bwd_res) saves the caller a copy of the residual gradient.
    defer_wb (ABI v12): the dw / db column sums are left as per-block partials; returns
    (dx, (workspace, blocks)) for a later layernorm_finalize_batched."""
    rows, cols = x2.shape
    if dx is None:
        dx = torch.empty(rows, cols, dtype=BF16, device=x2.device)
    ws = None
    if dw is not None or db is not None or defer_wb:
        n = _L().gvl_layernorm_bwd_workspace_size(rows, cols)
        ws = torch.empty(max(n, 4) // 4, dtype=F32, device=x2.device)
    if defer_wb:
        dw = db = None
        accumulate_wb = 2
    if residual is not None:
        _lib.check(_L().gvl_layernorm_bwd_res(
            dy2.data_ptr(), dy2.stride(0), x2.data_ptr(), x2.stride(0), w.data_ptr(),
            mean.data_ptr(), rstd.data_ptr(), residual.data_ptr(), residual.stride(0),
            dx.data_ptr(), dx.stride(0), _p(dw), _p(db), int(accumulate_wb), _p(ws), rows, cols,
            _stream()), "gvl_layernorm_bwd_res")
    else:
        _lib.check(_L().gvl_layernorm_bwd(dy2.data_ptr(), dy2.stride(0), x2.data_ptr(), x2.stride(0),
                                          w.data_ptr(), mean.data_ptr(), rstd.data_ptr(), dx.data_ptr(),
                                          dx.stride(0), int(accumulate_dx), _p(dw), _p(db),
                                          int(accumulate_wb), _p(ws), rows, cols, _stream()),
                   "gvl_layernorm_bwd")
    if defer_wb:
        return dx, (ws, int(_L().gvl_layernorm_bwd_blocks(rows)))
    return dx


def layernorm_finalize_batched(items, cols, accumulate=True):
    """The deferred LayerNorm weight / bias gradients of one width: items = [(workspace,
    blocks, dw or None, db or None)] from layernorm_bwd(defer_wb=True); one launch per 64."""
    for i in range(0, len(items), 64):
        chunk = items[i:i + 64]
        n = len(chunk)
        ws = (C.c_void_p * n)(*[t[0].data_ptr() for t in chunk])
        nb = (C.c_int32 * n)(*[t[1] for t in chunk])
        dw = (C.c_void_p * n)(*[_p(t[2]) for t in chunk])
        db = (C.c_void_p * n)(*[_p(t[3]) for t in chunk])
        _lib.check(_L().gvl_layernorm_bwd_finalize_batched(ws, nb, n, int(cols), dw, db,
                                                           int(bool(accumulate)), _stream()),
                   "gvl_layernorm_bwd_finalize_batched")


# ------------------------------------------------------------------------- attention
def _bthd(t, T, H):
    """strides (b, t, h) of a [B, T, *] tensor whose head h occupies cols h*64..h*64+63."""
    return t.stride(0), t.stride(1), 64


def attn_desc(q, k, v, o, lse, B, H, Tq, Tk, causal, scale, drop_p=0.0, seed=0, seed_ptr=None):
    d = AttnDesc()
    d.q, d.k, d.v, d.o, d.lse = q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), _p(lse)
    d.B, d.H, d.Tq, d.Tk = B, H, Tq, Tk
    d.q_sb, d.q_st, d.q_sh = q.stride(0), q.stride(1), 64
    d.k_sb, d.k_st, d.k_sh = k.stride(0), k.stride(1), 64
    d.v_sb, d.v_st, d.v_sh = v.stride(0), v.stride(1), 64
    d.o_sb, d.o_st, d.o_sh = o.stride(0), o.stride(1), 64
    d.causal = int(causal)
    d.scale = float(scale)
    d.drop_p = float(drop_p)
    d.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    d.seed_ptr = _p(seed_ptr)
    return d


def attn_fwd(q, k, v, H, causal, scale=None, drop_p=0.0, seed=0, out=None, seed_ptr=None):
    """q: [B,Tq,*] view whose cols h*64.. are head h (e.g. a slice of packed qkv);
    k, v: [B,Tk,*].  Returns (o [B,Tq,H*64] bf16, lse [B,H,Tq] fp32)."""
    _dev(q, k, v)
    for t in (q, k, v):
        if t.dtype != BF16 or t.stride(2) != 1:
            raise ValueError("gvl.attn_fwd: q/k/v must be bf16 with unit last stride")
    B, Tq = q.shape[0], q.shape[1]
    Tk = k.shape[1]
    if scale is None:
        scale = 1.0 / math.sqrt(64)
    if out is None:
        out = torch.empty(B, Tq, H * 64, dtype=BF16, device=q.device)
    lse = torch.empty(B, H, Tq, dtype=F32, device=q.device)
    d = attn_desc(q, k, v, out, lse, B, H, Tq, Tk, causal, scale, drop_p, seed, seed_ptr)
    _lib.check(_L().gvl_attn_fwd(C.byref(d), _stream()), "gvl_attn_fwd")
    return out, lse


def attn_bwd(dout, q, k, v, o, lse, H, causal, dq, dk, dv, scale=None, drop_p=0.0, seed=0,
             seed_ptr=None):
    """Writes dq/dk/dv (views with the layouts of q/k/v)."""
    B, Tq = q.shape[0], q.shape[1]
    Tk = k.shape[1]
    if scale is None:
        scale = 1.0 / math.sqrt(64)
    d = attn_desc(q, k, v, o, lse, B, H, Tq, Tk, causal, scale, drop_p, seed, seed_ptr)
    g = AttnBwdDesc()
    g.dout, g.do_sb, g.do_st, g.do_sh = dout.data_ptr(), dout.stride(0), dout.stride(1), 64
    g.dq, g.dq_sb, g.dq_st, g.dq_sh = dq.data_ptr(), dq.stride(0), dq.stride(1), 64
    g.dk, g.dk_sb, g.dk_st, g.dk_sh = dk.data_ptr(), dk.stride(0), dk.stride(1), 64
    g.dv, g.dv_sb, g.dv_st, g.dv_sh = dv.data_ptr(), dv.stride(0), dv.stride(1), 64
    n = _L().gvl_attn_bwd_workspace_size(C.byref(d))
    ws = torch.empty(max(n, 4) // 4, dtype=F32, device=q.device)
    g.workspace = ws.data_ptr()
    _lib.check(_L().gvl_attn_bwd(C.byref(d), C.byref(g), _stream()), "gvl_attn_bwd")


def attn_decode(q, k, v, H, out=None, scale=None):
    """One new query per sequence over a KV cache: q [B, *] (head h at cols h*64..), k/v
    [B, Tk, *] strided views (e.g. slices of a packed [B, Tmax, 3C] cache).  -> o [B, H*64]."""
    _dev(q, k, v)
    B, Tk = k.shape[0], k.shape[1]
    if out is None:
        out = torch.empty(B, H * 64, dtype=BF16, device=q.device)
    if scale is None:
        scale = 1.0 / math.sqrt(64)
    _lib.check(_L().gvl_attn_decode(q.data_ptr(), q.stride(0), k.data_ptr(), k.stride(0),
                                    k.stride(1), v.data_ptr(), v.stride(0), v.stride(1),
                                    out.data_ptr(), out.stride(0), B, H, Tk, float(scale),
                                    _stream()), "gvl_attn_decode")
    return out


def sample(logits2, u, temperature=1.0, top_k=0, top_p=1.0, out=None):
    """Fused temperature / top-k / top-p draw per row (include/gvl.h gvl_sample); u [rows]
    fp32 uniforms in [0, 1) on the device.  -> int64 [rows]."""
    _dev(logits2, u)
    _rowmajor(logits2, "logits")
    rows, V = logits2.shape
    if out is None:
        out = torch.empty(rows, dtype=torch.int64, device=logits2.device)
    _lib.check(_L().gvl_sample(logits2.data_ptr(), logits2.stride(0), int(logits2.dtype == F32),
                               rows, V, float(temperature), int(top_k), float(top_p),
                               u.data_ptr(), out.data_ptr(), _stream()), "gvl_sample")
    return out


# ---------------------------------------------------------------------- cross entropy
def cross_entropy(logits2, targets, *, rows_per_group=None, group_stride=0, row_offset=0,
                  mask=None, mask_mode=False, want_grad=True, vocab=None):
    """Returns (loss_and_inv [2] fp32 device tensor, dlogits [rows, V] bf16 or None).
    `vocab` < logits2.shape[1] marks the trailing columns as padding (V % 8 != 0)."""
    _dev(logits2, targets)
    Vp = logits2.shape[1]
    V = Vp if vocab is None else int(vocab)
    rows = targets.numel()
    if rows_per_group is None:
        rows_per_group = max(rows, 1)
    tg = targets.reshape(-1)
    if tg.dtype != torch.int64:
        tg = tg.long()
    tg = tg.contiguous()
    mk = None
    if mask is not None:
        mk = mask.reshape(-1).to(torch.uint8).contiguous()
    row_loss = torch.empty(max(rows, 1), dtype=F32, device=logits2.device)
    dl = torch.empty(rows, Vp, dtype=BF16, device=logits2.device) if want_grad else None
    out = torch.empty(2, dtype=F32, device=logits2.device)
    _lib.check(_L().gvl_cross_entropy(logits2.data_ptr(), logits2.stride(0), rows, V,
                                      rows_per_group, group_stride, row_offset, tg.data_ptr(),
                                      _p(mk), int(mask_mode), row_loss.data_ptr(), _p(dl),
                                      dl.stride(0) if dl is not None else 0, out.data_ptr(),
                                      _stream()), "gvl_cross_entropy")
    return out, dl


# -------------------------------------------------------------------------- embedding
def embedding_fwd(idx, wte, wpe, out, T, out_rows_per_seq, out_offset):
    _dev(idx, wte, wpe, out)
    idx = idx.contiguous()
    V, C_ = wte.shape
    _lib.check(_L().gvl_embedding_fwd(idx.data_ptr(), wte.data_ptr(), wpe.data_ptr(),
                                      out.data_ptr(), idx.numel(), T, C_, V, out_rows_per_seq,
                                      out_offset, _stream()), "gvl_embedding_fwd")
    return out


def embedding_bwd(idx, dout, dwte_acc, dwpe_acc, T, out_rows_per_seq, out_offset, C_, V):
    idx = idx.contiguous()
    _lib.check(_L().gvl_embedding_bwd(idx.data_ptr(), dout.data_ptr(), _p(dwte_acc),
                                      _p(dwpe_acc), idx.numel(), T, C_, V, out_rows_per_seq,
                                      out_offset, _stream()), "gvl_embedding_bwd")


def copy_rows(src, dst, T, G, src_rows, src_off, dst_rows, dst_off, zero_rest=False):
    """Grouped row copy (gvl_copy_rows) between row-major bf16 2-D views: dst row
    (g*dst_rows + dst_off + t) = src row (g*src_rows + src_off + t); zero_rest zeroes the
    other rows of every dst group.  src_rows = 0 broadcasts T rows to all G groups."""
    _dev(src, dst)
    if src.dtype != BF16 or dst.dtype != BF16 or src.stride(-1) != 1 or dst.stride(-1) != 1:
        raise TypeError("gvl.copy_rows: bf16 row-major views expected")
    _lib.check(_L().gvl_copy_rows(src.data_ptr(), src.stride(0), src_rows, src_off,
                                  dst.data_ptr(), dst.stride(0), dst_rows, dst_off, T, G,
                                  dst.shape[-1], int(zero_rest), _stream()), "gvl_copy_rows")
    return dst


_EMB_KEYS = {}


def embedding_bwd_det(idx, dout, dwte, dwpe, T, out_rows_per_seq, out_offset, C_, V):
    """Deterministic embedding backward into bf16 gradients, accumulating in place
    (gvl_embedding_bwd_det): dwte [V, C] += per-id row sums, dwpe [P, C] += per-position sums."""
    _dev(idx, dout)
    idx = idx.contiguous()
    n = idx.numel()
    for t in (dwte, dwpe):
        if t is not None and (t.dtype != BF16 or not t.is_contiguous()):
            raise TypeError("gvl.embedding_bwd_det: gradients must be contiguous bf16")
    keys = None
    if dwte is not None:
        need = int(_L().gvl_embedding_bwd_workspace(n))
        key = (dout.device, torch.cuda.current_stream(dout.device).cuda_stream)
        keys = _EMB_KEYS.get(key)
        if keys is None or keys.numel() < need:
            keys = torch.empty(max(need, 1), dtype=torch.int32, device=dout.device)
            _EMB_KEYS[key] = keys
    _lib.check(_L().gvl_embedding_bwd_det(idx.data_ptr(), dout.data_ptr(), _p(dwte), _p(dwpe), n,
                                          T, C_, V, out_rows_per_seq, out_offset, _p(keys),
                                          0 if keys is None else keys.numel(), _stream()),
               "gvl_embedding_bwd_det")


# ------------------------------------------------------------------------------- pool
def pool_clip(tokens, out_dtype=None, normalize=True):
    """[B, 1+s*s, D] -> [B, 33, D]: CLS + adaptive-avg (4,8) (+ L2 normalise)."""
    _dev(tokens)
    t = tokens.contiguous()
    if t.dtype not in (F32, BF16):
        t = t.float()
    B, L, D = t.shape
    out_dtype = out_dtype or t.dtype
    out = torch.empty(B, 33, D, dtype=out_dtype, device=t.device)
    _lib.check(_L().gvl_pool_clip_ex(t.data_ptr(), int(t.dtype == F32), out.data_ptr(),
                                     int(out_dtype == F32), B, L, D, int(normalize), _stream()),
               "gvl_pool_clip")
    return out


def l2_normalize_rows(x, out=None):
    """F.normalize(x, dim=-1, eps=1e-12) for bf16 / fp32 rows (D <= 1024)."""
    _dev(x)
    x = x.contiguous()
    if out is None:
        out = torch.empty_like(x)
    D = x.shape[-1]
    _lib.check(_L().gvl_l2_normalize_rows(x.data_ptr(), out.data_ptr(), int(x.dtype == F32),
                                          x.numel() // D, D, _stream()), "gvl_l2_normalize_rows")
    return out


# ------------------------------------------------------------------------- optimizer
def grad_norm(g_flat, max_norm, out=None):
    _dev(g_flat)
    n = g_flat.numel()
    ws = torch.empty(max(_L().gvl_grad_norm_workspace_size(n), 4) // 4, dtype=F32,
                     device=g_flat.device)
    if out is None:
        out = torch.empty(2, dtype=F32, device=g_flat.device)
    _lib.check(_L().gvl_grad_norm(g_flat.data_ptr(), n, float(max_norm), ws.data_ptr(),
                                  out.data_ptr(), _stream()), "gvl_grad_norm")
    return out


def adamw_dev(p, g, m, v, n_decay, hyper, beta1, beta2, eps, wd, grad_scale=None):
    """AdamW with lr / step read on the device from hyper[0:2] (graph-capturable)."""
    _dev(p, g, m, v, hyper)
    _lib.check(_L().gvl_adamw_dev(p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(),
                                  p.numel(), int(n_decay), hyper.data_ptr(), float(beta1),
                                  float(beta2), float(eps), float(wd), _p(grad_scale), _stream()),
               "gvl_adamw_dev")


def adamw_master_dev(p, p_master, g, m, v, n_decay, hyper, beta1, beta2, eps, wd,
                     grad_scale=None):
    """Mixed-precision AdamW: fp32 master / moments, bf16 compute copy p (gvl.h)."""
    _dev(p, p_master, g, m, v, hyper)
    if p_master.dtype != F32 or m.dtype != F32 or v.dtype != F32:
        raise TypeError("gvl.adamw_master_dev: master / moments must be fp32")
    _lib.check(_L().gvl_adamw_master_dev(p.data_ptr(), p_master.data_ptr(), g.data_ptr(),
                                         m.data_ptr(), v.data_ptr(), p.numel(), int(n_decay),
                                         hyper.data_ptr(), float(beta1), float(beta2), float(eps),
                                         float(wd), _p(grad_scale), _stream()),
               "gvl_adamw_master_dev")


def adamw(p, g, m, v, n_decay, lr, beta1, beta2, eps, wd, step, grad_scale=None):
    _dev(p, g, m, v)
    _lib.check(_L().gvl_adamw(p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), p.numel(),
                              int(n_decay), float(lr), float(beta1), float(beta2), float(eps),
                              float(wd), int(step), _p(grad_scale), _stream()), "gvl_adamw")


# ------------------------------------------------------------------------- elementwise
def colsum(x2, out=None, accumulate=False):
    rows, cols = x2.shape
    if out is None:
        out = torch.empty(cols, dtype=BF16, device=x2.device)
    ws = torch.empty(max(_L().gvl_colsum_workspace_size(rows, cols), 4) // 4, dtype=F32,
                     device=x2.device)
    _lib.check(_L().gvl_colsum(x2.data_ptr(), rows, cols, x2.stride(0), out.data_ptr(),
                               int(accumulate), ws.data_ptr(), _stream()), "gvl_colsum")
    return out


def colsum_batched(xs, outs, accumulate=False):
    """outs[i] (+)= column sums of xs[i] (one shape, <= 16 problems) in one launch pair."""
    n = len(xs)
    rows, cols = xs[0].shape
    for x, o in zip(xs, outs):
        _dev(x)
        if tuple(x.shape) != (rows, cols) or x.stride(0) != xs[0].stride(0) or x.stride(1) != 1:
            raise ValueError("gvl.colsum_batched: problems must share shape and row stride")
        if o.dtype != BF16 or o.numel() != cols or not o.is_contiguous():
            raise ValueError("gvl.colsum_batched: bad output")
    ws = torch.empty(max(_L().gvl_colsum_batched_workspace_size(n, rows, cols), 4) // 4,
                     dtype=F32, device=xs[0].device)
    xa = (C.c_void_p * n)(*[x.data_ptr() for x in xs])
    oa = (C.c_void_p * n)(*[o.data_ptr() for o in outs])
    _lib.check(_L().gvl_colsum_batched(xa, oa, n, rows, cols, xs[0].stride(0), int(accumulate),
                                       ws.data_ptr(), _stream()), "gvl_colsum_batched")


def dropout_mask_apply(x2, p, seed, out=None, seed_ptr=None):
    rows, cols = x2.shape
    if out is None:
        out = torch.empty(rows, cols, dtype=BF16, device=x2.device)
    _lib.check(_L().gvl_dropout_mask_apply(x2.data_ptr(), x2.stride(0), out.data_ptr(),
                                           out.stride(0), rows, cols, float(p),
                                           int(seed) & 0xFFFFFFFFFFFFFFFF, _p(seed_ptr),
                                           _stream()),
               "gvl_dropout_mask_apply")
    return out


def gate_bwd(dx, y, gate, gate_grad_f32=None, grad_bf16=None):
    """dy = tanh(gate) * dx; the gate gradient (1 - tanh^2) * sum(dx * y) added into
    gate_grad_f32 (fp32 scalar) or, with grad_bf16, into that bf16 scalar with autograd's
    roundings (ABI v13)."""
    n = dx.numel()
    dy = torch.empty_like(dx)
    ws = torch.empty(max(_L().gvl_gate_bwd_workspace_size(n), 4) // 4, dtype=F32,
                     device=dx.device)
    if grad_bf16 is not None:
        if grad_bf16.dtype != BF16 or grad_bf16.numel() != 1:
            raise TypeError("gvl.gate_bwd: grad_bf16 must be a bf16 scalar")
        _lib.check(_L().gvl_gate_bwd_acc_bf16(dx.data_ptr(), y.data_ptr(), gate.data_ptr(),
                                              dy.data_ptr(), grad_bf16.data_ptr(), n, ws.data_ptr(),
                                              _stream()), "gvl_gate_bwd_acc_bf16")
        return dy
    _lib.check(_L().gvl_gate_bwd(dx.data_ptr(), y.data_ptr(), gate.data_ptr(), dy.data_ptr(),
                                 gate_grad_f32.data_ptr(), n, ws.data_ptr(), _stream()),
               "gvl_gate_bwd")
    return dy


def f32_to_bf16(x, out, accumulate=False):
    _lib.check(_L().gvl_f32_to_bf16(x.data_ptr(), out.data_ptr(), x.numel(), int(accumulate),
                                    _stream()), "gvl_f32_to_bf16")
    return out
