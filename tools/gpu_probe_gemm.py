"""Early GPU probe: gvl_gemm layouts/epilogues vs torch fp32, plus a timing sweep.

Run on the GPU box: python tools/gpu_probe_gemm.py
"""
import ctypes as C
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "gpt2-vision-language_amd"))
from gvl._lib import GemmDesc  # noqa: E402

lib = C.CDLL(os.path.join(os.path.dirname(__file__), "..", "gpt2-vision-language_amd", "gvl", "libgvl.so"))
lib.gvl_gemm.argtypes = [C.POINTER(GemmDesc), C.c_void_p]
lib.gvl_last_error.restype = C.c_char_p


def gemm(A, B, M, N, K, a_mn, b_mn, bias=None, act=0, residual=None, c=None):
    if c is None:
        c = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
    d = GemmDesc()
    d.a, d.b, d.c = A.data_ptr(), B.data_ptr(), c.data_ptr()
    d.m, d.n, d.k = M, N, K
    d.lda, d.ldb, d.ldc = A.stride(0), B.stride(0), c.stride(0)
    d.a_mn, d.b_mn = a_mn, b_mn
    d.alpha = 1.0
    d.bias = bias.data_ptr() if bias is not None else None
    d.act = act
    d.residual = residual.data_ptr() if residual is not None else None
    d.ldr = residual.stride(0) if residual is not None else 0
    rc = lib.gvl_gemm(C.byref(d), C.c_void_p(torch.cuda.current_stream().cuda_stream))
    assert rc == 0, lib.gvl_last_error()
    return c


def check(M, N, K, a_mn, b_mn, **kw):
    torch.manual_seed(0)
    a = torch.randn(M, K, device="cuda").bfloat16()
    b = torch.randn(K, N, device="cuda").bfloat16()
    A = a.t().contiguous() if a_mn else a.contiguous()      # a_mn: stored [K][M]
    B = b.contiguous() if b_mn else b.t().contiguous()      # b_mn: stored [K][N] else [N][K]
    bias = torch.randn(N, device="cuda").bfloat16() if kw.get("bias") else None
    res = torch.randn(M, N, device="cuda").bfloat16() if kw.get("res") else None
    act = kw.get("act", 0)
    c = gemm(A, B, M, N, K, a_mn, b_mn, bias=bias, act=act, residual=res)
    ref = a.float() @ b.float()
    if bias is not None:
        ref = ref + bias.float()
    if act == 1:
        ref = torch.nn.functional.gelu(ref, approximate="tanh")
    if act == 2:
        ref = torch.nn.functional.gelu(ref)
    if res is not None:
        ref = ref + res.float()
    torch.cuda.synchronize()
    err = (c.float() - ref).abs().max().item()
    rel = err / ref.abs().max().item()
    print(f"M={M} N={N} K={K} a_mn={a_mn} b_mn={b_mn} {kw} maxabs={err:.4g} rel={rel:.3g}", flush=True)
    return rel


def bench(M, N, K, a_mn, b_mn, iters=20):
    a = torch.randn(K if a_mn else M, M if a_mn else K, device="cuda").bfloat16()
    b = torch.randn(K if b_mn else N, N if b_mn else K, device="cuda").bfloat16()
    c = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
    for _ in range(3):
        gemm(a, b, M, N, K, a_mn, b_mn, c=c)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        gemm(a, b, M, N, K, a_mn, b_mn, c=c)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / iters
    tf = 2 * M * N * K / ms / 1e9
    # torch reference timing
    at = a.t() if a_mn else a
    bt = b if b_mn else b.t()
    for _ in range(3):
        torch.mm(at, bt)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(iters):
        torch.mm(at, bt)
    e1.record()
    torch.cuda.synchronize()
    ms_t = e0.elapsed_time(e1) / iters
    print(f"BENCH M={M} N={N} K={K} a_mn={a_mn} b_mn={b_mn}: gvl {ms*1e3:.1f}us {tf:.0f} TF/s | "
          f"torch {ms_t*1e3:.1f}us {2*M*N*K/ms_t/1e9:.0f} TF/s", flush=True)


if __name__ == "__main__":
    worst = 0
    for (am, bm) in [(0, 0), (0, 1), (1, 0), (1, 1)]:
        worst = max(worst, check(256, 256, 128, am, bm))
        worst = max(worst, check(200, 136, 72, am, bm))
    worst = max(worst, check(384, 512, 768, 0, 0, bias=True, act=1))
    worst = max(worst, check(384, 512, 768, 0, 0, bias=True, act=2, res=True))
    print("WORST", worst, flush=True)
    for shp in [(8064, 768, 768, 0, 0), (8064, 2304, 768, 0, 0), (8064, 3072, 768, 0, 0),
                (8064, 768, 3072, 0, 0), (8064, 50304, 768, 0, 0), (8064, 768, 2304, 0, 1),
                (8064, 768, 3072, 0, 1), (3968, 768, 50304, 0, 1), (16384, 2304, 768, 0, 0),
                (768, 3072, 16384, 1, 1), (50304, 768, 16384, 1, 1), (8192, 8192, 8192, 0, 0)]:
        bench(*shp)
