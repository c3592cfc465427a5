"""GPU probe: GEMM implementations/tile configs — correctness (all layouts) and timing
against torch.mm (hipBLASLt) on the hot-path shapes.  python tools/gpu_probe_gemm.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "gpt2-vision-language_amd"))
from gvl import _lib  # noqa: E402
from gvl import kernels as K  # noqa: E402

L = _lib.load()
IMPLS = [("regstage", 0, -1), ("lds256x256", 1, 0), ("lds256x128", 1, 1), ("lds128x128", 1, 2),
         ("lds-auto", 1, -1), ("ring256", 2, 0), ("ring256x128", 2, 1), ("ring128", 2, 2),
         ("ring256s5", 2, 3), ("pp4", 2, 4), ("pp5", 2, 5)]
if os.environ.get("PROBE_ONLY_RING"):
    IMPLS = [x for x in IMPLS if x[1] == 2 or x[0] == "lds-auto"]


def mk(M, N, Kd, a_mn, b_mn, seed=0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    a = torch.randn(M, Kd, device="cuda", generator=g).bfloat16()
    b = torch.randn(Kd, N, device="cuda", generator=g).bfloat16()
    A = a.t().contiguous() if a_mn else a
    B = b.contiguous() if b_mn else b.t().contiguous()
    return a, b, A, B


def check():
    worst = 0.0
    for name, impl, cfg in IMPLS:
        L.gvl_gemm_tune(impl, cfg)
        for (M, N, Kd) in [(256, 256, 128), (200, 136, 192), (520, 264, 256), (64, 8, 64),
                           (264, 520, 96), (1032, 1024, 1024)]:
            for am, bm in [(0, 0), (0, 1), (1, 0), (1, 1)]:
                if (am and M % 8) or (bm and N % 8):
                    continue
                a, b, A, B = mk(M, N, Kd, am, bm, M + N)
                bias = torch.randn(N, device="cuda").bfloat16()
                res = torch.randn(M, N, device="cuda").bfloat16()
                c = K.gemm(A, B, a_mn=bool(am), b_mn=bool(bm), bias=bias, act=1, residual=res)
                ref = torch.nn.functional.gelu(a.float() @ b.float() + bias.float(),
                                               approximate="tanh") + res.float()
                rel = ((c.float() - ref).abs().max() / ref.abs().max()).item()
                worst = max(worst, rel)
                if rel > 1e-2:
                    print(f"FAIL {name} M={M} N={N} K={Kd} a_mn={am} b_mn={bm} rel={rel:.3g}",
                          flush=True)
    L.gvl_gemm_tune(1, -1)
    print("CHECK worst rel", worst, flush=True)
    return worst


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def bench(M, N, Kd, am, bm):
    a, b, A, B = mk(M, N, Kd, am, bm)
    c = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
    fl = 2.0 * M * N * Kd
    row = [f"M={M} N={N} K={Kd} a_mn={am} b_mn={bm}:"]
    for name, impl, cfg in IMPLS:
        L.gvl_gemm_tune(impl, cfg)
        ms = timeit(lambda: K.gemm(A, B, a_mn=bool(am), b_mn=bool(bm), out=c))
        row.append(f"{name} {fl / ms / 1e9:.0f}")
    L.gvl_gemm_tune(1, -1)
    at = A.t() if am else A
    bt = B if bm else B.t()
    ms = timeit(lambda: torch.mm(at, bt))
    row.append(f"torch {fl / ms / 1e9:.0f} TF/s")
    print(" | ".join(row), flush=True)


if __name__ == "__main__":
    w = check()
    for shp in [(8064, 768, 768, 0, 0), (8064, 2304, 768, 0, 0), (8064, 3072, 768, 0, 0),
                (8064, 768, 3072, 0, 0), (8064, 50304, 768, 0, 0), (8064, 768, 2304, 0, 1),
                (8064, 768, 3072, 0, 1), (8064, 3072, 768, 0, 1), (3968, 768, 50304, 0, 1),
                (16384, 2304, 768, 0, 0), (16384, 50304, 768, 0, 0), (16384, 768, 3072, 0, 1),
                (768, 3072, 16384, 1, 1), (50304, 768, 16384, 1, 1), (4096, 3072, 768, 0, 0),
                (8192, 8192, 8192, 0, 0)]:
        bench(*shp)
    sys.exit(0 if w < 1e-2 else 1)
