"""Row sweep of the wide K = 768 GEMMs (c_fc + bias + GELU with the pre-activation saved, the
mlp.c_proj dX * gelu', and the plain product of the same shape): time against M separates a
launch's fixed cost (ramp, tail, launch gap) from its per-tile cost.  Also times an empty
torch kernel (the launch gap alone).  HIP events, median of 5 x 20 launches, uniform [-1, 1)
operands.  python tools/pp3_sweep.py [N] [K]   (GVL_LIB=... for a variant build)"""
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpt2-vision-language_amd"))
from gvl import _lib  # noqa: E402
from gvl import kernels as K  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 3072
KD = int(sys.argv[2]) if len(sys.argv) > 2 else 768
_lib.load()
g = torch.Generator(device="cuda").manual_seed(0)
rnd = lambda *s: (torch.rand(*s, device="cuda", generator=g) * 2 - 1).bfloat16()  # noqa: E731


def timed(fn, n=20):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3  # us


def med(fn):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    return statistics.median(timed(fn) for _ in range(5))


x = torch.zeros(16, device="cuda")
print(f"empty kernel {med(lambda: x.add_(1)):6.2f} us", flush=True)
for M in (1024, 2048, 4096, 6144, 8064, 8192, 12288, 16384, 32768):
    A, W = rnd(M, KD), rnd(N, KD)
    Wt = rnd(KD, N)
    C, aux, bias = (torch.empty(M, N, dtype=torch.bfloat16, device="cuda"), rnd(M, N), rnd(N))
    cases = {"plain": lambda: K.gemm(A, W, out=C),
             "act": lambda: K.gemm(A, W, out=C, bias=bias, act=3, pre_out=aux),
             "dact": lambda: K.gemm(A, Wt, b_mn=True, out=C, dact=3, pre_in=aux)}
    t = {k: med(f) for k, f in cases.items()}
    fl = 2.0 * M * N * KD
    tiles = ((M + 255) // 256) * ((N + 191) // 192)
    print(f"M={M:6d} tiles(256x192)={tiles:5d} " + " ".join(
        f"{k} {v:7.1f}us ({fl / v / 1e6:5.0f} TF/s)" for k, v in t.items()), flush=True)
    del A, W, Wt, C, aux
