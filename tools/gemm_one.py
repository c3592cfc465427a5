"""Run one GEMM shape with one kernel config repeatedly (for rocprofv3 PMC passes).
python tools/gemm_one.py M N K a_mn b_mn impl cfg [iters] [epi]   (impl 9 = torch.mm;
epi: plain | bias | act (bias + gelu-tanh storing gelu') | dact (x gelu' operand) | bias_res)"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "gpt2-vision-language_amd"))
from gvl import _lib  # noqa: E402
from gvl import kernels as K  # noqa: E402

M, N, Kd, am, bm, impl, cfg = (int(x) for x in sys.argv[1:8])
iters = int(sys.argv[8]) if len(sys.argv) > 8 else 10
epi = sys.argv[9] if len(sys.argv) > 9 else "plain"
L = _lib.load()
g = torch.Generator(device="cuda").manual_seed(0)
A = (torch.randn(Kd, M, device="cuda", generator=g) if am else
     torch.randn(M, Kd, device="cuda", generator=g)).bfloat16()
B = (torch.randn(Kd, N, device="cuda", generator=g) if bm else
     torch.randn(N, Kd, device="cuda", generator=g)).bfloat16()
C = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
aux = torch.randn(M, N, device="cuda", generator=g).bfloat16()
bias = torch.randn(N, device="cuda", generator=g).bfloat16()
kw = {"plain": {}, "bias": dict(bias=bias), "act": dict(bias=bias, act=3, pre_out=aux),
      "dact": dict(dact=3, pre_in=aux), "bias_res": dict(bias=bias, residual=aux)}[epi]
if impl < 9:
    L.gvl_gemm_tune(impl, cfg)
    fn = lambda: K.gemm(A, B, a_mn=bool(am), b_mn=bool(bm), out=C, **kw)  # noqa: E731
else:
    at = A.t() if am else A
    bt = B if bm else B.t()
    fn = lambda: torch.mm(at, bt, out=C)  # noqa: E731
for _ in range(3):
    fn()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(iters):
    fn()
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / iters
print(f"M={M} N={N} K={Kd} epi={epi} impl={impl} cfg={cfg}: {ms:.3f} ms {2.0 * M * N * Kd / ms / 1e9:.0f} TF/s")
