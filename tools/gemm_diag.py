"""Decoder GEMM shapes with the model's exact epilogues: libgvl with the model epilogue, the same
GEMM with a plain epilogue, and torch.mm (hipBLASLt) as a yardstick.  Interleaved rounds in one
process (median of 5 rounds x 20 launches), HIP events, uniform [-1, 1) operands.
python tools/gemm_diag.py [M] [set]   set: narrow (N = 768 outputs, default) | wide (K = 768,
N >= 2304, plus the lm_head) | all.  GVL_DIAG_COLS=epi keeps only the gvl_epi column (variant
builds, GVL_LIB=...)."""
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpt2-vision-language_amd"))
from gvl import _lib  # noqa: E402
from gvl import kernels as K  # noqa: E402

M = int(sys.argv[1]) if len(sys.argv) > 1 else 8064
SET = sys.argv[2] if len(sys.argv) > 2 else "narrow"
L = _lib.load()
g = torch.Generator(device="cuda").manual_seed(0)
rnd = lambda *s: (torch.rand(*s, device="cuda", generator=g) * 2 - 1).bfloat16()  # noqa: E731
# (name, N, K, b_mn, epilogue)
NARROW = [("attn.c_proj+bias+res", 768, 768, 0, "bias_res"), ("mlp.c_proj+bias+res", 768, 3072, 0, "bias_res"),
          ("c_fc.dX", 768, 3072, 1, "plain"), ("attn.c_proj.dX", 768, 768, 1, "plain"),
          ("c_attn.dX", 768, 2304, 1, "plain")]
WIDE = [("c_attn+bias", 2304, 768, 0, "bias"), ("c_fc+bias+gelu'", 3072, 768, 0, "act"),
        ("mlp.c_proj.dX*gelu'", 3072, 768, 1, "dact"), ("lm_head", 50304, 768, 0, "plain")]
CASES = {"narrow": NARROW, "wide": WIDE, "all": WIDE + NARROW}[SET]
COLS = os.environ.get("GVL_DIAG_COLS", "all")


def timed(fn, n=20):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3  # us


for name, N, Kd, bm, epi in CASES:
    A = rnd(M, Kd)
    B = rnd(Kd, N) if bm else rnd(N, Kd)
    C = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
    aux, bias = rnd(M, N), rnd(N)
    kw = {"plain": {}, "bias": dict(bias=bias), "act": dict(bias=bias, act=3, pre_out=aux),
          "dact": dict(dact=3, pre_in=aux), "bias_res": dict(bias=bias, residual=aux)}[epi]
    fns = {"gvl_epi": lambda: K.gemm(A, B, b_mn=bool(bm), out=C, **kw)}
    if COLS == "all":
        fns["gvl_plain"] = lambda: K.gemm(A, B, b_mn=bool(bm), out=C)
        fns["torch.mm"] = lambda: torch.mm(A, B if bm else B.t(), out=C)
    for f in fns.values():
        for _ in range(3):
            f()
    torch.cuda.synchronize()
    res = {k: [] for k in fns}
    for _ in range(5):
        for k, f in fns.items():
            res[k].append(timed(f))
    med = {k: statistics.median(v) for k, v in res.items()}
    flop = 2.0 * M * N * Kd
    line = f"{name:24s} N={N:5d} K={Kd:5d} " + " ".join(
        f"{k} {v:7.1f}us ({flop / v / 1e6:6.0f} TF/s)" for k, v in med.items())
    print(line, flush=True)
    del A, B, C, aux
