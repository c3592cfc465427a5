"""Time every GEMM shape of the LM and Q-Former steps: libgvl (default pick and forced
configs) next to torch.mm (hipBLASLt) as a yardstick.  One process, HIP events.
python tools/gemm_shapes.py [lm|qf|xa|all] [impl:cfg comma list; 2:-1 = default pick]"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "gpt2-vision-language_amd"))
from gvl import _lib  # noqa: E402
from gvl import kernels as K  # noqa: E402

T = 16384  # LM tokens per micro-step
Q = 8064   # Q-Former caption rows (128 x 63)
QT = 3968  # caption text rows (128 x 31)
ZS = 4224  # cross-att vision rows (128 x 33)
# (name, M, N, K, a_mn, b_mn)
BIG = [("big8k", 8192, 8192, 8192, 0, 0)]
LM = [
    ("c_attn", T, 2304, 768, 0, 0), ("attn.c_proj", T, 768, 768, 0, 0),
    ("c_fc", T, 3072, 768, 0, 0), ("mlp.c_proj", T, 768, 3072, 0, 0),
    ("lm_head", T, 50304, 768, 0, 0),
    ("c_attn.dX", T, 768, 2304, 0, 1), ("attn.c_proj.dX", T, 768, 768, 0, 1),
    ("c_fc.dX", T, 768, 3072, 0, 1), ("mlp.c_proj.dX", T, 3072, 768, 0, 1),
    ("lm_head.dX", T, 768, 50304, 0, 1),
    ("c_attn.dW", 2304, 768, T, 1, 1), ("attn.c_proj.dW", 768, 768, T, 1, 1),
    ("c_fc.dW", 3072, 768, T, 1, 1), ("mlp.c_proj.dW", 768, 3072, T, 1, 1),
    ("lm_head.dW", 50304, 768, T, 1, 1),
]
QF = [
    ("q.c_attn", Q, 2304, 768, 0, 0), ("q.c_proj", Q, 768, 768, 0, 0),
    ("q.c_fc", Q, 3072, 768, 0, 0), ("q.mlp.c_proj", Q, 768, 3072, 0, 0),
    ("q.lm_head", Q, 50304, 768, 0, 0),
    ("q.lm_head.dX", QT, 768, 50304, 0, 1),
    ("q.c_attn.dX", Q, 768, 2304, 0, 1), ("q.c_fc.dX", Q, 768, 3072, 0, 1),
    ("q.mlp.c_proj.dX", Q, 3072, 768, 0, 1), ("q.c_proj.dX", Q, 768, 768, 0, 1),
]

XA = [  # cross-att caption step: text-only decoder rows (QT) + 33 projected CLIP tokens (ZS)
    ("x.q_proj", QT, 768, 768, 0, 0), ("x.kv_proj", ZS, 1536, 768, 0, 0),
    ("x.c_attn", QT, 2304, 768, 0, 0), ("x.c_fc", QT, 3072, 768, 0, 0),
    ("x.mlp.c_proj", QT, 768, 3072, 0, 0),
    ("x.q_proj.dX", QT, 768, 768, 0, 1), ("x.kv_proj.dX", ZS, 768, 1536, 0, 1),
    ("x.c_attn.dX", QT, 768, 2304, 0, 1), ("x.c_fc.dX", QT, 768, 3072, 0, 1),
    ("x.mlp.c_proj.dX", QT, 3072, 768, 0, 1),
    ("x.q_proj.dW", 768, 768, QT, 1, 1), ("x.kv_proj.dW", 1536, 768, ZS, 1, 1),
    ("x.kv_all", ZS, 18432, 768, 0, 0), ("x.kv_all.dX", ZS, 768, 18432, 0, 1),  # CrossKVFn
]


def epilogues():
    """Fused-epilogue cost at the LM step's shapes: each line times the plain GEMM and the
    same GEMM with the epilogue the model uses (default kernel pick)."""
    g = torch.Generator(device="cuda").manual_seed(0)
    ev = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731
    cases = [("c_fc+bias+gelu", T, 3072, 768, 0, "act"), ("mlp.c_proj.dX*dgelu", T, 3072, 768, 1, "dact"),
             ("c_attn+bias", T, 2304, 768, 0, "bias"), ("mlp.c_proj+bias+res", T, 768, 3072, 0, "bias_res"),
             ("c_fc.dW+=", 3072, 768, T, 2, "res"), ("q.c_fc+bias+gelu_erf", Q, 3072, 768, 0, "act_erf")]
    for name, M, N, Kd, kind, epi in cases:
        A = (torch.randn(Kd, M, device="cuda", generator=g) if kind == 2 else
             torch.randn(M, Kd, device="cuda", generator=g)).bfloat16()
        B = (torch.randn(Kd, N, device="cuda", generator=g) if kind else
             torch.randn(N, Kd, device="cuda", generator=g)).bfloat16()
        C = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
        aux = torch.randn(M, N, device="cuda", generator=g).bfloat16()
        bias = torch.randn(N, device="cuda", generator=g).bfloat16()
        kw = {"act": dict(bias=bias, act=1, pre_out=aux), "act_erf": dict(bias=bias, act=2, pre_out=aux),
              "dact": dict(dact=1, pre_in=aux), "bias": dict(bias=bias),
              "bias_res": dict(bias=bias, residual=aux), "res": dict(residual=C)}[epi]
        row = [f"{name:22s}"]
        for label, extra in (("plain", {}), (epi, kw)):
            fn = lambda: K.gemm(A, B, a_mn=kind == 2, b_mn=kind >= 1, out=C, **extra)  # noqa: E731
            for _ in range(3):
                fn()
            e0, e1 = ev(), ev()
            e0.record()
            for _ in range(20):
                fn()
            e1.record()
            torch.cuda.synchronize()
            row.append(f"{label}:{e0.elapsed_time(e1) / 20 * 1e3:8.1f}us")
        print(" ".join(row), flush=True)


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "all"
    if which == "epi":
        _lib.load()
        return epilogues()
    cfgs = sys.argv[2].split(",") if len(sys.argv) > 2 else ["2:-1"]
    shapes = ((BIG if which in ("big", "all") else []) + (LM if which in ("lm", "all") else [])
              + (QF if which in ("qf", "all") else []) + (XA if which in ("xa", "all") else []))
    L = _lib.load()
    g = torch.Generator(device="cuda").manual_seed(0)
    ev = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731
    tot = {}
    for name, M, N, Kd, am, bm in shapes:
        A = (torch.randn(Kd, M, device="cuda", generator=g) if am else
             torch.randn(M, Kd, device="cuda", generator=g)).bfloat16()
        B = (torch.randn(Kd, N, device="cuda", generator=g) if bm else
             torch.randn(N, Kd, device="cuda", generator=g)).bfloat16()
        C = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
        fl = 2.0 * M * N * Kd
        row = [f"{name:16s} {M:6d}x{N:6d}x{Kd:6d} {'tn'[am]}{'tn'[bm]}"]
        ref = None
        for cfg in cfgs + ["torch"]:
            if cfg == "torch":
                at = A.t() if am else A
                bt = B if bm else B.t()
                fn = lambda: torch.mm(at, bt, out=C)  # noqa: E731
            else:
                impl, c = (int(x) for x in cfg.split(":"))
                L.gvl_gemm_tune(impl, c)
                fn = lambda: K.gemm(A, B, a_mn=bool(am), b_mn=bool(bm), out=C)  # noqa: E731
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            if ref is None:
                ref = C.float().clone()
            elif ref is not None:
                err = (C.float() - ref).abs().max().item() / (ref.abs().max().item() + 1e-9)
                if err > 2e-2:
                    row.append(f"MISMATCH({err:.3g})")
            iters = max(3, min(50, int(2e12 / fl)))
            e0, e1 = ev(), ev()
            e0.record()
            for _ in range(iters):
                fn()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / iters * 1e3
            tf = fl / us / 1e6
            tot.setdefault(cfg, 0.0)
            tot[cfg] += us
            row.append(f"{cfg}:{us:8.1f}us {tf:6.0f}TF")
        print(" ".join(row), flush=True)
        del A, B, C
    print("totals(us):", {k: round(v, 1) for k, v in tot.items()}, flush=True)
    L.gvl_gemm_tune(2, -1)


if __name__ == "__main__":
    main()
