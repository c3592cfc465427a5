"""Stress the attention backward on the dropout case that failed once in a full GPU suite
(B=2 H=2 Tq=40 Tk=130, p=0.1): N repeats with the caching allocator's memory pre-filled with
NaN garbage between repeats; prints the worst dq/dk/dv relative errors vs the fp32 reference."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpt2-vision-language_amd"))
sys.path.insert(0, ROOT)
from gvl import kernels as K  # noqa: E402
from oracle import ops as O  # noqa: E402
from tests.helpers import rel_err  # noqa: E402
from tests.test_gpu_kernels import keep_mask  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 30
BF = torch.bfloat16
dev = "cuda"
B, H, Tq, Tk, p, seed = 2, 2, 40, 130, 0.1, 4242
C = H * 64
worst = {"o": 0, "dq": 0, "dk": 0, "dv": 0}
for it in range(N):
    junk = torch.full((64 << 20,), float("nan"), device=dev)  # 256 MB of NaN, then freed
    del junk
    torch.manual_seed(B * 100 + Tq + Tk + it)
    q, k, v = (torch.randn(B, T, C).to(BF) for T in (Tq, Tk, Tk))
    o, lse = K.attn_fwd(q.to(dev), k.to(dev), v.to(dev), H, False, drop_p=p, seed=seed)
    qr, kr, vr = (t.float().requires_grad_(True) for t in (q, k, v))
    sq, sk, sv = (O.split_heads(t, H) for t in (qr, kr, vr))
    pr = torch.softmax((sq @ sk.transpose(-1, -2)) / 8.0, dim=-1)
    keep = torch.from_numpy(keep_mask(seed, np.arange(B * H * Tq * Tk), p).reshape(B, H, Tq, Tk))
    pr = torch.where(keep, pr / (1 - p), torch.zeros_like(pr))
    ref = O.merge_heads(pr @ sv)
    do = torch.randn(B, Tq, C).to(BF)
    ref.backward(do.float())
    dq = torch.empty(B, Tq, C, dtype=BF, device=dev)
    dk = torch.empty(B, Tk, C, dtype=BF, device=dev)
    dv = torch.empty(B, Tk, C, dtype=BF, device=dev)
    K.attn_bwd(do.to(dev), q.to(dev), k.to(dev), v.to(dev), o, lse, H, False, dq, dk, dv, drop_p=p, seed=seed)
    torch.cuda.synchronize()
    errs = {"o": rel_err(o.float().cpu().numpy(), ref.detach().numpy()),
            "dq": rel_err(dq.float().cpu().numpy(), qr.grad.numpy()),
            "dk": rel_err(dk.float().cpu().numpy(), kr.grad.numpy()),
            "dv": rel_err(dv.float().cpu().numpy(), vr.grad.numpy())}
    for kk, e in errs.items():
        worst[kk] = max(worst[kk], e)
    if max(errs["dq"], errs["dk"], errs["dv"]) > 2.5e-2:
        print("BAD iteration", it, errs, flush=True)
print("worst", worst, flush=True)
