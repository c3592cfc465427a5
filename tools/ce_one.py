"""Time the fused cross-entropy (gvl_cross_entropy: loss + dlogits) on the LM's micro-step
logits ([16384, 50304] bf16) and the Q-Former step's text rows; HIP events, median of 5 x 20.
python tools/ce_one.py   (GVL_LIB=... for a variant build)"""
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpt2-vision-language_amd"))
from gvl import kernels as K  # noqa: E402


def timed(fn, n=20):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


g = torch.Generator(device="cuda").manual_seed(0)
for (B, S, T, off) in [(16, 1024, 1024, 0), (128, 63, 31, 32)]:
    V = 50304
    logits = (torch.randn(B * S, V, device="cuda", generator=g) * 2).bfloat16()
    tg = torch.randint(0, 50257, (B, T), device="cuda", generator=g)
    f = lambda: K.cross_entropy(logits, tg, rows_per_group=T, group_stride=S, row_offset=off,  # noqa: E731
                                want_grad=True, vocab=V)
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    t = statistics.median(timed(f) for _ in range(5))
    rows = B * T
    gb = rows * V * 2 * 2 / 1e9
    print(f"rows={rows} V={V}: {t:8.1f} us  {gb / t * 1e3:6.2f} TB/s (logits read + dlogits written)", flush=True)
    del logits
