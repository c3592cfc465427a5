"""LayerNorm forward / backward launch times at the bench's shapes (HIP events, median of 5 x 2 graph
replays of 50 launches): python tools/ln_one.py  (GVL_LIB selects a variant build)."""
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gpt2-vision-language_amd")]
from gvl import _lib  # noqa: E402
from gvl import kernels as K  # noqa: E402

_lib.load()
dev = torch.device("cuda:0")


def timeit(fn, reps=50, rounds=5):
    t = []
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        t.append(e0.elapsed_time(e1) * 1e3 / reps)
    return statistics.median(t)


torch.manual_seed(0)
for rows, C in [(16384, 768), (8064, 768), (4096, 768), (4224, 1024)]:
    x = torch.randn(rows, C, device=dev).to(torch.bfloat16)
    w = torch.randn(C, device=dev).to(torch.bfloat16)
    b = torch.randn(C, device=dev).to(torch.bfloat16)
    y = torch.empty_like(x)
    K.layernorm_fwd(x, w, b, out=y)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()  # 50 launches per replay: the python launch cost stays out
    with torch.cuda.graph(g):
        for _ in range(50):
            K.layernorm_fwd(x, w, b, out=y)
    tf = timeit(g.replay, reps=2) / 50
    gb = 2.0 * rows * C * 2 / 1e9
    print(f"ln_fwd rows={rows:6d} C={C:5d}: {tf:7.2f} us  {gb / tf * 1e6 / 1e3:6.2f} TB/s", flush=True)
    _, mean, rstd = K.layernorm_fwd(x, w, b, out=y)
    dy = torch.randn(rows, C, device=dev).to(torch.bfloat16)
    res = torch.randn(rows, C, device=dev).to(torch.bfloat16)
    dx = torch.empty_like(x)
    dw = torch.zeros(C, device=dev, dtype=torch.bfloat16)
    db = torch.zeros(C, device=dev, dtype=torch.bfloat16)
    torch.cuda.synchronize()
    g2 = torch.cuda.CUDAGraph()  # the LM's form: dx = residual grad + LN', dw / db accumulated
    with torch.cuda.graph(g2):
        for _ in range(50):
            K.layernorm_bwd(dy, x, w, mean, rstd, dx=dx, dw=dw, db=db, accumulate_wb=True, residual=res)
    tb = timeit(g2.replay, reps=2) / 50
    gb = 4.0 * rows * C * 2 / 1e9
    print(f"ln_bwd rows={rows:6d} C={C:5d}: {tb:7.2f} us  {gb / tb * 1e6 / 1e3:6.2f} TB/s (+ finalize)", flush=True)
