"""Do two half-batch kernel chains on two streams overlap on MI355X (eager and inside one
captured hipGraph)?  Bound for the Q-Former two-branch lever.

Chain per branch (rows = 4032, half of the Q-Former decoder's 8064): the frozen decoder
block's N = 768 products (direct-A kernel: 126 tiles, half the CUs) interleaved with
LayerNorm forwards / backwards — the non-GEMM work the lever hopes to hide.
Prints ms for: full batch on one stream (8064 rows), both halves serial on one stream,
two streams eager, one graph serial, one graph with a fork/join over two streams.
python tools/concurrency_probe.py [iters]"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "gpt2-vision-language_amd"))
from gvl import _lib  # noqa: E402
from gvl import kernels as K  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 20
_lib.load()
dev = torch.device("cuda")
g = torch.Generator(device="cuda").manual_seed(0)
C = 768
BF = torch.bfloat16


def bufs(rows):
    r = lambda *s: (torch.randn(*s, device=dev, generator=g) * 0.1).to(BF)  # noqa: E731
    return dict(x=r(rows, C), h=r(rows, 4 * C), qkv=r(rows, 3 * C), y=torch.empty(rows, C, dtype=BF, device=dev),
                ln=torch.empty(rows, C, dtype=BF, device=dev), dx=torch.empty(rows, C, dtype=BF, device=dev))


W = dict(fc=(torch.randn(4 * C, C, device=dev, generator=g) * 0.02).to(BF),
         proj=(torch.randn(C, 4 * C, device=dev, generator=g) * 0.02).to(BF),
         attn=(torch.randn(3 * C, C, device=dev, generator=g) * 0.02).to(BF),
         lnw=torch.ones(C, dtype=BF, device=dev), lnb=torch.zeros(C, dtype=BF, device=dev))


def chain(b):
    """One decoder block's worth of N = 768 dX products and LayerNorms (backward-like)."""
    for _ in range(2):
        K.gemm(b["h"], W["fc"], b_mn=True, out=b["y"])        # c_fc.dX: [rows, 3072] x [3072, 768]
        _, mean, rstd = K.layernorm_fwd(b["x"], W["lnw"], W["lnb"], out=b["ln"])
        K.layernorm_bwd(b["y"], b["x"], W["lnw"], mean, rstd, dx=b["dx"])
        K.gemm(b["qkv"], W["attn"], b_mn=True, out=b["y"])    # c_attn.dX: K = 2304
        K.layernorm_fwd(b["x"], W["lnw"], W["lnb"], out=b["ln"])
        K.gemm(b["x"], W["attn"][:C], out=b["y"])             # attn.c_proj-like: K = 768


full, ha, hb = bufs(8064), bufs(4032), bufs(4032)
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()


def serial():
    chain(ha)
    chain(hb)


def forked():
    cur = torch.cuda.current_stream()
    s1.wait_stream(cur)
    s2.wait_stream(cur)
    with torch.cuda.stream(s1):
        chain(ha)
    with torch.cuda.stream(s2):
        chain(hb)
    cur.wait_stream(s1)
    cur.wait_stream(s2)


def timeit(fn):
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


def graphed(fn):
    fn()
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        gr.capture_begin()
        fn()
        gr.capture_end()
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    return gr.replay


res = {}
res["full_8064_one_stream"] = timeit(lambda: chain(full))
res["halves_serial_eager"] = timeit(serial)
res["halves_two_streams_eager"] = timeit(forked)
res["full_8064_graph"] = timeit(graphed(lambda: chain(full)))
res["halves_serial_graph"] = timeit(graphed(serial))
res["halves_forked_graph"] = timeit(graphed(forked))
# GEMM-only and LN-only pieces (what perfect overlap could reach)
res["gemm_only_half_x2_serial"] = timeit(lambda: [K.gemm(b["h"], W["fc"], b_mn=True, out=b["y"]) for b in (ha, hb)])


def gemm_forked():
    cur = torch.cuda.current_stream()
    s1.wait_stream(cur)
    s2.wait_stream(cur)
    for s, b in ((s1, ha), (s2, hb)):
        with torch.cuda.stream(s):
            K.gemm(b["h"], W["fc"], b_mn=True, out=b["y"])
    cur.wait_stream(s1)
    cur.wait_stream(s2)


res["gemm_only_half_x2_forked_eager"] = timeit(gemm_forked)
res["gemm_only_half_x2_forked_graph"] = timeit(graphed(gemm_forked))
res["gemm_only_full"] = timeit(lambda: K.gemm(full["h"], W["fc"], b_mn=True, out=full["y"]))
for k, v in res.items():
    print(f"{k:34s} {v * 1e3:9.1f} us")
