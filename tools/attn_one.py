"""Time the attention kernels on the hot-path shapes.  python tools/attn_one.py [iters]
Prints fwd / bwd ms and TF/s (causal flops counted as half)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "gpt2-vision-language_amd"))
from gvl import kernels as K  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 10


def timeit(fn):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


for (B, H, Tq, Tk, causal, drop) in [(16, 12, 1024, 1024, True, 0.0), (128, 12, 63, 63, True, 0.0),
                                     (128, 12, 31, 31, True, 0.0),
                                     (128, 12, 32, 32, False, 0.1), (128, 12, 32, 257, False, 0.1),
                                     (128, 12, 31, 33, False, 0.0), (128, 12, 32, 33, False, 0.1)]:
    g = torch.Generator(device="cuda").manual_seed(0)
    qkv = torch.randn(B, Tq, 3 * H * 64, device="cuda", generator=g).bfloat16()
    kv = torch.randn(B, Tk, 2 * H * 64, device="cuda", generator=g).bfloat16()
    q = qkv[:, :, :H * 64]
    if Tq == Tk and causal:
        k, v = qkv[:, :, H * 64:2 * H * 64], qkv[:, :, 2 * H * 64:]
    else:
        k, v = kv[:, :, :H * 64], kv[:, :, H * 64:]
    o, lse = K.attn_fwd(q, k, v, H, causal, drop_p=drop, seed=1)
    do = torch.randn_like(o)
    dq = torch.empty_like(q)
    dk = torch.empty_like(k)
    dv = torch.empty_like(v)
    f = lambda: K.attn_fwd(q, k, v, H, causal, drop_p=drop, seed=1, out=o)  # noqa: E731
    bw = lambda: K.attn_bwd(do, q, k, v, o, lse, H, causal, dq, dk, dv, drop_p=drop, seed=1)  # noqa: E731
    tf = timeit(f)
    tb = timeit(bw)
    fl = 4.0 * B * H * Tq * Tk * 64 * (0.5 if causal else 1.0)
    print(f"B={B} H={H} Tq={Tq} Tk={Tk} causal={causal} drop={drop}: fwd {tf:.3f} ms "
          f"{fl / tf / 1e9:.0f} TF/s | bwd {tb:.3f} ms {2.5 * fl / tb / 1e9:.0f} TF/s", flush=True)
