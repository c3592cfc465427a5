"""Time gvl_embedding_bwd_det at the LM micro-batch (16 x 1024 tokens, V 50304, C 768)."""
import sys
import torch
sys.path.insert(0, "gpt2-vision-language_amd")
from gvl import kernels as K  # noqa: E402

dev = torch.device("cuda:0")
V, C, G, T = 50304, 768, 16, 1024
idx = torch.randint(0, 50257, (G, T), device=dev)
dout = torch.randn(G, T, C, device=dev).to(torch.bfloat16)
wte = torch.zeros(V, C, dtype=torch.bfloat16, device=dev)
wpe = torch.zeros(1024, C, dtype=torch.bfloat16, device=dev)
for which, a, b in (("wte+wpe", wte, wpe), ("wte", wte, None), ("wpe", None, wpe)):
    for _ in range(3):
        K.embedding_bwd_det(idx, dout, a, b, T, T, 0, C, V)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50):
        K.embedding_bwd_det(idx, dout, a, b, T, T, 0, C, V)
    e1.record()
    torch.cuda.synchronize()
    print(f"{which}: {e0.elapsed_time(e1) / 50 * 1000:.1f} us")
