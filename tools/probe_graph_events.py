"""Probe: do raw hipEventRecord calls made while capturing a hipGraph time the replayed kernels?"""
import ctypes as C
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "gpt2-vision-language_amd"))
from gvl import kernels as K  # noqa: E402

hip = C.CDLL("libamdhip64.so")
BF = torch.bfloat16
a = torch.randn(8192, 1024, device="cuda").to(BF)
b = torch.randn(4096, 1024, device="cuda").to(BF)
c = torch.empty(8192, 4096, device="cuda", dtype=BF)
K.gemm(a, b, out=c)
torch.cuda.synchronize()
e = [C.c_void_p() for _ in range(2)]
for x in e:
    print("create", hip.hipEventCreateWithFlags(C.byref(x), 0))
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    print("rec0", hip.hipEventRecord(e[0], s))
    K.gemm(a, b, out=c)
    print("rec1", hip.hipEventRecord(e[1], s))
for _ in range(3):
    g.replay()
torch.cuda.synchronize()
ms = C.c_float()
print("elapsed rc", hip.hipEventElapsedTime(C.byref(ms), e[0], e[1]), ms.value)
t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
t0.record(); K.gemm(a, b, out=c); t1.record(); torch.cuda.synchronize()
print("eager ms", t0.elapsed_time(t1))
