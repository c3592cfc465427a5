"""Time the frozen CLIP ViT-L/14 feature stage (BASELINE configs[3]'s pixel input) alone:
python tools/clip_prof.py [B] [iters] [mode]   mode: eager (default) | graph | native (gvl
encoder, gvl/clip.py) | native_graph"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "gpt2-vision-language_amd"))
from gvl.clip import FLOP_PER_IMAGE, CLIPFeatureStage, synthetic_pixels  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 128
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 10
mode = sys.argv[3] if len(sys.argv) > 3 else "eager"
clip = CLIPFeatureStage(native=mode.startswith("native")).cuda().to(torch.bfloat16)
px = synthetic_pixels(B)
fn = lambda: clip.features(px)  # noqa: E731
for _ in range(3):
    fn()
torch.cuda.synchronize()
if mode.endswith("graph"):
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        g.capture_begin()
        out = fn()
        g.capture_end()
    torch.cuda.current_stream().wait_stream(s)
    fn = g.replay
    fn()
    torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(iters):
    fn()
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / iters
print(f"CLIP {mode} B={B}: {dt * 1e3:.2f} ms/batch, {B / dt:.0f} images/s, "
      f"{FLOP_PER_IMAGE * B / dt / 1e12:.0f} TFLOP/s")
