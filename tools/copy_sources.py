"""Which Python lines launch the framework-side copies (aten::copy_ / clone / fill / memcpy) of one
eager caption or LM step: torch.profiler with Python stacks, grouped by the innermost gvl frame.
python tools/copy_sources.py [qformer|linear|cross|lm]"""
import collections
import os
import sys
import types

import torch

ROOT = os.path.join(os.path.dirname(__file__), "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "gpt2-vision-language_amd"))
import bench  # noqa: E402

kind = sys.argv[1] if len(sys.argv) > 1 else "qformer"
dev = torch.device("cuda")
args = types.SimpleNamespace(caption_batch=128, micro_batch=16, bucket_mb=None)
step = bench.run_lm(args, 1, 0, dev)[0] if kind == "lm" else bench.run_caption(kind, args, 1, 0, dev)[0]
for i in range(2):
    step(i)
torch.cuda.synchronize()
acts = [torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]
with torch.profiler.profile(activities=acts, with_stack=True, record_shapes=True) as prof:
    step(2)
    torch.cuda.synchronize()
WATCH = ("aten::copy_", "aten::clone", "aten::fill_", "aten::zero_", "aten::cat", "aten::contiguous",
         "aten::to", "aten::_to_copy", "aten::index", "aten::masked_fill", "aten::where")
by = collections.Counter()
for e in prof.events():
    if e.name not in WATCH or e.device_type != torch.autograd.DeviceType.CPU:
        continue
    frames = [f for f in (e.stack or []) if "gvl" in f or "bench.py" in f]
    key = (e.name, frames[0] if frames else "?", tuple(e.input_shapes[0]) if e.input_shapes else ())
    by[key] += 1
for (name, frame, shp), n in sorted(by.items(), key=lambda kv: -kv[1]):
    print(f"{n:4d}  {name:18s} {str(shp):24s} {frame}")
