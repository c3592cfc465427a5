"""World-size-1 RCCL run of the data-parallel LM step with the gradient buckets forced on
(GradBuckets(force=True)), for a rocprofv3 kernel trace that shows the bucket all-reduces
overlapping the backward GEMMs: eager (block-group flushes) and the captured step (segment
graphs, buckets issued between replays).  Run under rocprofv3 --kernel-trace, then
tools/dp_overlap_report.py on the trace.
The Q-Former caption step (CFG5: B = 128, frozen decoder, bridge gradients) likewise:
qf_eager / qf_graph; GVL_BUCKET_MB sets the bucket size (default 32, the bench's).
python tools/dp_overlap_trace.py [eager|graph|qf_eager|qf_graph]"""
import os
import socket
import sys

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gpt2-vision-language_amd")]

mode = sys.argv[1] if len(sys.argv) > 1 else "eager"
with socket.socket() as s:
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                        device_id=dev)
import gvl.gpt2 as g2  # noqa: E402
from gvl import _lib  # noqa: E402
from gvl.dist import GradBuckets  # noqa: E402
from gvl.train import lm_batch, train_step  # noqa: E402
_lib.load()
bucket_mb = float(os.environ.get("GVL_BUCKET_MB", "32"))
if mode.startswith("qf"):
    import bench
    from gvl.caption import pool_clip_197_to_33_avg_with_cls as pool
    from gvl.train import caption_batch, caption_labels
    m = bench.build_caption("qformer", dev)
    m.train()
    opt = bench._quiet(lambda: m.configure_optimizers(0.1, 1e-3, "cuda"))
    z, x, y, msk = caption_batch(128, device=dev)
    lab = caption_labels(y, msk)
    mbs = [(z, x, y, msk)]
    loss_fn = lambda mm, b: mm(pool(b[0]), b[1], labels=lab)[1]  # noqa: E731
else:
    torch.manual_seed(0)
    m = g2.GPT(g2.GPTConfig(vocab_size=50304)).to(dev).to(torch.bfloat16)
    opt = m.configure_optimizers(0.1, 6e-4, "cuda")
    mbs = [lm_batch(8, 1024, step=i, device=dev) for i in range(2)]
    loss_fn = lambda mm, b: mm(b[0], b[1])[1]  # noqa: E731
bk = GradBuckets(opt, bucket_mb=bucket_mb, model=m, force=True)
if mode.endswith("graph"):
    from gvl.graph import GraphedStep
    gs = GraphedStep(m, opt, mbs, loss_fn, 6e-4, warmup=1, buckets=bk, segmented=True)
    for _ in range(3):
        r = gs(6e-4)
else:
    for _ in range(3):
        r = train_step(m, opt, mbs, loss_fn, 6e-4, buckets=bk)
torch.cuda.synchronize()
print(mode, "loss", float(r.loss), "buckets", len(bk.buckets), "launch order", bk.launch_log[-len(bk.buckets):])
dist.destroy_process_group()
