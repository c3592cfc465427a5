"""One training step as one hipGraph (HIP graphs instead of a tracing compiler).

The caption steps launch ~450 small kernels per optimizer step from Python (autograd
Functions over ctypes); on MI355X the GPU finishes many of them faster than the host can
issue them.  `GraphedStep` captures the whole step — zero_grad, every micro-step's forward
and backward, loss reduction, grad-norm + clip coefficient, AdamW — once, and replays it
with a single launch.  What changes between steps stays correct under replay:

  * lr and the AdamW step count live on the device (`AdamW.stage_hyper`, read by
    gvl_adamw_dev) and are staged from the host before each replay;
  * dropout seeds are frozen at capture but re-keyed on the device by a step offset
    (`gvl.kernels.seed_offset`, include/gvl.h seed_eff) that the graph itself advances;
  * inputs are the captured tensors: feed new data with `copy_` into `micro_batches`
    (static buffers), as a reference loop's next_batch() would.

Data-parallel steps (world > 1, `buckets` given) are captured in two segments around the
exchange: graph A = zero_grad + every micro-step's forward/backward (the bucket hooks stay
idle), then ONE eager RCCL AVG all-reduce of the whole grad arena plus the scalar loss
all-reduce on the current stream, then graph B = grad-norm + clip + AdamW.  No collective is
captured (so replay cannot deadlock on a rank that captured differently); the exchange loses
its overlap with the last backward, which costs ~2(N-1)/N x 39 MB (Q-Former) / 249 MB (LM)
over xGMI per optimizer step — small next to the step.
"""
from __future__ import annotations

import torch

import torch.distributed as dist

from . import kernels as K
from .dist import _avg, all_reduce_mean_
from .train import StepResult, accumulate, finish, train_step


class GraphedStep:
    def __init__(self, model, optimizer, micro_batches, loss_fn, lr, *, max_norm: float = 1.0,
                 warmup: int = 2, buckets=None, process_group=None, segmented=None):
        """Runs `warmup` eager steps at `lr` on a side stream (allocator + kernel caches
        warm, the optimizer arenas built), then captures one step.  Hyper-parameters other
        than lr (betas, eps, weight_decay, max_norm) are frozen into the graph."""
        self.model, self.opt = model, optimizer
        self.pg = process_group
        world = dist.get_world_size(process_group) if dist.is_initialized() else 1
        # segmented=True forces the two-graph DP form (tests drive it at world size 1)
        self.dp = buckets is not None and (world > 1 if segmented is None else segmented)
        dev = next(model.parameters()).device
        self.seed_off = K.seed_offset(dev)
        K._gemm_workspace(dev)
        K._gemm_tickets(dev)
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            for _ in range(max(1, warmup)):
                train_step(model, optimizer, micro_batches, loss_fn, lr, max_norm=max_norm,
                           buckets=buckets if self.dp else None, process_group=process_group)
                self.seed_off.add_(1)
        torch.cuda.current_stream(dev).wait_stream(side)
        torch.cuda.synchronize(dev)
        if not self.dp:
            self.graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph):
                res = train_step(model, optimizer, micro_batches, loss_fn, None, max_norm=max_norm)
                self.seed_off.add_(1)
            self.result = StepResult(res.loss, res.norm)
            return
        buckets.set_sync(False)  # hooks idle inside the capture: no collective is recorded
        self.graph_a = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph_a):
            loss = accumulate(model, optimizer, micro_batches, loss_fn, None)
        self.graph_b = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph_b):
            norm = finish(optimizer, None, max_norm)
            self.seed_off.add_(1)
        self.result = StepResult(loss, norm)

    def __call__(self, lr) -> StepResult:
        """One optimizer step at learning rate `lr` (every param group, like
        train_gpt2.py:474-475).  Returns device scalars (no host sync)."""
        for g in self.opt.param_groups:
            g["lr"] = lr
        self.opt.advance()
        if not self.dp:
            self.graph.replay()
            return self.result
        self.graph_a.replay()
        _avg(self.opt.grad_arena, self.pg, async_op=False)
        all_reduce_mean_(self.result.loss, self.pg)
        self.graph_b.replay()
        return self.result
