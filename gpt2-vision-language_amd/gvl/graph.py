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

Data-parallel steps (buckets) stay eager: the RCCL all-reduce hooks are not captured.
"""
from __future__ import annotations

import torch

from . import kernels as K
from .train import StepResult, train_step


class GraphedStep:
    def __init__(self, model, optimizer, micro_batches, loss_fn, lr, *, max_norm: float = 1.0,
                 warmup: int = 2):
        """Runs `warmup` eager steps at `lr` on a side stream (allocator + kernel caches
        warm, the optimizer arenas built), then captures one step.  Hyper-parameters other
        than lr (betas, eps, weight_decay, max_norm) are frozen into the graph."""
        self.model, self.opt = model, optimizer
        dev = next(model.parameters()).device
        self.seed_off = K.seed_offset(dev)
        K._gemm_workspace(dev)
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            for _ in range(max(1, warmup)):
                train_step(model, optimizer, micro_batches, loss_fn, lr, max_norm=max_norm)
                self.seed_off.add_(1)
        torch.cuda.current_stream(dev).wait_stream(side)
        torch.cuda.synchronize(dev)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            res = train_step(model, optimizer, micro_batches, loss_fn, None, max_norm=max_norm)
            self.seed_off.add_(1)
        self.result = StepResult(res.loss, res.norm)

    def __call__(self, lr) -> StepResult:
        """One optimizer step at learning rate `lr` (every param group, like
        train_gpt2.py:474-475).  Returns device scalars (no host sync)."""
        for g in self.opt.param_groups:
            g["lr"] = lr
        self.opt.advance()
        self.graph.replay()
        return self.result
