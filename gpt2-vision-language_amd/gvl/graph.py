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

Data-parallel steps (world > 1, `buckets` given) keep the gradient exchange overlapped
with backward without capturing any collective (so a replay cannot deadlock on a rank that
captured differently): the last micro-step's backward runs in segments
(gvl.dist.BackwardSegments, cut every few GPT-2 blocks / between Q-Former layers), each
segment captured as its own graph in one shared memory pool:

    A_0 = zero_grad + micro-steps 0..n-2 + the last forward + backward of the top segment
    A_j = backward of segment j (its deferred weight gradients flush at its end)
    B   = grad-norm + clip + AdamW

Replay: A_0, then for each segment the all-reduces of the buckets the previous segment
finalised (recorded at capture time) are issued on RCCL's stream before A_j is replayed,
so they run while A_j's kernels do; the rest, the scalar loss all-reduce and B follow.

Teardown (the reference ends every train script with destroy_process_group():
train_gpt2.py:523, gpt2_linear/train.py:372, gpt2_cross-att/train.py:348): `close()`
joins the step's outstanding bucket work, drains the device, resets every captured graph
(frees the private memory pool) and drops the references to the optimizer, buckets and
process group; a weakref finalizer does the same when a step is collected unclosed.
`gvl.dist.destroy_process_group()` closes every live GraphedStep before it destroys the
communicator, so a drop-in script's teardown never depends on garbage-collection order.
"""
from __future__ import annotations

import weakref

import torch

import torch.distributed as dist

from . import kernels as K
from .dist import all_reduce_mean_
from .train import StepResult, finish, train_step


_LIVE = weakref.WeakSet()  # GraphedSteps not yet closed (gvl.dist.destroy_process_group)


def _release(graphs, dev):
    """Finalizer / close(): drain the device, then reset the captured graphs (their
    executable graphs and the private memory pool go with the last reset)."""
    try:
        if torch.cuda.is_initialized():
            torch.cuda.synchronize(dev)
    finally:
        for g in graphs:
            g.reset()
        graphs.clear()


def live_steps():
    """GraphedSteps created and not closed yet (tests / teardown)."""
    return list(_LIVE)


class GraphedStep:
    def __init__(self, model, optimizer, micro_batches, loss_fn, lr, *, max_norm: float = 1.0,
                 warmup: int = 2, buckets=None, process_group=None, segmented=None,
                 cuts=None):
        """`cuts`: modules where the DP backward is segmented (default
        gvl.dist.segment_cuts(model)).  Runs `warmup` eager steps at `lr` on a side stream (allocator + kernel caches
        warm, the optimizer arenas built), then captures one step.  Hyper-parameters other
        than lr (betas, eps, weight_decay, max_norm) are frozen into the graph."""
        self.model, self.opt = model, optimizer
        self.pg = process_group
        self.buckets = None
        self._all_graphs = []  # every captured graph, in capture order (close() resets them)
        world = dist.get_world_size(process_group) if dist.is_initialized() else 1
        # segmented=True forces the two-graph DP form (tests drive it at world size 1)
        self.dp = buckets is not None and (world > 1 if segmented is None else segmented)
        dev = next(model.parameters()).device
        self.device = dev
        self._finalizer = weakref.finalize(self, _release, self._all_graphs, dev)
        _LIVE.add(self)
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
            self._all_graphs.append(self.graph)
            with torch.cuda.graph(self.graph):
                res = train_step(model, optimizer, micro_batches, loss_fn, None, max_norm=max_norm)
                self.seed_off.add_(1)
            self.result = StepResult(res.loss, res.norm)
            return
        self._capture_dp(model, optimizer, micro_batches, loss_fn, max_norm, buckets, cuts)

    def _capture_dp(self, model, optimizer, micro_batches, loss_fn, max_norm, buckets, cuts):
        from .dist import BackwardSegments, segment_cuts
        segs = BackwardSegments(segment_cuts(model) if cuts is None else cuts)
        accum = len(micro_batches)
        self.graphs, self.logs = [], []
        side = torch.cuda.Stream()
        torch.cuda.synchronize()

        def begin():
            g = torch.cuda.CUDAGraph()
            pool = self.graphs[0].pool() if self.graphs else None
            g.capture_begin(*(() if pool is None else (pool,)))
            self.graphs.append(g)
            self._all_graphs.append(g)
            self.logs.append([])
            buckets.capture_log = self.logs[-1]

        try:
            with torch.cuda.stream(side):
                begin()
                buckets.set_sync(False)
                optimizer.zero_grad()
                loss_accum = None
                for i, batch in enumerate(micro_batches):
                    last = i == accum - 1
                    if last:
                        buckets.set_sync(True)
                        segs.arm(True)
                    loss = loss_fn(model, batch) / accum
                    la = loss.detach().float()
                    loss_accum = la if loss_accum is None else loss_accum + la
                    if last:
                        segs.backward(loss, between=lambda j: (self.graphs[-1].capture_end(),
                                                               begin()))
                    else:
                        loss.backward()
                buckets.wait()  # (capture mode: only records the buckets still pending)
                self.graphs[-1].capture_end()
                buckets.capture_log = None
                self.graph_b = torch.cuda.CUDAGraph()
                self._all_graphs.append(self.graph_b)
                self.graph_b.capture_begin(self.graphs[0].pool())
                norm = finish(optimizer, None, max_norm)
                self.seed_off.add_(1)
                self.graph_b.capture_end()
        finally:
            buckets.capture_log = None
            segs.remove()
        torch.cuda.current_stream().wait_stream(side)
        self.buckets = buckets
        self.result = StepResult(loss_accum, norm)

    @property
    def closed(self) -> bool:
        return not self._finalizer.alive

    def close(self):
        """Release the captured step before its process group goes (idempotent).

        Order: join the bucket all-reduces the last replay issued (the current stream waits
        for RCCL's stream), drain the device, reset every graph (executable graphs and the
        shared private pool), then drop the references to the buckets and process group.
        After close() the step cannot be replayed."""
        if self.closed:
            return
        _LIVE.discard(self)
        try:
            if self.buckets is not None:
                self.buckets.join()
        finally:
            self._finalizer()  # _release: synchronize + reset every graph
            self.graphs = self.logs = []
            self.graph = self.graph_b = None
            self.buckets = self.pg = None
            self.result = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
        return False

    def __call__(self, lr) -> StepResult:
        """One optimizer step at learning rate `lr` (every param group, like
        train_gpt2.py:474-475).  Returns device scalars (no host sync)."""
        if self.closed:
            raise RuntimeError("GraphedStep.__call__ after close()")
        for g in self.opt.param_groups:
            g["lr"] = lr
        self.opt.advance()
        if not self.dp:
            self.graph.replay()
            return self.result
        bk = self.buckets
        self.graphs[0].replay()
        for log, g in zip(self.logs[:-1], self.graphs[1:]):
            bk.launch_logged(log)  # overlaps the next segment's replay
            g.replay()
        bk.launch_logged(self.logs[-1])
        bk.join()
        all_reduce_mean_(self.result.loss, self.pg)
        self.graph_b.replay()
        return self.result
