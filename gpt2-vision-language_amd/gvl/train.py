"""The gradient-accumulation data-parallel training step (the hot loop of
train_gpt2.py:457-482, gpt2_linear/train.py:292-322, gpt2_cross-att/train.py:273-301):

    zero_grad -> for each micro-step: forward, loss/accum, backward (bucketed all-reduce
    on the last one) -> loss all-reduce -> clip_grad_norm_(1.0) -> set lr -> AdamW

with the MI355X pieces: flat grad arena + fused norm/clip/AdamW (gvl.optim), bucketed
RCCL all-reduce overlapped with backward (gvl.dist), and no host synchronisation inside
the step (loss and norm stay on the device until the caller reads them).

Also holds the synthetic-batch makers of SURVEY.md §8(d) and the caption-label rule of
gpt2_linear/data.py:35-49 (labels = y.masked_fill(~mask, -100), train.py:305-306).
"""
from __future__ import annotations

from dataclasses import dataclass

import torch

from .dist import GradBuckets, all_reduce_mean_
from .optim import clip_grad_norm_


@dataclass
class StepResult:
    loss: torch.Tensor  # 0-dim fp32 on device (mean over micro-steps and ranks)
    norm: torch.Tensor  # 0-dim fp32 on device (pre-clip global grad norm)


def accumulate(model, optimizer, micro_batches, loss_fn, buckets: GradBuckets = None):
    """zero_grad, then forward / loss/accum / backward per micro-step (train_gpt2.py:458-469);
    with `buckets` the gradient all-reduce fires during the last micro-step's backward.
    Returns the summed micro-step losses (device scalar)."""
    accum = len(micro_batches)
    optimizer.zero_grad()
    loss_accum = None
    for i, batch in enumerate(micro_batches):
        loss = loss_fn(model, batch)
        # loss/accum without the division kernels: backward is seeded with a cached 1/accum
        # scalar (no ones-fill, no div forward/backward per micro-step) and the running mean
        # is one scaled add
        la = loss.detach().float()
        if loss_accum is None:
            loss_accum = la if accum == 1 else la * (1.0 / accum)
        else:
            loss_accum = loss_accum.add(la, alpha=1.0 / accum)
        if buckets is not None:
            buckets.set_sync(i == accum - 1)
        loss.backward(_grad_seed(loss, accum))
    if buckets is not None:
        buckets.wait()
    return loss_accum


_SEEDS = {}


def _grad_seed(loss, accum):
    """d(loss/accum)/d(loss) as a cached device scalar of loss's dtype (created once, so a
    captured step replays no fill for it)."""
    key = (loss.device, loss.dtype, accum)
    t = _SEEDS.get(key)
    if t is None:
        t = torch.full((), 1.0 / accum, dtype=loss.dtype, device=loss.device)
        _SEEDS[key] = t
    return t


def finish(optimizer, lr, max_norm: float = 1.0):
    """clip_grad_norm_ (device-side coefficient) -> lr -> AdamW (train_gpt2.py:472-476)."""
    norm = clip_grad_norm_(optimizer, max_norm)
    if lr is not None:  # None: keep the groups' lr (a captured step stages it per replay)
        for g in optimizer.param_groups:
            g["lr"] = lr
    optimizer.step()
    return norm


def train_step(model, optimizer, micro_batches, loss_fn, lr, *, buckets: GradBuckets = None,
               max_norm: float = 1.0, process_group=None) -> StepResult:
    """One optimizer step over len(micro_batches) micro-steps.

    loss_fn(model, batch) -> scalar loss tensor.  `buckets` (gvl.dist.GradBuckets) enables
    the data-parallel gradient all-reduce on the last micro-step.
    """
    loss_accum = accumulate(model, optimizer, micro_batches, loss_fn, buckets)
    all_reduce_mean_(loss_accum, process_group)
    norm = finish(optimizer, lr, max_norm)
    return StepResult(loss_accum, norm)


# ------------------------------------------------------------- synthetic inputs (§8d)
def lm_batch(B, T, vocab=50257, seed=1234, device="cuda", step=0, rank=0):
    """(x, y) = (buf[:-1], buf[1:]) over a B*T+1 token window (train_gpt2.py:177-187)."""
    g = torch.Generator(device="cpu")
    g.manual_seed(seed + 1_000_003 * rank + 7919 * step)
    buf = torch.randint(0, vocab, (B * T + 1,), generator=g, dtype=torch.long)
    x = buf[:-1].view(B, T)
    y = buf[1:].view(B, T)
    return x.to(device, non_blocking=True), y.to(device, non_blocking=True)


def caption_labels(y, mask):
    """labels = y.masked_fill(~m, -100) (gpt2_linear/train.py:305-306)."""
    return y.masked_fill(~mask, -100)


def caption_batch(B, L=257, D=768, T=31, vocab=50257, seed=1234, device="cuda", step=0, rank=0,
                  eot=50256):
    """Synthetic COCO-shape caption batch: CLIP tokens z ~ N(0,1) [B, L, D] fp32, caption
    length U{8..31}, ids padded with EOT exactly like _encode_caption
    (gpt2_linear/data.py:35-49): x = ids[:-1], y = ids[1:], mask[:max(len-1,1)] = True."""
    g = torch.Generator(device="cpu")
    g.manual_seed(seed + 1_000_003 * rank + 7919 * step)
    z = torch.randn(B, L, D, generator=g)
    n_tok = torch.randint(7, T, (B,), generator=g)  # caption tokens before EOT
    ids = torch.full((B, T + 1), eot, dtype=torch.long)
    body = torch.randint(0, eot, (B, T), generator=g)
    pos = torch.arange(T + 1)
    keep = pos.unsqueeze(0) < n_tok.unsqueeze(1)
    ids[:, :T][keep[:, :T]] = body[keep[:, :T]]
    x, y = ids[:, :-1], ids[:, 1:]
    L_ = n_tok + 1
    valid = torch.clamp(L_ - 1, min=1)
    mask = pos[:T].unsqueeze(0) < valid.unsqueeze(1)
    return (z.to(device, non_blocking=True), x.to(device, non_blocking=True),
            y.to(device, non_blocking=True), mask.to(device, non_blocking=True))
