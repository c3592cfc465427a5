"""Greedy caption/text decoding (the parity variant of the reference's sampling loops,
gpt2_linear/data.py:105-131 and train_gpt2.py:440-449).

Like the reference, every new token re-runs the full forward over the whole sequence (no
KV cache); the next token is argmax(logits[:, -1]) with torch's first-max tie-break.
Returns the generated ids and the per-step top-1/top-2 logit margins (used by the parity
tests to skip near-ties where bf16 rounding may legitimately flip the choice).
"""
from __future__ import annotations

import torch


@torch.no_grad()
def greedy_caption(model, z_pooled, prompt_ids, n_new):
    """model: GPT_Caption (forward(patch_tokens, ids)) ; z_pooled [B, 33, D]."""
    x = prompt_ids
    margins = []
    for _ in range(n_new):
        logits, _ = model(z_pooled, x)
        last = logits[:, -1, :].float()
        top2 = torch.topk(last, 2, dim=-1)
        margins.append((top2.values[:, 0] - top2.values[:, 1]))
        nxt = torch.argmax(last, dim=-1, keepdim=True)
        x = torch.cat([x, nxt], dim=1)
    return x[:, prompt_ids.shape[1]:], torch.stack(margins, dim=1)


@torch.no_grad()
def greedy_lm(model, prompt_ids, n_new, z=None):
    """model: GPT (forward(idx)) or cross-att GPT (forward(idx, z=z))."""
    x = prompt_ids
    margins = []
    for _ in range(n_new):
        logits, _ = model(x) if z is None else model(x, z=z)
        last = logits[:, -1, :].float()
        top2 = torch.topk(last, 2, dim=-1)
        margins.append((top2.values[:, 0] - top2.values[:, 1]))
        nxt = torch.argmax(last, dim=-1, keepdim=True)
        x = torch.cat([x, nxt], dim=1)
    return x[:, prompt_ids.shape[1]:], torch.stack(margins, dim=1)
