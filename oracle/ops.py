"""Per-op CPU fp32 restatements (TEST INFRASTRUCTURE; see oracle/__init__.py).

Explicit math, no fused torch kernels: these are the checkers for the HIP kernels.

FAST_PATHS (off by default; bench.py's cpu_baseline turns it on): attention, LayerNorm,
GELU and CE call the very torch ops the reference calls (F.scaled_dot_product_attention,
F.layer_norm, F.gelu, F.cross_entropy) instead of the explicit math, so the timed CPU
baseline runs at the reference CPU path's speed.  Same results to fp32 rounding (tested).
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as TF

F32 = torch.float32
FAST_PATHS = False


def layernorm(x, w, b, eps=1e-5):
    """nn.LayerNorm (train_gpt2.py:66): biased variance over the last dim."""
    if FAST_PATHS:
        return TF.layer_norm(x.to(F32), (x.shape[-1],), w.to(F32), b.to(F32), eps)
    x = x.to(F32)
    mu = x.mean(dim=-1, keepdim=True)
    var = ((x - mu) ** 2).mean(dim=-1, keepdim=True)
    return (x - mu) / torch.sqrt(var + eps) * w.to(F32) + b.to(F32)


def gelu_tanh(x):
    """nn.GELU(approximate='tanh') (train_gpt2.py:52)."""
    if FAST_PATHS:
        return TF.gelu(x, approximate="tanh")
    return 0.5 * x * (1.0 + torch.tanh(math.sqrt(2.0 / math.pi) * (x + 0.044715 * x ** 3)))


def gelu_erf(x):
    """nn.GELU() exact (gpt2_q_former/model.py:128)."""
    if FAST_PATHS:
        return TF.gelu(x)
    return 0.5 * x * (1.0 + torch.erf(x / math.sqrt(2.0)))


def linear(x, w, b=None):
    """nn.Linear: y = x W^T + b, W stored (out, in)."""
    y = x.to(F32) @ w.to(F32).t()
    return y if b is None else y + b.to(F32)


def attention(q, k, v, causal, scale=None):
    """softmax(q k^T * scale [+ causal mask]) v for [B, H, T, 64] tensors
    (F.scaled_dot_product_attention at train_gpt2.py:40, gpt2_cross-att/model.py:55;
    is_causal uses the top-left aligned lower-triangular mask)."""
    if FAST_PATHS and scale is None:
        return TF.scaled_dot_product_attention(q.to(F32), k.to(F32), v.to(F32), is_causal=causal)
    if scale is None:
        scale = 1.0 / math.sqrt(q.shape[-1])
    s = (q.to(F32) @ k.to(F32).transpose(-1, -2)) * scale
    if causal:
        Tq, Tk = s.shape[-2], s.shape[-1]
        mask = torch.ones(Tq, Tk, dtype=torch.bool).tril()
        s = s.masked_fill(~mask, float("-inf"))
    s = s - s.amax(dim=-1, keepdim=True)
    p = torch.exp(s)
    p = p / p.sum(dim=-1, keepdim=True)
    return p @ v.to(F32)


def split_heads(x, H):
    B, T, C = x.shape
    return x.view(B, T, H, C // H).transpose(1, 2)


def merge_heads(y):
    B, H, T, D = y.shape
    return y.transpose(1, 2).reshape(B, T, H * D)


def cross_entropy(logits, targets, ignore_index=-100):
    """F.cross_entropy mean over non-ignored targets (train_gpt2.py:124)."""
    if FAST_PATHS:
        return TF.cross_entropy(logits.to(F32).reshape(-1, logits.shape[-1]), targets.reshape(-1),
                                ignore_index=ignore_index)
    lg = logits.to(F32).reshape(-1, logits.shape[-1])
    t = targets.reshape(-1)
    valid = t != ignore_index
    lse = torch.logsumexp(lg, dim=-1)
    tt = torch.where(valid, t, torch.zeros_like(t))
    nll = lse - lg.gather(1, tt.unsqueeze(1)).squeeze(1)
    nll = torch.where(valid, nll, torch.zeros_like(nll))
    return nll.sum() / valid.sum()


def masked_cross_entropy(logits, targets, mask):
    """sum(CE * mask) / clamp(sum(mask), 1) (gpt2_cross-att/model.py:176-185)."""
    lg = logits.to(F32).reshape(-1, logits.shape[-1])
    t = targets.reshape(-1)
    m = mask.reshape(-1).to(F32)
    valid = t != -100
    lse = torch.logsumexp(lg, dim=-1)
    tt = torch.where(valid, t, torch.zeros_like(t))
    nll = lse - lg.gather(1, tt.unsqueeze(1)).squeeze(1)
    nll = torch.where(valid, nll, torch.zeros_like(nll))
    return (nll * m).sum() / m.sum().clamp_min(1)


def pool_clip(tokens):
    """pool_clip_197_to_33_avg_with_cls (gpt2_linear/model.py:240-254): CLS + 4x8
    adaptive average windows [floor(i*s/o), ceil((i+1)*s/o)) + L2 normalise (eps 1e-12)."""
    t = tokens.to(F32)
    B, L, D = t.shape
    side = int(round((L - 1) ** 0.5))
    assert side * side == L - 1
    grid = t[:, 1:].view(B, side, side, D)
    outs = [t[:, 0]]
    for i in range(4):
        r0, r1 = (i * side) // 4, -(-((i + 1) * side) // 4)
        for j in range(8):
            c0, c1 = (j * side) // 8, -(-((j + 1) * side) // 8)
            outs.append(grid[:, r0:r1, c0:c1].mean(dim=(1, 2)))
    z = torch.stack(outs, dim=1)
    n = z.norm(dim=-1, keepdim=True).clamp_min(1e-12)
    return z / n


def get_lr(it, max_lr, min_lr, warmup_steps, max_steps):
    """Cosine schedule with linear warmup (train_gpt2.py:277-285)."""
    if it < warmup_steps:
        return max_lr * (it + 1) / warmup_steps
    if it > max_steps:
        return min_lr
    ratio = (it - warmup_steps) / (max_steps - warmup_steps)
    return min_lr + 0.5 * (1.0 + math.cos(math.pi * ratio)) * (max_lr - min_lr)


def clip_coef(grads, max_norm):
    """clip_grad_norm_ (train_gpt2.py:472): total L2 norm, coef = min(1, max/(norm+1e-6))."""
    tot = torch.sqrt(sum((g.to(F32) ** 2).sum() for g in grads))
    return tot, min(1.0, max_norm / (float(tot) + 1e-6))


def adamw_update(p, g, m, v, step, lr, betas=(0.9, 0.95), eps=1e-8, wd=0.0):
    """AdamW, decoupled decay (torch.optim.AdamW, train_gpt2.py:143). In-place on p, m, v."""
    b1, b2 = betas
    p.mul_(1.0 - lr * wd)
    m.mul_(b1).add_(g, alpha=1.0 - b1)
    v.mul_(b2).addcmul_(g, g, value=1.0 - b2)
    bc1 = 1.0 - b1 ** step
    bc2 = 1.0 - b2 ** step
    denom = v.sqrt() / math.sqrt(bc2) + eps
    p.addcdiv_(m, denom, value=-lr / bc1)


def encode_caption(ids, max_len, eot):
    """_encode_caption semantics (gpt2_linear/data.py:35-49) on a token list."""
    if len(ids) == 0:
        ids = [eot]
    ids = ids[: max_len - 1] + [eot]
    L = len(ids)
    if L < max_len:
        ids = ids + [eot] * (max_len - L)
    t = torch.tensor(ids, dtype=torch.long)
    x, y = t[:-1], t[1:]
    mask = torch.zeros_like(y, dtype=torch.bool)
    mask[: max(L - 1, 1)] = True
    return x, y, mask


def sampling_distribution(logits, temperature=1.0, top_k=0, top_p=1.0):
    """The filtered next-token distribution of the reference's samplers, float64 numpy:
    softmax(logits / T); top-k keeps the k largest (train_gpt2.py:444-446); top-p keeps the
    sorted prefix whose preceding cumulative probability is <= top_p (gpt2_linear/data.py:
    116-122: cutoff = cumprobs > p shifted right by one), renormalised."""
    import numpy as np
    x = np.asarray(logits, dtype=np.float64) / temperature
    pr = np.exp(x - x.max())
    pr /= pr.sum()
    if 0 < top_k < pr.size:  # ties at the k-th value: lowest index first (stable order)
        order = np.argsort(-pr, kind="stable")
        keep = np.zeros(pr.size, dtype=bool)
        keep[order[:top_k]] = True
        pr = np.where(keep, pr, 0.0)
        pr /= pr.sum()
    if top_p < 1.0:
        order = np.argsort(-pr, kind="stable")
        cum = np.cumsum(pr[order])
        cut = cum > top_p
        cut[1:] = cut[:-1].copy()
        cut[0] = False
        keep = np.zeros(pr.size, dtype=bool)
        keep[order[~cut]] = True
        pr = np.where(keep, pr, 0.0)
        pr /= pr.sum()
    return pr


def inverse_cdf_index(dist, u):
    """Token drawn by uniform u from `dist` walking token indices in order (gvl_sample's
    draw; same distribution as torch.multinomial over the reference's sorted list)."""
    import numpy as np
    cdf = np.cumsum(dist)
    i = int(np.searchsorted(cdf, u * cdf[-1], side="right"))
    kept = np.nonzero(dist > 0)[0]
    return int(min(i, kept[-1]))
