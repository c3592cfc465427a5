"""Drop-in for source/gpt2_cross-att/model.py: GPT-2 whose blocks insert a tanh-gated
cross-attention over projected CLIP tokens before the (frozen) self-attention.

Only vis_proj, every xattn and every cross_gate train (model.py:131-139); ln_x stays
frozen at (1, 0).  Compute: CrossAttnFn + GPTBlockFn per block on the HIP path.
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import torch
import torch.nn as nn

from . import functional as Fn
from .functional import bf
from .gpt2 import MLP, build_optimizer, init_gpt_weights
from .gpt2 import CausalSelfAttention as CausalSelfAttention  # with the mask buffer (:19)
from .caption import pool_clip_197_to_33_avg_with_cls

# kv_proj of all blocks as one GEMM over the shared z_proj (Fn.CrossKVFn); GVL_XKV_BATCH=0 runs
# each block's own kv_proj inside Fn.CrossAttnFn (A/B).
XKV_BATCH = os.environ.get("GVL_XKV_BATCH", "1") != "0"

__all__ = ["GPTConfig", "CausalSelfAttention", "CrossAttention", "MLP", "Vision_projector",
           "Block", "GPT", "pool_clip_197_to_33_avg_with_cls"]


@dataclass
class GPTConfig:
    """gpt2_cross-att/model.py:106-114."""
    block_size: int = 1024
    vocab_size: int = 50257
    n_layer: int = 12
    n_head: int = 12
    n_embd: int = 768
    img_embd: int = 768


class CrossAttention(nn.Module):
    """model.py:34-58: q_proj over text, kv_proj over vision tokens, non-causal SDPA, c_proj."""

    def __init__(self, config):
        super().__init__()
        assert config.n_embd % config.n_head == 0
        self.q_proj = nn.Linear(config.n_embd, config.n_embd)
        self.kv_proj = nn.Linear(config.n_embd, 2 * config.n_embd)
        self.c_proj = nn.Linear(config.n_embd, config.n_embd)
        self.c_proj.NANOGPT_SCALE_INIT = 1
        self.n_head = config.n_head
        self.n_embd = config.n_embd

    def forward(self, x, z):
        """Stand-alone cross-attention (model.py:46-58): c_proj(SDPA(q_proj(x), kv_proj(z))),
        non-causal, no gate (Block applies tanh(cross_gate) and the residual; the Block path
        fuses all of it into CrossAttnFn / CrossAttnKVFn)."""
        q = Fn.LinearFn.apply(x, bf(self.q_proj.weight), bf(self.q_proj.bias))
        kv = Fn.LinearFn.apply(z, bf(self.kv_proj.weight), bf(self.kv_proj.bias))
        y = _CrossSDPAFn.apply(q, kv, self.n_head)
        return Fn.LinearFn.apply(y, bf(self.c_proj.weight), bf(self.c_proj.bias))


class _CrossSDPAFn(torch.autograd.Function):
    """Non-causal attention of q [B, T, C] over a packed kv [B, S, 2C] (K = kv[..., :C],
    V = kv[..., C:], strided views: no split/transpose copies)."""

    @staticmethod
    def forward(ctx, q, kv, n_head: int):
        from . import kernels as K
        C = q.shape[2]
        q = q.to(torch.bfloat16).contiguous()
        kv = kv.to(torch.bfloat16).contiguous()
        y, lse = K.attn_fwd(q, kv[:, :, :C], kv[:, :, C:], n_head, False)
        ctx.save_for_backward(q, kv, y, lse)
        ctx.n_head = n_head
        return y

    @staticmethod
    def backward(ctx, dy):
        from . import kernels as K
        q, kv, y, lse = ctx.saved_tensors
        C = q.shape[2]
        dq = torch.empty_like(q)
        dkv = torch.empty_like(kv)
        K.attn_bwd(dy.to(torch.bfloat16).contiguous(), q, kv[:, :, :C], kv[:, :, C:], y, lse,
                   ctx.n_head, False, dq, dkv[:, :, :C], dkv[:, :, C:])
        return dq, dkv, None


class Vision_projector(nn.Module):
    """model.py:78-84."""

    def __init__(self, config):
        super().__init__()
        self.z_proj = nn.Linear(config.img_embd, config.n_embd)

    def forward(self, z):
        return Fn.LinearFn.apply(z, bf(self.z_proj.weight), bf(self.z_proj.bias))


class Block(nn.Module):
    """model.py:87-104."""

    def __init__(self, config):
        super().__init__()
        self.ln_x = nn.LayerNorm(config.n_embd)
        self.xattn = CrossAttention(config)
        self.ln_1 = nn.LayerNorm(config.n_embd)
        self.attn = CausalSelfAttention(config)
        self.ln_2 = nn.LayerNorm(config.n_embd)
        self.mlp = MLP(config)
        self.cross_gate = nn.Parameter(torch.tensor(0.0))

    def forward(self, x, z, kv=None):
        """kv = (packed kv_proj of every block, this block's index, KVGradSlab) when the GPT
        runs all kv_proj as one GEMM (Fn.CrossKVFn); None: this block's own kv_proj(z)."""
        if x.dtype != torch.bfloat16:
            x = x.to(torch.bfloat16)
        xa = self.xattn
        if kv is not None:
            x = Fn.CrossAttnKVFn.apply(x, kv[0], kv[1], kv[2], bf(self.ln_x.weight),
                                       bf(self.ln_x.bias), bf(xa.q_proj.weight),
                                       bf(xa.q_proj.bias), bf(xa.c_proj.weight),
                                       bf(xa.c_proj.bias), bf(self.cross_gate), xa.n_head)
        elif z is not None:
            x = Fn.CrossAttnFn.apply(x, z, bf(self.ln_x.weight), bf(self.ln_x.bias),
                                     bf(xa.q_proj.weight), bf(xa.q_proj.bias),
                                     bf(xa.kv_proj.weight), bf(xa.kv_proj.bias),
                                     bf(xa.c_proj.weight), bf(xa.c_proj.bias),
                                     bf(self.cross_gate), xa.n_head)
        a, m = self.attn, self.mlp
        return Fn.GPTBlockFn.apply(
            x, bf(self.ln_1.weight), bf(self.ln_1.bias), bf(a.c_attn.weight), bf(a.c_attn.bias),
            bf(a.c_proj.weight), bf(a.c_proj.bias), bf(self.ln_2.weight), bf(self.ln_2.bias),
            bf(m.c_fc.weight), bf(m.c_fc.bias), bf(m.c_proj.weight), bf(m.c_proj.bias), a.n_head,
            True)


class GPT(nn.Module):
    """model.py:116-186."""

    def __init__(self, config):
        super().__init__()
        self.config = config
        self.transformer = nn.ModuleDict(dict(
            wte=nn.Embedding(config.vocab_size, config.n_embd),
            wpe=nn.Embedding(config.block_size, config.n_embd),
            vis_proj=Vision_projector(config),
            h=nn.ModuleList([Block(config) for _ in range(config.n_layer)]),
            ln_f=nn.LayerNorm(config.n_embd),
        ))
        self.lm_head = nn.Linear(config.n_embd, config.vocab_size, bias=False)
        self.transformer.wte.weight = self.lm_head.weight
        self.apply(lambda m: init_gpt_weights(m, self.config.n_layer))
        for p in self.parameters():
            p.requires_grad = False
        for p in self.transformer["vis_proj"].parameters():
            p.requires_grad = True
        for blk in self.transformer["h"]:
            for p in blk.xattn.parameters():
                p.requires_grad = True
            blk.cross_gate.requires_grad = True
            # consecutive arena slots for the stacked kv_proj GEMM (gvl.optim, Fn._stacked)
            blk.xattn.kv_proj.weight._gvl_stack_key = "xattn.kv_proj.weight"
            blk.xattn.kv_proj.bias._gvl_stack_key = "xattn.kv_proj.bias"

    def forward(self, idx, z=None, targets=None, target_mask=None):
        B, T = idx.size()
        if T > self.config.block_size:
            raise AssertionError(f"Cannot forward sequence of length {T}, block size is only "
                                 f"{self.config.block_size}")
        tr = self.transformer
        x = Fn.EmbedFn.apply(idx, bf(tr.wte.weight), bf(tr.wpe.weight), None)
        zp = kv = None
        if z is not None:
            zp = tr.vis_proj(z).to(dtype=x.dtype)
            if XKV_BATCH and len(tr.h) > 1:
                slab = Fn.KVGradSlab(len(tr.h))
                wb = [bf(t) for blk in tr.h for t in (blk.xattn.kv_proj.weight, blk.xattn.kv_proj.bias)]
                kv = Fn.CrossKVFn.apply(zp, slab, *wb)
        for i, blk in enumerate(tr.h):
            x = blk(x, zp, None if kv is None else (kv, i, slab))
        x = Fn.LayerNormFn.apply(x, bf(tr.ln_f.weight), bf(tr.ln_f.bias), 1e-5)
        w = bf(self.lm_head.weight)
        if targets is None:
            return Fn.lm_logits(x, w), None
        if target_mask is None:
            return Fn.lm_head_loss(x, w, targets, 0, None, False)
        return Fn.lm_head_loss(x, w, targets, 0, target_mask.to(x.device), True)

    def configure_optimizers(self, weight_decay, learning_rate, device):
        return build_optimizer(self, weight_decay, learning_rate, device)
