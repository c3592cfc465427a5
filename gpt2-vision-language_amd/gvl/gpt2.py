"""Drop-in GPT-2 modules for source/gpt2/train_gpt2.py:21-144 (CausalSelfAttention, MLP,
Block, GPTConfig, GPT) on the MI355X kernel path.

The module tree, parameter names, buffers and init recipe are those of the reference, so
state_dicts load both ways and `torch.manual_seed(s); GPT(cfg)` draws the same initial
weights.  nn.Linear / nn.LayerNorm / nn.Embedding serve only as parameter holders: every
forward goes through the fused HIP units of gvl.functional (no ATen compute, no CPU path).
"""
from __future__ import annotations

import inspect
from dataclasses import dataclass

import torch
import torch.nn as nn

from . import functional as Fn
from .functional import bf


@dataclass
class GPTConfig:
    """train_gpt2.py:76-83 (the train script overrides vocab_size to 50304)."""
    block_size: int = 1024
    vocab_size: int = 50257
    n_layer: int = 12
    n_head: int = 12
    n_embd: int = 768


class CausalSelfAttention(nn.Module):
    """train_gpt2.py:21-43: c_attn (C->3C), causal SDPA over 64-wide heads, c_proj."""

    def __init__(self, config, register_mask: bool = True):
        super().__init__()
        if config.n_embd % config.n_head != 0 or config.n_embd // config.n_head != 64:
            raise ValueError("gvl kernels implement head_dim == 64 (n_embd / n_head)")
        self.c_attn = nn.Linear(config.n_embd, 3 * config.n_embd)
        self.c_proj = nn.Linear(config.n_embd, config.n_embd)
        self.c_proj.NANOGPT_SCALE_INIT = 1
        self.n_head = config.n_head
        self.n_embd = config.n_embd
        if register_mask:
            # unused by the computation; kept because checkpoints carry it (train_gpt2.py:31)
            bs = config.block_size
            self.register_buffer("bias", torch.tril(torch.ones(bs, bs)).view(1, 1, bs, bs))

    def forward(self, x):
        """Stand-alone attention sub-layer (the Block path fuses it with its neighbours)."""
        B, T, C = x.shape
        qkv = Fn.LinearFn.apply(x, bf(self.c_attn.weight), bf(self.c_attn.bias))
        y = _SelfAttnFn.apply(qkv, self.n_head)
        return Fn.LinearFn.apply(y, bf(self.c_proj.weight), bf(self.c_proj.bias))


class _SelfAttnFn(torch.autograd.Function):
    """Causal attention over a packed [B, T, 3C] qkv tensor (used by the stand-alone
    CausalSelfAttention.forward; blocks use GPTBlockFn)."""

    @staticmethod
    def forward(ctx, qkv, n_head: int):
        from . import kernels as K
        B, T, C3 = qkv.shape
        C = C3 // 3
        q = qkv.contiguous()
        y, lse = K.attn_fwd(q[:, :, :C], q[:, :, C:2 * C], q[:, :, 2 * C:], n_head, True)
        ctx.save_for_backward(q, y, lse)
        ctx.n_head = n_head
        return y

    @staticmethod
    def backward(ctx, dy):
        from . import kernels as K
        q, y, lse = ctx.saved_tensors
        B, T, C3 = q.shape
        C = C3 // 3
        dq = torch.empty_like(q)
        K.attn_bwd(dy.to(torch.bfloat16).contiguous(), q[:, :, :C], q[:, :, C:2 * C], q[:, :, 2 * C:],
                   y, lse, ctx.n_head, True, dq[:, :, :C], dq[:, :, C:2 * C], dq[:, :, 2 * C:])
        return dq, None


class MLP(nn.Module):
    """train_gpt2.py:46-59: c_fc (C->4C), GELU(tanh), c_proj (4C->C)."""

    def __init__(self, config):
        super().__init__()
        self.c_fc = nn.Linear(config.n_embd, 4 * config.n_embd)
        self.gelu = nn.GELU(approximate="tanh")
        self.c_proj = nn.Linear(4 * config.n_embd, config.n_embd)
        self.c_proj.NANOGPT_SCALE_INIT = 1

    def forward(self, x):
        return Fn.MLPFn.apply(x, bf(self.c_fc.weight), bf(self.c_fc.bias), bf(self.c_proj.weight),
                              bf(self.c_proj.bias), None, 1, 0.0, 0)


class Block(nn.Module):
    """train_gpt2.py:62-74, executed as one fused GPTBlockFn."""

    def __init__(self, config, register_mask: bool = True):
        super().__init__()
        self.ln_1 = nn.LayerNorm(config.n_embd)
        self.attn = CausalSelfAttention(config, register_mask=register_mask)
        self.ln_2 = nn.LayerNorm(config.n_embd)
        self.mlp = MLP(config)

    def block_params(self):
        a, m = self.attn, self.mlp
        return (bf(self.ln_1.weight), bf(self.ln_1.bias), bf(a.c_attn.weight), bf(a.c_attn.bias),
                bf(a.c_proj.weight), bf(a.c_proj.bias), bf(self.ln_2.weight), bf(self.ln_2.bias),
                bf(m.c_fc.weight), bf(m.c_fc.bias), bf(m.c_proj.weight), bf(m.c_proj.bias))

    def forward(self, x):
        if x.dtype != torch.bfloat16:
            x = x.to(torch.bfloat16)
        return Fn.GPTBlockFn.apply(x, *self.block_params(), self.attn.n_head, True)


def init_gpt_weights(module, n_layer):
    """The nanoGPT init (train_gpt2.py:100-109): N(0, 0.02), c_proj scaled by
    (2*n_layer)^-0.5, zero biases; LayerNorm keeps (1, 0)."""
    if isinstance(module, nn.Linear):
        std = 0.02
        if hasattr(module, "NANOGPT_SCALE_INIT"):
            std *= (2 * n_layer) ** -0.5
        torch.nn.init.normal_(module.weight, mean=0.0, std=std)
        if module.bias is not None:
            torch.nn.init.zeros_(module.bias)
    elif isinstance(module, nn.Embedding):
        torch.nn.init.normal_(module.weight, mean=0.0, std=0.02)


def build_optimizer(model, weight_decay, learning_rate, device):
    """configure_optimizers (train_gpt2.py:127-144): AdamW, betas (0.9, 0.95), eps 1e-8,
    weight decay on >=2-D trainable tensors only.  On a GPU device the fused MI355X AdamW
    over flat bf16 arenas is returned (gvl.optim.AdamW); on CPU, torch.optim.AdamW."""
    params = [(n, p) for n, p in model.named_parameters() if p.requires_grad]
    decay = [p for _, p in params if p.dim() >= 2]
    nodecay = [p for _, p in params if p.dim() < 2]
    groups = [{"params": decay, "weight_decay": weight_decay},
              {"params": nodecay, "weight_decay": 0.0}]
    print(f"num decayed parameter tensors: {len(decay)}, with "
          f"{sum(p.numel() for p in decay):,} parameters")
    print(f"num non-decayed parameter tensors: {len(nodecay)}, with "
          f"{sum(p.numel() for p in nodecay):,} parameters")
    use_fused = "cuda" in str(device)
    print(f"using fused AdamW:{use_fused}")
    if use_fused:
        from .optim import AdamW
        return AdamW(groups, lr=learning_rate, betas=(0.9, 0.95), eps=1e-8)
    kw = {"fused": False} if "fused" in inspect.signature(torch.optim.AdamW).parameters else {}
    return torch.optim.AdamW(groups, lr=learning_rate, betas=(0.9, 0.95), eps=1e-8, **kw)


class GPT(nn.Module):
    """train_gpt2.py:85-125: GPT-2 with tied wte / lm_head."""

    def __init__(self, config):
        super().__init__()
        self.config = config
        self.transformer = nn.ModuleDict(dict(
            wte=nn.Embedding(config.vocab_size, config.n_embd),
            wpe=nn.Embedding(config.block_size, config.n_embd),
            h=nn.ModuleList([Block(config) for _ in range(config.n_layer)]),
            ln_f=nn.LayerNorm(config.n_embd),
        ))
        self.lm_head = nn.Linear(config.n_embd, config.vocab_size, bias=False)
        self.transformer.wte.weight = self.lm_head.weight
        # tied: its gradient is final only after both the lm_head and the embedding backward
        # (gvl.dist.GradBuckets reduces it at the end of backward)
        self.lm_head.weight._gvl_tied = True
        self.apply(lambda m: init_gpt_weights(m, self.config.n_layer))

    def forward(self, idx, targets=None):
        B, T = idx.size()
        if T > self.config.block_size:
            raise AssertionError(f"Cannot forward sequence of length {T}, block size is only "
                                 f"{self.config.block_size}")
        tr = self.transformer
        x = Fn.EmbedFn.apply(idx, bf(tr.wte.weight), bf(tr.wpe.weight), None)
        for blk in tr.h:
            x = blk(x)
        x = Fn.LayerNormFn.apply(x, bf(tr.ln_f.weight), bf(tr.ln_f.bias), 1e-5)
        if targets is None:
            logits = Fn.lm_logits(x, bf(self.lm_head.weight))
            return logits, None
        return Fn.lm_head_loss(x, bf(self.lm_head.weight), targets, 0, None, False)

    def configure_optimizers(self, weight_decay, learning_rate, device):
        return build_optimizer(self, weight_decay, learning_rate, device)
