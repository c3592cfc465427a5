"""Drop-in caption models: frozen GPT-2 + trainable vision bridge.

Covers source/gpt2_linear/model.py (Linear_Bridge) and source/gpt2_q_former/model.py
(BLIP2Bridge / QFormerLayer): GPTConfig, CausalSelfAttention, MLP, Block, GPT_previous,
the bridges, GPT_Caption and pool_clip_197_to_33_avg_with_cls.  Module names, parameter
names (including the `wte`/`wpe` alias entries of GPT_Caption's state_dict) and the init
recipe follow the reference; compute runs on the fused HIP units of gvl.functional.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import functional as Fn
from .functional import bf, new_seed
from .gpt2 import MLP, GPTConfig, build_optimizer, init_gpt_weights
from .gpt2 import Block as _Block
from .gpt2 import CausalSelfAttention as _CSA

__all__ = ["GPTConfig", "CausalSelfAttention", "MLP", "Block", "GPT_previous", "Linear_Bridge",
           "QFormerLayer", "BLIP2Bridge", "GPT_Caption", "LinearCaption", "QFormerCaption",
           "pool_clip_197_to_33_avg_with_cls"]


class CausalSelfAttention(_CSA):
    """gpt2_linear/model.py:7-27 — same as the pretrain attention minus the mask buffer."""

    def __init__(self, config):
        super().__init__(config, register_mask=False)


class Block(_Block):
    """gpt2_linear/model.py:43-54."""

    def __init__(self, config):
        super().__init__(config, register_mask=False)


class GPT_previous(nn.Module):
    """gpt2_linear/model.py:67-111: the pretrained decoder, loaded then frozen."""

    def __init__(self, config: GPTConfig):
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
        self.apply(self._init_weights)

    def _init_weights(self, module):
        init_gpt_weights(module, self.config.n_layer)

    def decode(self, x):
        """blocks -> ln_f on a [B, S, C] embedding sequence."""
        for blk in self.transformer.h:
            x = blk(x)
        tr = self.transformer
        return Fn.LayerNormFn.apply(x, bf(tr.ln_f.weight), bf(tr.ln_f.bias), 1e-5)

    def forward(self, idx, targets=None):
        B, T = idx.size()
        assert T <= self.config.block_size
        tr = self.transformer
        x = Fn.EmbedFn.apply(idx, bf(tr.wte.weight), bf(tr.wpe.weight), None)
        x = self.decode(x)
        if targets is None:
            return Fn.lm_logits(x, bf(self.lm_head.weight)), None
        return Fn.lm_head_loss(x, bf(self.lm_head.weight), targets, 0, None, False)


class Linear_Bridge(nn.Module):
    """gpt2_linear/model.py:114-129: one nn.Linear(enc_dim, d_lm) over every CLIP token."""

    def __init__(self, enc_dim, d_lm, n_heads=None, n_queries=None, n_layers=None, drop=0.1):
        super().__init__()
        self.vis_proj = nn.Linear(enc_dim, d_lm)

    def forward(self, patch_tokens):
        return Fn.LinearFn.apply(patch_tokens, bf(self.vis_proj.weight), bf(self.vis_proj.bias))


class QFormerLayer(nn.Module):
    """gpt2_q_former/model.py:114-145: pre-LN self-attention, cross-attention to the
    projected CLIP tokens, exact-GELU MLP; dropout on attention probabilities and on the
    three residual branches while training."""

    def __init__(self, d, n_heads, drop=0.1):
        super().__init__()
        self.ln1 = nn.LayerNorm(d)
        self.self_attn = nn.MultiheadAttention(d, n_heads, dropout=drop, batch_first=True)
        self.ln2_q = nn.LayerNorm(d)
        self.ln2_v = nn.LayerNorm(d)
        self.cross_attn = nn.MultiheadAttention(d, n_heads, dropout=drop, batch_first=True)
        self.ln3 = nn.LayerNorm(d)
        self.mlp = nn.Sequential(nn.Linear(d, 4 * d), nn.GELU(), nn.Linear(4 * d, d))
        self.drop = nn.Dropout(drop)
        if d // n_heads != 64:
            raise ValueError("gvl kernels implement head_dim == 64")

    def _mha(self, mha, q_in, kv_in, residual, self_attn):
        p_attn = mha.dropout if self.training else 0.0
        p_out = self.drop.p if self.training else 0.0
        seed = new_seed() if (p_attn > 0 or p_out > 0) else 0
        return Fn.MHAFn.apply(q_in, kv_in, bf(mha.in_proj_weight), bf(mha.in_proj_bias),
                              bf(mha.out_proj.weight), bf(mha.out_proj.bias), residual,
                              mha.num_heads, self_attn, p_attn, p_out, seed)

    def _ln(self, ln, x, tape=None):
        return Fn.LayerNormFn.apply(x, bf(ln.weight), bf(ln.bias), ln.eps, tape)

    def forward(self, q, v):
        # q -> q + f(LN(q)) three times: each unit takes q detached as its residual and a
        # Fn.ResTape carries the output gradient to the LayerNorm backward of the same q, so
        # q's two gradients are summed inside that launch (no autograd add kernels)
        t = Fn.ResTape()
        q2 = self._ln(self.ln1, q, t)
        q = Fn.ResTapFn.apply(self._mha(self.self_attn, q2, q2, q.detach(), True), t)
        t = Fn.ResTape()
        q = Fn.ResTapFn.apply(self._mha(self.cross_attn, self._ln(self.ln2_q, q, t),
                                        self._ln(self.ln2_v, v), q.detach(), False), t)
        t = Fn.ResTape()
        q2 = self._ln(self.ln3, q, t)
        p = self.drop.p if self.training else 0.0
        fc1, fc2 = self.mlp[0], self.mlp[2]
        return Fn.ResTapFn.apply(
            Fn.MLPFn.apply(q2, bf(fc1.weight), bf(fc1.bias), bf(fc2.weight), bf(fc2.bias),
                           q.detach(), 2, p, new_seed() if p > 0 else 0), t)


class BLIP2Bridge(nn.Module):
    """gpt2_q_former/model.py:147-168: vis_proj, n_queries learned query tokens, Q-Former."""

    def __init__(self, enc_dim, d_lm, n_heads, n_queries=2, n_layers=2, drop=0.1):
        super().__init__()
        self.vis_proj = nn.Linear(enc_dim, d_lm)
        self.n_queries = n_queries
        self.query_tokens = nn.Parameter(torch.randn(n_queries, d_lm))
        self.layers = nn.ModuleList([QFormerLayer(d_lm, n_heads, drop=drop) for _ in range(n_layers)])

    def forward(self, patch_tokens):
        x = Fn.LinearFn.apply(patch_tokens, bf(self.vis_proj.weight), bf(self.vis_proj.bias))
        B = x.shape[0]
        q = Fn.QueryExpandFn.apply(self.query_tokens, B)  # query_tokens.expand(B, -1, -1)
        for layer in self.layers:
            q = layer(q, x)
        return q


class GPT_Caption(nn.Module):
    """gpt2_linear/model.py:134-237 (== gpt2_q_former/model.py:172-275 with BLIP2Bridge).

    forward(patch_tokens, input_ids, labels=None): bridge(image tokens) prepended to the
    text embeddings (positions on text only), frozen decoder, loss over the text slice.
    """

    bridge_cls = Linear_Bridge

    def __init__(self, enc_dim: int, lm: nn.Module, m_vis_tokens: int = 8,
                 use_cls_only: bool = False, freeze_lm: bool = True):
        super().__init__()
        self.use_cls_only = use_cls_only
        self.gpt = lm
        cfg = self.gpt.config
        self.d = cfg.n_embd
        self.block_size = cfg.block_size
        self.bridge = self.bridge_cls(enc_dim=enc_dim, d_lm=self.d, n_heads=cfg.n_head,
                                      n_queries=m_vis_tokens, n_layers=2, drop=0.1)
        self.wte = self.gpt.transformer.wte
        self.wpe = self.gpt.transformer.wpe
        if freeze_lm:
            for p in self.gpt.parameters():
                p.requires_grad_(False)
        for p in self.bridge.parameters():
            p.requires_grad_(True)

    def _decode_transformer(self, full_embeds):
        x = self.gpt.decode(full_embeds)
        return Fn.lm_logits(x, bf(self.gpt.lm_head.weight))

    def forward(self, patch_tokens, input_ids, labels=None):
        B, T_txt = input_ids.shape
        if patch_tokens.dim() == 2:
            patch_tokens = patch_tokens.unsqueeze(1)
        assert patch_tokens.shape[0] == B, "batch size image != batch size texte"
        x_img = patch_tokens[:, 0:1, :] if self.use_cls_only else patch_tokens
        img = self.bridge(x_img)
        M = img.size(1)
        if M + T_txt > self.block_size:
            cut = self.block_size - M
            input_ids = input_ids[:, :cut]
            if labels is not None:
                labels = labels[:, :cut]
            T_txt = cut
        full = Fn.EmbedFn.apply(input_ids, bf(self.wte.weight), bf(self.wpe.weight), img)
        x = self.gpt.decode(full)
        w = bf(self.gpt.lm_head.weight)
        if labels is None:
            return Fn.lm_logits(x, w), None
        return Fn.lm_head_loss(x, w, labels, M, None, False)

    def configure_optimizers(self, weight_decay, learning_rate, device):
        return build_optimizer(self, weight_decay, learning_rate, device)


class LinearCaption(GPT_Caption):
    bridge_cls = Linear_Bridge


class QFormerCaption(GPT_Caption):
    bridge_cls = BLIP2Bridge


def pool_clip_197_to_33_avg_with_cls(tokens_197: torch.Tensor) -> torch.Tensor:
    """gpt2_linear/model.py:240-254 on the GPU: [B, 1+s*s, D] -> [B, 33, D] (CLS + 4x8
    adaptive average pool + L2 normalise), one fused HBM pass."""
    return Fn.pool_clip(tokens_197)
