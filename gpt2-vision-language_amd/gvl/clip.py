"""Pixel-input caption path (BASELINE configs[3]): frozen CLIP ViT-L/14 on
stock PyTorch-ROCm -> pooled 33 tokens -> the caption bridges.

The reference never runs CLIP: its features are precomputed offline into (B, 257, 768)
token tensors (gpt2_linear/data.py:25-28, 56-62) and pooled at gpt2_linear/train.py:307.
Here the tower is instantiated from a local config (24 layers, width 1024, 16 heads, patch 14,
224 px, quick-GELU, 768-d projection — weights are not available offline, so they are
deterministic random) and run in bf16 with torch's SDPA.  Its per-token features are
visual_projection(post_layernorm(hidden)) (B, 257, 768).

Fused pool (the MI355X part): pool_clip_197_to_33_avg_with_cls averages windows of tokens and
L2-normalises (gpt2_linear/model.py:240-254).  The average is linear and the projection is a
bias-free linear map, so pool(LN(h) @ P^T) == pool(LN(h)) @ P^T: the gvl pool kernel runs on
the layer-normed 1024-d hidden states (no normalisation), the gvl GEMM projects only 33 of
257 tokens (7.8x less projection work and no (B, 257, 768) intermediate), and
gvl_l2_normalize_rows finishes.  `features(..., fused=False)` is the unfused composition.
"""
from __future__ import annotations

import torch

from . import kernels as K

BF16 = torch.bfloat16

VIT_L14 = dict(hidden_size=1024, intermediate_size=4096, num_hidden_layers=24,
               num_attention_heads=16, image_size=224, patch_size=14, projection_dim=768,
               hidden_act="quick_gelu", layer_norm_eps=1e-5)
CLIP_MEAN = (0.48145466, 0.4578275, 0.40821073)
CLIP_STD = (0.26862954, 0.26130258, 0.27577711)
FLOP_PER_IMAGE = 162e9  # ViT-L/14 forward at 224 px


class CLIPFeatureStage(torch.nn.Module):
    """Frozen ViT-L/14 vision tower + projection producing the caption models' inputs."""

    def __init__(self, seed: int = 0, **over):
        super().__init__()
        from transformers import CLIPVisionConfig, CLIPVisionModelWithProjection
        cfg = CLIPVisionConfig(**dict(VIT_L14, **over))
        cfg._attn_implementation = "sdpa"
        g = torch.random.fork_rng()
        with g:
            torch.manual_seed(seed)
            self.tower = CLIPVisionModelWithProjection(cfg)
        self.tower.requires_grad_(False)
        self.tower.eval()
        self.register_buffer("mean", torch.tensor(CLIP_MEAN).view(1, 3, 1, 1), persistent=False)
        self.register_buffer("std", torch.tensor(CLIP_STD).view(1, 3, 1, 1), persistent=False)

    @torch.no_grad()
    def hidden(self, pixels):
        """Normalised pixels in [0, 1] (B, 3, 224, 224) -> layer-normed hidden (B, 257, 1024)."""
        vm = self.tower.vision_model
        x = ((pixels - self.mean) / self.std).to(next(self.tower.parameters()).dtype)
        h = vm(pixel_values=x).last_hidden_state
        return vm.post_layernorm(h)

    @torch.no_grad()
    def tokens(self, pixels):
        """(B, 257, 768) per-token projected features (the reference's stored CLIP tokens)."""
        return self.tower.visual_projection(self.hidden(pixels))

    @torch.no_grad()
    def features(self, pixels, fused: bool = True):
        """Pooled, normalised (B, 33, 768) caption inputs."""
        if not fused:
            return K.pool_clip(self.tokens(pixels).contiguous())
        h = self.hidden(pixels).to(BF16).contiguous()
        B = h.shape[0]
        pooled = K.pool_clip(h, normalize=False)  # (B, 33, 1024)
        w = self.tower.visual_projection.weight.to(BF16)
        proj = K.linear(pooled.view(B * 33, -1), w)  # (B*33, 768)
        return K.l2_normalize_rows(proj).view(B, 33, -1)


def synthetic_pixels(B, seed=1234, device="cuda"):
    """U[0, 1) pixels (SURVEY §8(d) pixel variant)."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    return torch.rand(B, 3, 224, 224, generator=g).to(device)
