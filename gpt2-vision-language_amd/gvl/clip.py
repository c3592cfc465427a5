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

gvl-native tower (`CLIPFeatureStage(native=True)`, round 6; the stock tower stays the default,
as the north star keeps CLIP on stock PyTorch-ROCm): the same frozen weights run through libgvl
— per encoder layer LayerNorm -> ONE packed q|k|v GEMM (+ bias) -> the flash-attention forward
(non-causal, 257 tokens, 16 heads of 64) reading q / k / v as strided views of it -> out_proj GEMM
with bias + residual in its epilogue -> LayerNorm -> fc1 GEMM with bias + quick-GELU in its
epilogue (ABI v14 act 5) -> fc2 GEMM with bias + residual.  The stock tower runs the same layer
as separate q / k / v GEMMs, SDPA and five elementwise passes over the 32896 x 4096 fc1 output
and the residual stream (quick-GELU as mul, sigmoid, mul; two residual adds):
profiles/r6/clip_stock_kernel_table_r6g.txt.  Checked against the stock tower on the same
weights (tests/test_gpu_decode.py::test_clip_native_matches_stock).
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
    """Frozen ViT-L/14 vision tower + projection producing the caption models' inputs.
    native=True runs the tower's encoder on libgvl's kernels (module docstring)."""

    def __init__(self, seed: int = 0, native: bool = False, **over):
        super().__init__()
        self.native = native
        self._packed = None
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
        if self.native:
            return self._native_hidden(vm, x)
        h = vm(pixel_values=x).last_hidden_state
        return vm.post_layernorm(h)

    def _pack(self, vm):
        """bf16 copies of the encoder weights in libgvl's layouts (q|k|v packed), built once."""
        if self._packed is None:
            bf = lambda t: t.detach().to(BF16).contiguous()  # noqa: E731
            layers = []
            for L in vm.encoder.layers:
                a = L.self_attn
                layers.append(dict(
                    ln1=(bf(L.layer_norm1.weight), bf(L.layer_norm1.bias), L.layer_norm1.eps),
                    wqkv=bf(torch.cat([a.q_proj.weight, a.k_proj.weight, a.v_proj.weight], 0)),
                    bqkv=bf(torch.cat([a.q_proj.bias, a.k_proj.bias, a.v_proj.bias], 0)),
                    wo=bf(a.out_proj.weight), bo=bf(a.out_proj.bias), heads=a.num_heads,
                    scale=float(a.scale),
                    ln2=(bf(L.layer_norm2.weight), bf(L.layer_norm2.bias), L.layer_norm2.eps),
                    w1=bf(L.mlp.fc1.weight), b1=bf(L.mlp.fc1.bias),
                    w2=bf(L.mlp.fc2.weight), b2=bf(L.mlp.fc2.bias)))
            pre, post = vm.pre_layrnorm, vm.post_layernorm
            self._packed = dict(layers=layers,
                                pre=(bf(pre.weight), bf(pre.bias), pre.eps),
                                post=(bf(post.weight), bf(post.bias), post.eps))
        return self._packed

    @staticmethod
    def _gemm(a, w, bias, residual=None, act=0):
        """A W^T + bias (+ residual / quick-GELU) over the B x 257 token rows, as two launches: the
        first 256 x floor(M / 256) rows and the tail.  32896 rows are 128.5 row blocks of 256: one
        launch would run out_proj / fc2 (N = 1024) as 516 tiles of 256 x 256 = 2.02 rounds of 256
        CUs (a third round for 4 tiles), the q|k|v and fc1 GEMMs as 6.05 / 8.06 rounds; split, the
        bulk is exactly 2 / 6 / 8 rounds and the 128-row tail a small launch of its own."""
        M = a.shape[0]
        Mb = M // 256 * 256
        if Mb == M or Mb == 0:
            return K.gemm(a, w, bias=bias, residual=residual, act=act)
        out = torch.empty(M, w.shape[0], dtype=BF16, device=a.device)
        for r0, r1 in ((0, Mb), (Mb, M)):
            K.gemm(a[r0:r1], w, bias=bias, act=act, out=out[r0:r1],
                   residual=None if residual is None else residual[r0:r1])
        return out

    def _native_hidden(self, vm, x):
        """The encoder on libgvl (module docstring): (B, 257, 1024) bf16, post-layernormed."""
        P = self._pack(vm)
        emb = vm.embeddings(pixel_values=x).to(BF16)  # conv patch embed + class + positions
        B, T, C = emb.shape
        h = K.layernorm_fwd(emb.reshape(B * T, C).contiguous(), *P["pre"][:2], eps=P["pre"][2],
                            stats=False)[0]
        for L in P["layers"]:
            a = K.layernorm_fwd(h, *L["ln1"][:2], eps=L["ln1"][2], stats=False)[0]
            qkv = self._gemm(a, L["wqkv"], L["bqkv"]).view(B, T, 3 * C)
            o, _ = K.attn_fwd(qkv[..., :C], qkv[..., C:2 * C], qkv[..., 2 * C:], L["heads"], False,
                              scale=L["scale"])
            h = self._gemm(o.view(B * T, C), L["wo"], L["bo"], residual=h)
            a = K.layernorm_fwd(h, *L["ln2"][:2], eps=L["ln2"][2], stats=False)[0]
            f = self._gemm(a, L["w1"], L["b1"], act=5)  # fc1 + bias + quick-GELU
            h = self._gemm(f, L["w2"], L["b2"], residual=h)
        h = K.layernorm_fwd(h, *P["post"][:2], eps=P["post"][2], stats=False)[0]
        return h.view(B, T, C)

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
