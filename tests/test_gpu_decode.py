"""KV-cached decoding and the sampling kernel on the MI355X:

  * gvl_attn_decode vs an fp32 torch reference over strided packed-qkv cache views;
  * gvl_sample vs the restated reference samplers (oracle/ops.py sampling_distribution:
    softmax / top-k of train_gpt2.py:444-446 / top-p of gpt2_linear/data.py:116-122) with the
    same uniforms: every draw lies in the reference's kept set, and the drawn index equals
    the inverse-CDF index of the reference distribution (index-order walk) except where u
    falls within fp32 rounding of a CDF boundary; greedy = torch.argmax (first maximum);
  * KV-cached greedy decode == the reference's full-recompute greedy tokens (greedy.npz) and
    == gvl's own full-recompute decode; per-step logits of the cached path vs recompute.
"""
import numpy as np
import pytest
import torch

from oracle import ops as O
from tests.test_gpu_parity_full import GREEDY_BOUND, _build_full, _build_tiny, _recipe, _z

pytestmark = pytest.mark.gpu
BF = torch.bfloat16


def test_attn_decode_matches_reference(cuda):
    import gvl.kernels as K
    g = torch.Generator(device="cuda").manual_seed(0)
    B, H, Tmax, C = 3, 4, 300, 256
    for Tk in (1, 37, 300):
        cache = torch.randn(B, Tmax, 3 * C, device=cuda, generator=g).to(BF)
        q = cache[:, Tk - 1, :C]
        k = cache[:, :Tk, C:2 * C]
        v = cache[:, :Tk, 2 * C:]
        o = K.attn_decode(q, k, v, H)
        qf = q.float().view(B, H, 64)
        kf = k.float().view(B, Tk, H, 64).transpose(1, 2)
        vf = v.float().view(B, Tk, H, 64).transpose(1, 2)
        s = torch.einsum("bhd,bhtd->bht", qf, kf) / 8.0
        want = torch.einsum("bht,bhtd->bhd", s.softmax(-1), vf).reshape(B, C)
        err = (o.float() - want).abs().max().item() / want.abs().max().item()
        print(f"Tk={Tk}: rel err {err:.2e}")
        assert err < 1e-2


@pytest.mark.parametrize("temperature,top_k,top_p", [(1.0, 0, 1.0), (1.0, 50, 1.0), (0.8, 0, 0.9),
                                                     (1.3, 0, 0.5), (0.7, 20, 0.8)])
def test_sampler_matches_reference_distribution(cuda, temperature, top_k, top_p):
    import gvl.kernels as K
    rng = np.random.default_rng(1)
    rows, V = 64, 50304
    logits = (rng.standard_normal((rows, V)) * 2.0).astype(np.float32)
    logits[:, 7] += 6.0  # a peaked head, like a trained LM
    u = rng.random(rows).astype(np.float32)
    lg = torch.from_numpy(logits).to(cuda).to(BF)
    got = K.sample(lg, torch.from_numpy(u).to(cuda), temperature, top_k, top_p).cpu().numpy()
    lb = lg.float().cpu().numpy()  # the bf16 values the kernel read
    exact = 0
    for r in range(rows):
        dist = O.sampling_distribution(lb[r], temperature, top_k, top_p)
        assert dist[got[r]] > 0, f"row {r}: drew {got[r]} outside the reference's kept set"
        if got[r] == O.inverse_cdf_index(dist, float(u[r])):
            exact += 1
        else:  # only a CDF boundary within fp32 rounding of u may flip the index
            cdf = np.cumsum(dist)
            assert np.min(np.abs(cdf - u[r])) < 1e-5, (r, got[r])
    print(f"T={temperature} k={top_k} p={top_p}: {exact}/{rows} draws identical to the oracle")
    assert exact >= rows - 2


def test_sampler_greedy_is_first_argmax(cuda):
    import gvl.kernels as K
    g = torch.Generator(device="cuda").manual_seed(2)
    lg = torch.randn(16, 50304, device=cuda, generator=g).to(BF)
    lg[3, 100] = lg[3, 4000] = 50.0  # a tie: torch.argmax picks the first
    out = K.sample(lg, torch.zeros(16, device=cuda), 1.0, 1, 1.0)
    assert torch.equal(out, lg.float().argmax(-1))


def test_sampler_frequencies(cuda):
    """Many draws from one row: empirical frequencies follow the top-p distribution."""
    import gvl.kernels as K
    rng = np.random.default_rng(3)
    V, N = 512, 200000
    row = (rng.standard_normal(V) * 1.5).astype(np.float32)
    lg = torch.from_numpy(row).to(cuda).expand(N, V)
    u = torch.rand(N, device=cuda, generator=torch.Generator(device="cuda").manual_seed(4))
    got = K.sample(lg, u, 0.8, 0, 0.9).cpu().numpy()
    dist = O.sampling_distribution(row, 0.8, 0, 0.9)
    freq = np.bincount(got, minlength=V) / got.size
    tv = 0.5 * np.abs(freq - dist).sum()
    # sampling noise alone: E[TV] ~ 0.4 * sum(sqrt(p)) / sqrt(N)
    noise = 0.4 * np.sqrt(dist).sum() / np.sqrt(N)
    print(f"total variation {tv:.4f} (noise level {noise:.4f}), kept {int((dist > 0).sum())} tokens")
    assert (freq[dist == 0] == 0).all() and tv < 3 * noise


GREEDY_CASES = [f"{s}_{k}" for s in ("tiny", "full") for k in ("gpt", "linear", "qformer", "cross")]


@pytest.mark.parametrize("case", GREEDY_CASES)
def test_kv_cached_greedy_vs_reference(cuda, golden, case):
    from gvl.decode import generate
    from gvl.generate import greedy_caption, greedy_lm
    from tests.helpers import TINY
    fx = golden("greedy")
    size, kind = case.split("_")
    model = _build_full({"gpt": "lm"}.get(kind, kind)) if size == "full" else _build_tiny(kind)
    model, _ = _recipe(model, cuda)
    model.eval()
    prompt = torch.from_numpy(fx[case + "_prompt"]).to(cuda)
    D = 768 if size == "full" else TINY["n_embd"]
    z = None if kind == "gpt" else _z(int(fx["z_seed"]), 1, D, cuda)
    toks, lg = generate(model, prompt, 16, z=z, greedy=True, return_logits=True)
    got = toks[0].cpu().numpy()
    want, marg = fx[case + "_tokens"][0], fx[case + "_margins"][0]
    n = 0
    for i in range(16):
        if got[i] != want[i]:
            assert marg[i] < GREEDY_BOUND, (case, i, got.tolist(), want.tolist())
            break
        n += 1
    # the cached path against gvl's own full-recompute decode: same tokens, close logits
    if kind == "gpt":
        ref_toks, _ = greedy_lm(model, prompt, 16)
    elif kind == "cross":
        ref_toks, _ = greedy_lm(model, prompt, 16, z=z)
    else:
        ref_toks, _ = greedy_caption(model, z, prompt, 16)
    with torch.no_grad():
        seq = torch.cat([prompt, toks[:, :-1]], 1)
        full = (model(seq)[0] if kind == "gpt" else model(seq, z=z)[0] if kind == "cross"
                else model(z, seq)[0]).float()
    P = prompt.shape[1] + full.shape[1] - seq.shape[1]  # caption logits lead with M image rows
    ref_lg = full[0, P - 1:P - 1 + 16]
    err = (lg[0] - ref_lg).abs().max().item() / ref_lg.abs().max().item()
    same = int((ref_toks[0] == toks[0]).sum())
    print(f"{case}: {n}/16 tokens = reference; {same}/16 = full-recompute gvl; logits rel {err:.2e}")
    assert err < 3e-2


def test_topk_sampling_reproducible(cuda):
    """Top-k 50 sampling as train_gpt2.py:438-449 (4 sequences, seeded generator): same
    seed -> same tokens; every token lies in the top-50 of its step's logits."""
    from gvl.decode import generate
    model, _ = _recipe(_build_tiny("gpt"), cuda)
    model.eval()
    prompt = torch.randint(0, 512, (1, 6), device=cuda).repeat(4, 1)
    outs = []
    for _ in range(2):
        gen = torch.Generator(device="cuda").manual_seed(42)
        outs.append(generate(model, prompt, 12, top_k=50, generator=gen, return_logits=True))
    assert torch.equal(outs[0][0], outs[1][0])
    toks, lg = outs[0]
    top = lg.topk(50, dim=-1).indices
    assert (top == toks.unsqueeze(-1)).any(-1).all()


def test_clip_fused_pool_equals_unfused(cuda):
    """Pixel path (BASELINE configs[3]): pooling CLIP's layer-normed hidden states before the
    bias-free projection (gvl) == pool_clip_197_to_33_avg_with_cls of the projected tokens
    (gpt2_linear/model.py:240-254), up to bf16 rounding."""
    from gvl.clip import CLIPFeatureStage, synthetic_pixels
    clip = CLIPFeatureStage().to(cuda).to(BF)
    px = synthetic_pixels(2, device=cuda)
    a = clip.features(px, fused=True).float()
    b = clip.features(px, fused=False).float()
    assert tuple(a.shape) == (2, 33, 768)
    err = (a - b).abs().max().item() / b.abs().max().item()
    norms = a.norm(dim=-1)
    print(f"fused vs unfused pool: rel err {err:.2e}; row norms {norms.min().item():.4f}..{norms.max().item():.4f}")
    assert err < 3e-2 and torch.allclose(norms, torch.ones_like(norms), atol=1e-2)


def test_clip_native_matches_stock(cuda):
    """gvl-native CLIP encoder (packed q|k|v GEMM, gvl flash attention, bias + residual and
    bias + quick-GELU GEMM epilogues, gvl LayerNorm; gvl/clip.py) against the stock transformers
    tower on the same frozen bf16 weights: the post-layernormed hidden states after 24 layers and
    the pooled, normalised caption features.  Both sides compute in bf16 with different rounding
    points (the stock quick-GELU rounds after each of its three ops), so the bound is a bf16
    drift bound, recorded in parity_margins; the pooled features are the caption models' input."""
    from gvl.clip import CLIPFeatureStage, synthetic_pixels
    from tests.helpers import margins_out
    clip = CLIPFeatureStage().to(cuda).to(BF)
    px = synthetic_pixels(4, device=cuda)
    hs = clip.hidden(px).float()
    fs = clip.features(px).float()
    clip.native = True
    hn = clip.hidden(px).float()
    fn = clip.features(px).float()
    assert hn.shape == hs.shape == (4, 257, 1024)
    h_rel = float((hn - hs).norm() / hs.norm())
    f_rel = float((fn - fs).norm() / fs.norm())
    cos = torch.nn.functional.cosine_similarity(fn.reshape(-1, 768), fs.reshape(-1, 768), dim=-1)
    print(f"native vs stock CLIP: hidden rel-L2 {h_rel:.3e}, features rel-L2 {f_rel:.3e}, "
          f"min cosine {cos.min().item():.5f}")
    margins_out("clip_native_vs_stock", dict(hidden_rel_l2=h_rel, features_rel_l2=f_rel,
                                             min_cosine=float(cos.min())))
    assert torch.isfinite(hn).all()
    assert h_rel < 5e-2 and f_rel < 3e-2 and float(cos.min()) > 0.999
