"""Per-kernel parity on the MI355X: every libgvl entry point vs the CPU oracle.

Inputs are rounded to bf16 first and the oracle runs in fp32 on the rounded values, so the
tolerances measure only the kernels' own rounding (bf16 outputs: ~2^-8 relative).
"""
import math
import os

import numpy as np
import pytest
import torch

from oracle import ops as O
from tests.helpers import rel_err

pytestmark = pytest.mark.gpu
BF = torch.bfloat16


def _k():
    from gvl import kernels as K
    return K


def _r(t):
    """round to bf16, back to fp32 CPU"""
    return t.to(BF).float().cpu()


def keep_mask(seed, idx, p):
    """numpy restatement of common.h rng_keep (splitmix64 finaliser)."""
    G, M1, M2 = np.uint64(0x9E3779B97F4A7C15), np.uint64(0xBF58476D1CE4E5B9), np.uint64(0x94D049BB133111EB)
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + (idx.astype(np.uint64) + np.uint64(1)) * G
        z = (z ^ (z >> np.uint64(30))) * M1
        z = (z ^ (z >> np.uint64(27))) * M2
        z = z ^ (z >> np.uint64(31))
    u = z >> np.uint64(32)
    thresh = np.uint64(int(float(np.float32(p)) * 4294967296.0))
    return u >= thresh


# ------------------------------------------------------------------------------ GEMM
@pytest.mark.parametrize("a_mn,b_mn", [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize("M,N,K", [(256, 384, 192), (200, 136, 72), (8, 8, 8), (130, 264, 1000)])
def test_gemm_layouts(cuda, a_mn, b_mn, M, N, K):
    if (a_mn and M % 8) or (b_mn and N % 8):
        pytest.skip("MN-major operands need multiples of 8")
    K_ = _k()
    torch.manual_seed(M + N + K)
    a = torch.randn(M, K).to(BF)
    b = torch.randn(K, N).to(BF)
    A = (a.t().contiguous() if a_mn else a).to(cuda)
    B = (b if b_mn else b.t().contiguous()).to(cuda)
    c = K_.gemm(A, B, a_mn=bool(a_mn), b_mn=bool(b_mn))
    ref = a.float() @ b.float()
    assert rel_err(c.float().cpu().numpy(), ref.numpy()) < 8e-3


@pytest.mark.parametrize("a_mn,b_mn", [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize("epi", ["plain", "bias", "bias_res", "res_inplace", "bias_act", "dact",
                                 "generic"])
@pytest.mark.parametrize("M,N,K", [(5000, 3080, 160), (4104, 2312, 32)])
def test_gemm_persistent_epilogues(cuda, a_mn, b_mn, epi, M, N, K):
    """Shapes with >= 160 tiles of 256x256 run the persistent ping-pong kernel (several tiles
    per workgroup at 260 tiles, ragged M/N edges, 1- and 5-step tiles) with each
    compile-time epilogue kind; 'generic' (dropout-free gate) takes the fallback path."""
    K_ = _k()
    torch.manual_seed(M + K + len(epi))
    a = torch.randn(M, K).to(BF)
    b = (torch.randn(K, N) * 0.1).to(BF)
    A = (a.t().contiguous() if a_mn else a).to(cuda)
    B = (b if b_mn else b.t().contiguous()).to(cuda)
    h = a.float() @ b.float()
    kw, ref = {}, h
    bias = torch.randn(N).to(BF)
    res = torch.randn(M, N).to(BF)
    if epi == "bias":
        kw, ref = dict(bias=bias.to(cuda)), h + bias.float()
    elif epi == "bias_res":
        kw, ref = dict(bias=bias.to(cuda), residual=res.to(cuda)), h + bias.float() + res.float()
    elif epi == "res_inplace":  # fused gradient accumulation: C += AB
        acc = res.to(cuda)
        kw, ref = dict(residual=acc, out=acc), h + res.float()
    elif epi == "bias_act":
        pre = torch.empty(M, N, dtype=BF, device=cuda)
        kw, ref = dict(bias=bias.to(cuda), act=1, pre_out=pre), O.gelu_tanh(h + bias.float())
    elif epi == "dact":
        hpre = torch.randn(M, N).to(BF)
        hx = hpre.float().requires_grad_(True)
        O.gelu_erf(hx).sum().backward()
        kw, ref = dict(dact=2, pre_in=hpre.to(cuda)), h * hx.grad
    elif epi == "generic":
        gate = torch.tensor(0.3).to(BF)
        kw = dict(residual=res.to(cuda), gate=gate.to(cuda))
        ref = res.float() + math.tanh(float(gate.float())) * h
    y = K_.gemm(A, B, a_mn=bool(a_mn), b_mn=bool(b_mn), **kw)
    assert rel_err(y.float().cpu().numpy(), ref.detach().numpy()) < 8e-3
    if epi == "bias_act":
        assert rel_err(kw["pre_out"].float().cpu().numpy(), (h + bias.float()).numpy()) < 8e-3


@pytest.mark.parametrize("M,N,K", [(4104, 2312, 160), (16384, 768, 64), (300, 392, 96)])
@pytest.mark.parametrize("act", [3, 4])
def test_gemm_gelu_derivative_epilogues(cuda, M, N, K, act):
    """act 3/4: GELU (tanh/erf) with pre_out <- gelu'(x) (what the MLP backward multiplies
    by); dact 3: C = AB * pre_in.  Persistent (256- and 192-wide tiles) and ring kernels."""
    K_ = _k()
    torch.manual_seed(M + N + K + act)
    a = torch.randn(M, K).to(BF)
    b = (torch.randn(K, N) * 0.1).to(BF)
    bias = torch.randn(N).to(BF)
    A, B = a.to(cuda), b.t().contiguous().to(cuda)
    x = (a.float() @ b.float() + bias.float()).requires_grad_(True)
    g = O.gelu_tanh(x) if act == 3 else O.gelu_erf(x)
    g.sum().backward()
    d = torch.empty(M, N, dtype=BF, device=cuda)
    y = K_.gemm(A, B, bias=bias.to(cuda), act=act, pre_out=d)
    assert rel_err(y.float().cpu().numpy(), g.detach().numpy()) < 8e-3
    assert rel_err(d.float().cpu().numpy(), x.grad.numpy()) < 8e-3
    # backward multiply: dY @ W2 (MN-major B) * stored derivative
    dy = torch.randn(M, K).to(BF)
    w2 = (torch.randn(N, K) * 0.1).to(BF)  # nn.Linear(N -> K) weight [K, N] viewed as [N, K]^T
    z = K_.gemm(dy.to(cuda), w2.t().contiguous().to(cuda), b_mn=True, dact=3, pre_in=d)
    ref = (dy.float() @ w2.float().t()) * d.float().cpu()
    assert rel_err(z.float().cpu().numpy(), ref.numpy()) < 8e-3


class _pp3_routing:
    """gvl_gemm_tune(3, 11): default routing without the four-wave kernels (gemm_w4 and the
    AGPR gemm_w4x, which takes the plain / bias + residual M = 16384, N = 768 shapes by
    default), for the tests that pin the persistent kernel on such shapes."""

    def __enter__(self):
        from gvl import _lib
        _lib.lib().gvl_gemm_tune(3, 11)

    def __exit__(self, *exc):
        from gvl import _lib
        _lib.lib().gvl_gemm_tune(3, -1)


def _kernel_name(A, B, a_mn, b_mn, M, N, K, tickets=False, epi=None):
    """Kernel gvl_gemm picks for this shape; `epi` (a test epilogue name) sets the
    descriptor's epilogue fields the way gvl.kernels.gemm does (the routing depends on it)."""
    import ctypes as C
    from gvl import _lib
    d = _lib.GemmDesc()
    d.a, d.b, d.c = A.data_ptr(), B.data_ptr(), A.data_ptr()
    d.m, d.n, d.k = M, N, K
    d.lda, d.ldb, d.ldc = A.stride(0), B.stride(0), N
    d.a_mn, d.b_mn = a_mn, b_mn
    d.alpha = 1.0
    p = A.data_ptr()  # any aligned device pointer: only the routing is asked
    if epi in ("bias", "bias_res", "bias_act_d", "drop_res", "qgelu"):
        d.bias = p
    if epi == "qgelu":
        d.act = 5
    if epi in ("bias_res", "res_inplace", "drop_res"):
        d.residual, d.ldr = p, N
    if epi == "bias_act_d":
        d.act, d.pre_out, d.ldp = 3, p, N
    if epi in ("mul", "dact", "dact_erf"):
        d.dact, d.pre_in, d.ldp = {"mul": 3, "dact": 1, "dact_erf": 2}[epi], p, N
    if epi == "drop_res":
        d.drop_p, d.seed = 0.1, 1
    if epi == "gate_res":
        d.bias, d.residual, d.ldr, d.gate, d.pre_out, d.ldp = p, p, N, p, p, N
    if True:  # as gvl.kernels.gemm passes them (workspace + in-launch combine tickets, always)
        K_ = _k()
        ws, tk = K_._gemm_workspace(A.device), K_._gemm_tickets(A.device)
        d.workspace, d.workspace_bytes = ws.data_ptr(), ws.numel() * 4
        d.tickets, d.ticket_count = tk.data_ptr(), tk.numel()
    buf = C.create_string_buffer(128)
    _lib.lib().gvl_gemm_kernel_name(C.byref(d), buf, 128)
    return buf.value.decode()


@pytest.mark.parametrize("K,b_mn,epi", [(3072, 1, "plain"), (2304, 1, "plain"), (768, 1, "plain"),
                                         (3072, 0, "bias_res"), (768, 0, "bias_res")])
def test_gemm_linear_decoder_rows(cuda, K, b_mn, epi):
    """The linear caption decoder's 8192-row N = 768 GEMMs: 258 of the direct-A kernel's 192 x 128
    tiles (one round and 2 tiles), so the default routing takes the AGPR kernel's 128 x 192 tiles
    (exactly 256); vs the fp32 product (round 5; before: the 128 x 128 ring kernel)."""
    K_ = _k()
    M, N = 8192, 768
    torch.manual_seed(K + b_mn)
    a = torch.randn(M, K).to(BF)
    b = (torch.randn(K, N) * 0.05).to(BF)
    A = a.to(cuda)
    B = (b if b_mn else b.t().contiguous()).to(cuda)
    name = _kernel_name(A, B, 0, b_mn, M, N, K, epi=epi)
    if os.environ.get("GVL_W4X_128", "2") != "0":
        assert name.startswith("gemm_w4x_kernel<128, 192"), name
    h = a.float() @ b.float()
    kw, ref = {}, h
    if epi == "bias_res":
        bias, res = torch.randn(N).to(BF), torch.randn(M, N).to(BF)
        kw, ref = dict(bias=bias.to(cuda), residual=res.to(cuda)), h + bias.float() + res.float()
    y = K_.gemm(A, B, b_mn=bool(b_mn), **kw)
    torch.cuda.synchronize()
    assert rel_err(y.float().cpu().numpy(), ref.numpy()) < 8e-3


@pytest.mark.parametrize("M,N,K,a_mn,b_mn", [(8064, 768, 3072, 0, 1), (8064, 768, 3072, 0, 0),
                                               (4096, 768, 3072, 0, 1)])
def test_gemm_caption_dx_on_own_kernels(cuda, M, N, K, a_mn, b_mn):
    """The plain N = 768 products that round 4 handed to hipBLASLt (the caption decoder's and the
    Q-Former MLP's c_fc.dX) run on libgvl's four-wave kernels since ABI v10: vs the fp32
    product, with alpha, and replayed from a captured hipGraph."""
    K_ = _k()
    torch.manual_seed(M + N + K)
    a = torch.randn(M, K).to(BF)
    b = (torch.randn(K, N) * 0.05).to(BF)
    A = (a.t().contiguous() if a_mn else a).to(cuda)
    B = (b if b_mn else b.t().contiguous()).to(cuda)
    assert _kernel_name(A, B, a_mn, b_mn, M, N, K, epi="plain").startswith("gemm_w4")
    ref = a.float() @ b.float()
    y = K_.gemm(A, B, a_mn=bool(a_mn), b_mn=bool(b_mn), alpha=0.5)
    assert rel_err(y.float().cpu().numpy(), 0.5 * ref.numpy()) < 8e-3
    out = torch.empty(M, N, dtype=BF, device=cuda)
    K_.gemm(A, B, a_mn=bool(a_mn), b_mn=bool(b_mn), out=out)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        K_.gemm(A, B, a_mn=bool(a_mn), b_mn=bool(b_mn), out=out)
    out.zero_()
    g.replay()
    torch.cuda.synchronize()
    assert rel_err(out.float().cpu().numpy(), ref.numpy()) < 8e-3


@pytest.mark.parametrize("a_mn,b_mn", [(0, 0), (0, 1), (1, 0), (1, 1)])
def test_gemm_strided_output_view(cuda, a_mn, b_mn):
    """Every operand layout with ragged sizes into a strided output view: the columns past N
    are never written."""
    K_ = _k()
    M, N, K = 1000, 776, 160
    torch.manual_seed(a_mn * 2 + b_mn)
    a = torch.randn(M, K).to(BF)
    b = torch.randn(K, N).to(BF)
    A = (a.t().contiguous() if a_mn else a).to(cuda)
    B = (b if b_mn else b.t().contiguous()).to(cuda)
    big = torch.full((M, N + 8), 7.0, dtype=BF, device=cuda)
    K_.gemm(A, B, a_mn=bool(a_mn), b_mn=bool(b_mn), out=big[:, :N])
    assert rel_err(big[:, :N].float().cpu().numpy(), (a.float() @ b.float()).numpy()) < 8e-3
    assert torch.all(big[:, N:] == 7.0)


@pytest.mark.parametrize("b_mn", [0, 1])
@pytest.mark.parametrize("epi", ["plain", "bias_res"])
@pytest.mark.parametrize("M,N,K", [(16384, 768, 3072), (16384, 768, 768), (1000, 776, 160),
                                   (4096, 2304, 96), (512, 768, 64), (16384, 3072, 768),
                                   (8064, 768, 3072), (8064, 768, 768)])
def test_gemm_w4x(cuda, b_mn, epi, M, N, K):
    """Four-wave AGPR-accumulator kernel (gemm_w4x.hip), forced with gvl_gemm_tune(3, 12) (and
    chosen by default for the LM's N = 768 shapes, checked by name):
    256- and 128-row tiles (the latter below ~0.9 chip of 256-row tiles: M = 8064), both B
    layouts, plain (alpha 0.5) and bias + residual epilogues, ragged M / N tiles, K of 2 and 3
    steps (shorter than the ring), one and four tiles per CU; the output is a strided
    view inside a sentinel-filled buffer (no store past the tile edges)."""
    from gvl import _lib
    K_ = _k()
    torch.manual_seed(M + N + K + b_mn)
    a = torch.randn(M, K).to(BF)
    b = (torch.randn(K, N) * 0.05).to(BF)
    A = a.to(cuda)
    B = (b if b_mn else b.t().contiguous()).to(cuda)
    h = a.float() @ b.float()
    _lib.lib().gvl_gemm_tune(3, 12)
    try:
        assert _kernel_name(A, B, 0, b_mn, M, N, K, epi=epi).startswith("gemm_w4x")
        big = torch.full((M + 3, N + 8), 7.0, dtype=BF, device=cuda)
        out = big[:M, :N]
        if epi == "plain":
            K_.gemm(A, B, b_mn=bool(b_mn), out=out, alpha=0.5)
            ref = 0.5 * h
        else:
            bias, res = torch.randn(N).to(BF), torch.randn(M, N).to(BF)
            K_.gemm(A, B, b_mn=bool(b_mn), out=out, bias=bias.to(cuda), residual=res.to(cuda))
            ref = h + bias.float() + res.float()
        torch.cuda.synchronize()
    finally:
        _lib.lib().gvl_gemm_tune(3, -1)
    if M == 16384 and N == 768:
        assert _kernel_name(A, B, 0, b_mn, M, N, K, epi=epi).startswith("gemm_w4x_kernel")
    assert rel_err(out.float().cpu().numpy(), ref.numpy()) < 8e-3
    assert torch.all(big[:, N:] == 7.0) and torch.all(big[M:, :] == 7.0)


@pytest.mark.parametrize("epi", ["plain", "bias", "bias_act_d", "bias_act_erf_d"])
@pytest.mark.parametrize("M,N,K", [(8064, 3072, 768), (7999, 2240, 768), (16384, 768, 3072),
                                   (4096, 2304, 768), (2048, 50304, 768)])
def test_gemm_counted_epilogue(cuda, epi, M, N, K):
    """Counted epilogue of the persistent kernel (gemm_pp3.h CntEpi: bias row in LDS, buffer
    stores with dropped out-of-range lanes, the next NS - 2 waits counting them): every kind
    it takes, ragged M and N (M-tail rows, a partial last column tile), several tiles per CU,
    the lm_head width; vs the fp32 product + bias (+ GELU / gelu'), and a sentinel-bordered
    output for the tails."""
    K_ = _k()
    if epi == "bias" and N > 4096:
        pytest.skip("lm_head carries no bias")
    torch.manual_seed(M + N + K + len(epi))
    a = torch.randn(M, K).to(BF)
    b = (torch.randn(K, N) * 0.05).to(BF)
    A, B = a.to(cuda), b.t().contiguous().to(cuda)
    with _pp3_routing():
        name = _kernel_name(A, B, 0, 0, M, N, K, epi={"bias_act_erf_d": "bias_act_d"}.get(epi, epi))
    assert name.startswith("gemm_pp3_kernel"), name
    bias = torch.randn(N).to(BF)
    h = a.float() @ b.float() + (0 if epi == "plain" else bias.float())
    kw, ref = {}, h
    if epi == "bias":
        kw = dict(bias=bias.to(cuda))
    elif epi != "plain":
        erf = epi == "bias_act_erf_d"
        x = h.clone().requires_grad_(True)
        g = O.gelu_erf(x) if erf else O.gelu_tanh(x)
        g.sum().backward()
        pre = torch.empty(M, N, dtype=BF, device=cuda)
        kw, ref = dict(bias=bias.to(cuda), act=4 if erf else 3, pre_out=pre), g.detach()
    with _pp3_routing():
        y = K_.gemm(A, B, **kw)
    assert rel_err(y.float().cpu().numpy(), ref.numpy()) < 8e-3
    if "pre_out" in kw:
        assert rel_err(kw["pre_out"].float().cpu().numpy(), x.grad.numpy()) < 8e-3
    if M % 256 or N % 192:  # tail stores must not land outside the output
        big = torch.full((M + 3, N + 64), 7.0, dtype=BF, device=cuda)
        if "pre_out" in kw:
            pbig = torch.full((M + 3, N + 64), 7.0, dtype=BF, device=cuda)
            kw["pre_out"] = pbig[:M, :N]
        K_.gemm(A, B, out=big[:M, :N], **kw)
        assert torch.all(big[M:] == 7.0) and torch.all(big[:, N:] == 7.0)
        assert torch.equal(big[:M, :N], y)
        if "pre_out" in kw:
            assert torch.all(pbig[M:] == 7.0) and torch.all(pbig[:, N:] == 7.0)


@pytest.mark.parametrize("M,N,K,bn", [(50304, 768, 4096, 256), (16000, 768, 4096, 192)])
def test_gemm_w4x_wgrad_single(cuda, M, N, K, bn):
    """The tied lm_head's weight gradient through gvl_gemm (C += alpha * dY^T X, both operands
    MN-contiguous, alpha from a device scalar) on the AGPR four-wave kernel: 256 x 256 tiles
    at the vocabulary's 50304 rows (591 tiles), 256 x 192 where they fill the chip better."""
    K_ = _k()
    torch.manual_seed(M + K)
    dy = (torch.randn(K, M) * 0.1).to(BF)
    x = (torch.randn(K, N) * 0.1).to(BF)
    c0 = torch.randn(M, N).to(BF)
    A, B = dy.to(cuda), x.to(cuda)
    out = c0.to(cuda)
    name = _kernel_name(A, B, 1, 1, M, N, K, epi="res_inplace")
    assert name.startswith(f"gemm_w4x_kernel<256, {bn}, true, true"), name
    scale = torch.tensor([0.25], device=cuda)
    K_.gemm(A, B, a_mn=True, b_mn=True, alpha_ptr=scale, out=out, residual=out)
    ref = 0.25 * (dy.float().t() @ x.float()) + c0.float()
    assert rel_err(out.float().cpu().numpy(), ref.numpy()) < 8e-3


@pytest.mark.parametrize("act", [0, 3])
def test_gemm_counted_epilogue_streaming_stores(cuda, act):
    """Outputs past 1 GiB (the LM's lm_head logits) take the counted epilogue's streaming (sc1 nt)
    stores: 10800 x 50304 bf16 = 1.09 GB, plain and with the GELU side output (two streams),
    ragged M, vs the fp32 product."""
    K_ = _k()
    M, N, K = 10800, 50304, 128
    torch.manual_seed(act)
    a = torch.randn(M, K).to(BF)
    b = (torch.randn(K, N) * 0.05).to(BF)
    A, B = a.to(cuda), b.t().contiguous().to(cuda)
    h = a.float() @ b.float()
    if act:
        bias = torch.randn(N).to(BF)
        pre = torch.empty(M, N, dtype=BF, device=cuda)
        y = K_.gemm(A, B, bias=bias.to(cuda), act=3, pre_out=pre)
        x = (h + bias.float()).requires_grad_(True)
        g = O.gelu_tanh(x)
        g.sum().backward()
        assert rel_err(y.float().cpu().numpy(), g.detach().numpy()) < 8e-3
        assert rel_err(pre.float().cpu().numpy(), x.grad.numpy()) < 8e-3
    else:
        y = K_.gemm(A, B)
        assert rel_err(y.float().cpu().numpy(), h.numpy()) < 8e-3


@pytest.mark.parametrize("a_mn,b_mn", [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize("epi", ["plain", "bias_res", "res_inplace", "bias_act", "dact"])
@pytest.mark.parametrize("M,N,K", [(16384, 768, 768), (12000, 1536, 320), (16384, 2304, 32)])
def test_gemm_tile192(cuda, a_mn, b_mn, epi, M, N, K):
    """192-wide output tiles of the persistent kernel (picked when they fill the last round of
    CUs better: 16384 x 768 -> 256 tiles instead of 192): every layout incl. the split
    [32][128] + [32][64] MN-contiguous B image, odd fragment count in the epilogue (3 x 16
    columns per wave), ragged M, a single K-step."""
    K_ = _k()
    torch.manual_seed(M + N + K + len(epi) + 5 * a_mn + 11 * b_mn)
    a = torch.randn(M, K).to(BF)
    b = (torch.randn(K, N) * 0.1).to(BF)
    A = (a.t().contiguous() if a_mn else a).to(cuda)
    B = (b if b_mn else b.t().contiguous()).to(cuda)
    with _pp3_routing():
        assert ", 192, " in _kernel_name(A, B, a_mn, b_mn, M, N, K)  # 256- or 128-row tiles
    h = a.float() @ b.float()
    bias = torch.randn(N).to(BF)
    res = torch.randn(M, N).to(BF)
    kw, ref = {}, h
    if epi == "bias_res":
        kw, ref = dict(bias=bias.to(cuda), residual=res.to(cuda)), h + bias.float() + res.float()
    elif epi == "res_inplace":
        acc = res.to(cuda)
        kw, ref = dict(residual=acc, out=acc), h + res.float()
    elif epi == "bias_act":
        pre = torch.empty(M, N, dtype=BF, device=cuda)
        kw, ref = dict(bias=bias.to(cuda), act=1, pre_out=pre), O.gelu_tanh(h + bias.float())
    elif epi == "dact":
        hpre = torch.randn(M, N).to(BF)
        hx = hpre.float().requires_grad_(True)
        O.gelu_tanh(hx).sum().backward()
        kw, ref = dict(dact=1, pre_in=hpre.to(cuda)), h * hx.grad
    with _pp3_routing():
        y = K_.gemm(A, B, a_mn=bool(a_mn), b_mn=bool(b_mn), **kw)
    assert rel_err(y.float().cpu().numpy(), ref.detach().numpy()) < 8e-3
    if epi == "bias_act":
        assert rel_err(kw["pre_out"].float().cpu().numpy(), (h + bias.float()).numpy()) < 8e-3


@pytest.mark.parametrize("a_mn,b_mn", [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize("epi", ["plain", "bias_res", "res_inplace", "bias_act_d", "mul", "dact_erf"])
@pytest.mark.parametrize("M,N,K", [(8064, 768, 3072), (8064, 768, 768), (7992, 768, 2304)])
def test_gemm_splitk_combined_in_launch(cuda, a_mn, b_mn, epi, M, N, K):
    """The caption decoder's N = 768 GEMMs at M = 8064: 128 tiles of 256x192, each K split in
    two halves that meet inside the launch (write-through partials + per-(tile, wave) arrival
    tickets; the last arriver adds and runs the epilogue).  Every layout and epilogue kind,
    ragged M; the result is bitwise reproducible (two-term fp32 sums commute, whichever half
    arrives last) and the tickets are all zero again afterwards."""
    K_ = _k()
    torch.manual_seed(M + N + K + len(epi) + 5 * a_mn + 11 * b_mn)
    a = torch.randn(M, K).to(BF)
    b = (torch.randn(K, N) * 0.05).to(BF)
    A = (a.t().contiguous() if a_mn else a).to(cuda)
    B = (b if b_mn else b.t().contiguous()).to(cuda)
    from gvl import _lib
    _lib.lib().gvl_gemm_tune(3, 13)  # default routing minus the four-wave kernels, pp3 combine on
    try:
        name = _kernel_name(A, B, a_mn, b_mn, M, N, K, tickets=True)
    finally:
        _lib.lib().gvl_gemm_tune(3, -1)
    assert name.startswith("gemm_pp3_kernel") and name.endswith(", 192, 256>"), name
    h = a.float() @ b.float()
    bias = torch.randn(N).to(BF)
    res = torch.randn(M, N).to(BF)
    kw, ref = {}, h
    if epi == "bias_res":
        kw, ref = dict(bias=bias.to(cuda), residual=res.to(cuda)), h + bias.float() + res.float()
    elif epi == "res_inplace":
        kw, ref = dict(residual=None, out=None), h + res.float()
    elif epi == "bias_act_d":
        x = (h + bias.float()).requires_grad_(True)
        g = O.gelu_erf(x)
        g.sum().backward()
        pre = torch.empty(M, N, dtype=BF, device=cuda)
        kw, ref = dict(bias=bias.to(cuda), act=4, pre_out=pre), g.detach()
    elif epi == "mul":
        d = torch.randn(M, N).to(BF)
        kw, ref = dict(dact=3, pre_in=d.to(cuda)), h * d.float()
    elif epi == "dact_erf":
        hpre = torch.randn(M, N).to(BF)
        hx = hpre.float().requires_grad_(True)
        O.gelu_erf(hx).sum().backward()
        kw, ref = dict(dact=2, pre_in=hpre.to(cuda)), h * hx.grad
    outs = []
    _lib.lib().gvl_gemm_tune(3, 13)
    try:
        for _ in range(2):
            if epi == "res_inplace":
                acc = res.to(cuda)
                kw = dict(residual=acc, out=acc)
            outs.append(K_.gemm(A, B, a_mn=bool(a_mn), b_mn=bool(b_mn), **kw))
    finally:
        _lib.lib().gvl_gemm_tune(3, -1)
    torch.cuda.synchronize()
    assert rel_err(outs[0].float().cpu().numpy(), ref.detach().numpy()) < 8e-3
    assert torch.equal(outs[0], outs[1])
    if epi == "bias_act_d":
        assert rel_err(kw["pre_out"].float().cpu().numpy(), x.grad.numpy()) < 8e-3
    assert int(K_._gemm_tickets(A.device).abs().sum()) == 0


@pytest.mark.parametrize("a_mn,b_mn", [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize("epi", ["plain", "bias_res", "res_inplace", "bias_act_d", "mul", "dact"])
@pytest.mark.parametrize("M,N,K", [(8064, 768, 3072), (8064, 768, 768), (7992, 768, 32)])
def test_gemm_tile128x192(cuda, a_mn, b_mn, epi, M, N, K):
    """128x192 tiles of the persistent kernel (the caption decoder's N = 768 GEMMs at
    M = 8064: 63 x 4 = 252 tiles, one round on 256 CUs): every layout (the 128-row A slab is
    one DMA piece per wave) and epilogue kind, ragged M, a single K-step."""
    K_ = _k()
    torch.manual_seed(M + N + K + len(epi) + 3 * a_mn + 7 * b_mn)
    a = torch.randn(M, K).to(BF)
    b = (torch.randn(K, N) * 0.05).to(BF)
    A = (a.t().contiguous() if a_mn else a).to(cuda)
    B = (b if b_mn else b.t().contiguous()).to(cuda)
    name = _kernel_name(A, B, a_mn, b_mn, M, N, K, epi=epi)
    if not a_mn and K % 192 == 0:  # K-contiguous A: a four-wave 192x128 kernel takes it
        assert name.startswith(_w4_name(M, K, epi)), name
    elif a_mn and K >= 3072:  # with gvl.kernels' workspace the planner splits K: 128x128 ring
        assert name.startswith("gemm_ring_kernel") or name.endswith(", 192, 128>"), name
    else:
        assert name.startswith("gemm_pp3_kernel") and name.endswith(", 192, 128>"), name
    h = a.float() @ b.float()
    bias = torch.randn(N).to(BF)
    res = torch.randn(M, N).to(BF)
    kw, ref = {}, h
    if epi == "bias_res":
        kw, ref = dict(bias=bias.to(cuda), residual=res.to(cuda)), h + bias.float() + res.float()
    elif epi == "res_inplace":
        acc = res.to(cuda)
        kw, ref = dict(residual=acc, out=acc), h + res.float()
    elif epi == "bias_act_d":
        x = (h + bias.float()).requires_grad_(True)
        g = O.gelu_tanh(x)
        g.sum().backward()
        pre = torch.empty(M, N, dtype=BF, device=cuda)
        kw, ref = dict(bias=bias.to(cuda), act=3, pre_out=pre), g.detach()
    elif epi == "mul":
        d = torch.randn(M, N).to(BF)
        kw, ref = dict(dact=3, pre_in=d.to(cuda)), h * d.float()
    elif epi == "dact":
        hpre = torch.randn(M, N).to(BF)
        hx = hpre.float().requires_grad_(True)
        O.gelu_tanh(hx).sum().backward()
        kw, ref = dict(dact=1, pre_in=hpre.to(cuda)), h * hx.grad
    y = K_.gemm(A, B, a_mn=bool(a_mn), b_mn=bool(b_mn), **kw)
    assert rel_err(y.float().cpu().numpy(), ref.detach().numpy()) < 8e-3
    if epi == "bias_act_d":
        assert rel_err(kw["pre_out"].float().cpu().numpy(), x.grad.numpy()) < 8e-3


# epilogues gemm_w4d_kernel is instantiated for (gemm_w4d.h epi_supported)
W4D_EPIS = ("plain", "bias", "bias_res", "res_inplace", "drop_res")


def _w4_tiles(M, N, b_mn=0, cus=256):
    """(128-row tiles?, 128 x 96 tiles?) as gemm_w4.hip's w4_use128 / w4_use96 decide (96-column
    tiles for a K-contiguous B only, unless GVL_W4_BN96=2)."""
    tn = -(-N // 128)
    t192, t128 = -(-M // 192) * tn, -(-M // 128) * tn
    r128 = t192 * 4 < cus * 3 and t128 > t192 and t128 <= cus
    t96 = -(-M // 128) * -(-N // 96)
    mode = int(os.environ.get("GVL_W4_BN96", "1"))
    c96 = r128 and mode != 0 and (not b_mn or mode >= 2) and t128 < t96 <= cus
    return r128, c96


def _w4_rows96(M, N, b_mn, epi, cus=256):
    """96 x 128 dX tiles (gemm_w4r_kernel) as gemm_w4.hip's w4_use96r decides: MN-contiguous B,
    plain epilogue, 128-row tiles in use and 96-row ones filling more of the chip in one round."""
    r128, _ = _w4_tiles(M, N, b_mn, cus)
    tn = -(-N // 128)
    t128, t96 = -(-M // 128) * tn, -(-M // 96) * tn
    return (r128 and b_mn and epi == "plain" and os.environ.get("GVL_W4_BM96", "1") != "0"
            and t128 < t96 <= cus)


def _w4_name(M, K, epi, N=768, b_mn=0):
    """Kernel the default four-wave routing picks (GVL_W4D unset): the direct-A variant
    (gemm_w4d.h) when K is a multiple of six 64-deep steps and the epilogue is one of its;
    128-row tiles where 192-row ones fill under 3/4 of the chip, 128 x 96 ones (gemm_w4n_kernel)
    where those fill more of it in one round."""
    mode = os.environ.get("GVL_W4D", "1")
    r128, c96 = _w4_tiles(M, N, b_mn)
    rows = "m" if r128 else ""
    direct = K % 384 == 0 and epi in W4D_EPIS and mode != "0" and (mode == "2" or not rows)
    if direct:
        return f"gemm_w4d{rows}_kernel"
    if _w4_rows96(M, N, b_mn, epi):
        return "gemm_w4r_kernel"
    return "gemm_w4n_kernel" if c96 else f"gemm_w4{rows}_kernel"


@pytest.mark.parametrize("b_mn", [0, 1])
@pytest.mark.parametrize("epi", ["plain", "bias", "bias_res", "res_inplace", "bias_act_d", "mul", "dact_erf"])
@pytest.mark.parametrize("M,N,K", [(8064, 768, 3072), (8064, 768, 2304), (7992, 776, 192),
                                   (16384, 768, 384), (300, 128, 192), (8064, 3072, 768),
                                   (3968, 768, 3072), (4096, 768, 768), (3970, 776, 192),
                                   (7992, 776, 384), (3970, 904, 768)])
def test_gemm_w4(cuda, b_mn, epi, M, N, K):
    """Four-wave 192x128 / 128x128 deep-ring kernel (gemm_w4.hip), forced with gvl_gemm_tune(3, 10):
    the caption decoder's N = 768 shapes (252 tiles, one per CU), ragged M and N (N % 128 != 0),
    several tiles per workgroup with the ring running across tiles (516 tiles), a tile grid
    smaller than the ring, and every epilogue kind."""
    from gvl import _lib
    K_ = _k()
    torch.manual_seed(M + N + K + len(epi) + 7 * b_mn)
    a = torch.randn(M, K).to(BF)
    b = (torch.randn(K, N) * 0.05).to(BF)
    A = a.to(cuda)
    B = (b if b_mn else b.t().contiguous()).to(cuda)
    h = a.float() @ b.float()
    bias = torch.randn(N).to(BF)
    res = torch.randn(M, N).to(BF)
    kw, ref = {}, h
    if epi == "bias":
        kw, ref = dict(bias=bias.to(cuda)), h + bias.float()
    elif epi == "bias_res":
        kw, ref = dict(bias=bias.to(cuda), residual=res.to(cuda)), h + bias.float() + res.float()
    elif epi == "res_inplace":
        acc = res.to(cuda)
        kw, ref = dict(residual=acc, out=acc), h + res.float()
    elif epi == "bias_act_d":
        x = (h + bias.float()).requires_grad_(True)
        g = O.gelu_tanh(x)
        g.sum().backward()
        pre = torch.empty(M, N, dtype=BF, device=cuda)
        kw, ref = dict(bias=bias.to(cuda), act=3, pre_out=pre), g.detach()
    elif epi == "mul":
        d = torch.randn(M, N).to(BF)
        kw, ref = dict(dact=3, pre_in=d.to(cuda)), h * d.float()
    elif epi == "dact_erf":
        hpre = torch.randn(M, N).to(BF)
        hx = hpre.float().requires_grad_(True)
        O.gelu_erf(hx).sum().backward()
        kw, ref = dict(dact=2, pre_in=hpre.to(cuda)), h * hx.grad
    _lib.lib().gvl_gemm_tune(3, 10)
    try:
        name = _kernel_name(A, B, 0, b_mn, M, N, K, epi=epi)
        y = K_.gemm(A, B, a_mn=False, b_mn=bool(b_mn), **kw)
        torch.cuda.synchronize()
    finally:
        _lib.lib().gvl_gemm_tune(3, -1)
    # 128-row tiles (gemm_w4m_kernel / gemm_w4dm_kernel) where 192-row ones would fill < 3/4
    # of the CUs; the direct-A variant where K % 384 == 0 and its epilogue is instantiated
    assert name.startswith(_w4_name(M, K, epi, N, b_mn)), name
    assert rel_err(y.float().cpu().numpy(), ref.detach().numpy()) < 8e-3
    if epi == "bias_act_d":
        assert rel_err(kw["pre_out"].float().cpu().numpy(), x.grad.numpy()) < 8e-3


@pytest.mark.parametrize("M,N,K,force", [(3968, 768, 768, False), (3970, 776, 192, True),
                                         (300, 128, 192, True), (8064, 768, 768, True)])
def test_gemm_w4_gated_residual(cuda, M, N, K, force):
    """y = residual + tanh(gate) * (x W^T + b) with the un-gated branch stored (EPI_GATE_RES,
    gemm_w4.hip): the cross-att decoder's xattn.c_proj (gpt2_cross-att/model.py:57,99-101).  At
    its shape (3968 x 768 x 768) the default routing takes the 128-row four-wave kernel (round 4:
    the generic-epilogue ring kernel); forced on ragged M / N, a sub-chip grid and 192-row tiles."""
    from gvl import _lib
    K_ = _k()
    torch.manual_seed(M + N + K)
    x = torch.randn(M, K).to(BF)
    w = (torch.randn(N, K) * 0.05).to(BF)
    bias = torch.randn(N).to(BF)
    res = torch.randn(M, N).to(BF)
    gate = torch.tensor(-0.45).to(BF)
    ybr = torch.full((M, N), float("nan"), dtype=BF, device=cuda)
    A, B = x.to(cuda), w.to(cuda)
    if force:
        _lib.lib().gvl_gemm_tune(3, 10)
    try:
        name = _kernel_name(A, B, 0, 0, M, N, K, epi="gate_res")
        y = K_.gemm(A, B, bias=bias.to(cuda), residual=res.to(cuda), gate=gate.to(cuda), pre_out=ybr)
        torch.cuda.synchronize()
    finally:
        _lib.lib().gvl_gemm_tune(3, -1)
    assert "gemm_w4" in name and name.endswith(", 13>"), name
    h = x.float() @ w.float().t() + bias.float()
    ref = res.float() + math.tanh(float(gate.float())) * h
    assert rel_err(y.float().cpu().numpy(), ref.numpy()) < 8e-3
    assert rel_err(ybr.float().cpu().numpy(), h.numpy()) < 8e-3


@pytest.mark.parametrize("a_mn,b_mn,M,N,K", [(1, 1, 768, 768, 8192), (0, 1, 256, 512, 4096),
                                             (0, 0, 384, 256, 6144)])
@pytest.mark.parametrize("impl", [3, 2])
def test_gemm_splitk_epilogue(cuda, a_mn, b_mn, M, N, K, impl):
    """Few output tiles + long K -> split-K partials + reduce kernel applying the epilogue."""
    K_ = _k()
    torch.manual_seed(M + K)
    a = torch.randn(M, K).to(BF)
    b = (torch.randn(K, N) * 0.05).to(BF)
    A = (a.t().contiguous() if a_mn else a).to(cuda)
    B = (b if b_mn else b.t().contiguous()).to(cuda)
    bias = torch.randn(N).to(BF)
    res = torch.randn(M, N).to(BF)
    alpha = torch.tensor([0.5], dtype=torch.float32)
    from gvl import _lib
    _lib.lib().gvl_gemm_tune(impl, -1)
    try:
        y = K_.gemm(A, B, a_mn=bool(a_mn), b_mn=bool(b_mn), bias=bias.to(cuda), act=1,
                    residual=res.to(cuda), alpha_ptr=alpha.to(cuda))
    finally:
        _lib.lib().gvl_gemm_tune(3, -1)
    ref = O.gelu_tanh(0.5 * (a.float() @ b.float()) + bias.float()) + res.float()
    assert rel_err(y.float().cpu().numpy(), ref.numpy()) < 8e-3


@pytest.mark.parametrize("M,N,K", [(768, 768, 16384), (2304, 768, 8192), (768, 3072, 4096)])
@pytest.mark.parametrize("impl", [3, 2])
def test_gemm_wgrad_inplace_accumulate(cuda, M, N, K, impl):
    """Weight-gradient GEMM accumulating into the gradient it reads (C = dY^T X + C, the
    fused gradient accumulation of gvl.functional), through split-K and whole-K tiles."""
    K_ = _k()
    torch.manual_seed(M + N + K)
    dy = torch.randn(K, M).to(BF)
    x = (torch.randn(K, N) * 0.05).to(BF)
    g0 = torch.randn(M, N).to(BF)
    from gvl import _lib
    _lib.lib().gvl_gemm_tune(impl, -1)
    try:
        g = g0.to(cuda)
        K_.linear_dw(dy.to(cuda), x.to(cuda), out=g, residual=g)
    finally:
        _lib.lib().gvl_gemm_tune(3, -1)
    ref = dy.float().t() @ x.float() + g0.float()
    assert rel_err(g.float().cpu().numpy(), ref.numpy()) < 8e-3


@pytest.mark.parametrize("a_mn,b_mn", [(0, 0), (0, 1), (1, 0)])
@pytest.mark.parametrize("epi", ["bias_res", "bias_act", "dact"])
@pytest.mark.parametrize("M,N,K", [(8064, 768, 768), (8064, 768, 3072), (5000, 904, 96)])
@pytest.mark.parametrize("cfg", [-1, 6, 1])
def test_gemm_ring_band(cuda, a_mn, b_mn, epi, M, N, K, cfg):
    """Outputs of 256..512 tiles of 128x128 (the caption step's N = 768 GEMMs at M = 8064)
    through the ring tile configs selectable for them: the default 128x128, 64x128 (K-contiguous
    A only; an MN-contiguous A falls back to 128x128) and 256x128; ragged M/N edges and each
    epilogue kind the caption step uses."""
    K_ = _k()
    from gvl import _lib
    torch.manual_seed(M + N + K + len(epi))
    a = torch.randn(M, K).to(BF)
    b = (torch.randn(K, N) * 0.05).to(BF)
    A = (a.t().contiguous() if a_mn else a).to(cuda)
    B = (b if b_mn else b.t().contiguous()).to(cuda)
    h = a.float() @ b.float()
    bias = torch.randn(N).to(BF)
    if epi == "bias_res":
        res = torch.randn(M, N).to(BF)
        kw, ref = dict(bias=bias.to(cuda), residual=res.to(cuda)), h + bias.float() + res.float()
    elif epi == "bias_act":
        kw, ref = dict(bias=bias.to(cuda), act=2), O.gelu_erf(h + bias.float())
    else:
        hpre = torch.randn(M, N).to(BF)
        hx = hpre.float().requires_grad_(True)
        O.gelu_tanh(hx).sum().backward()
        kw, ref = dict(dact=1, pre_in=hpre.to(cuda)), h * hx.grad
    _lib.lib().gvl_gemm_tune(2 if cfg >= 0 else 3, cfg)
    try:
        y = K_.gemm(A, B, a_mn=bool(a_mn), b_mn=bool(b_mn), **kw)
    finally:
        _lib.lib().gvl_gemm_tune(3, -1)
    assert rel_err(y.float().cpu().numpy(), ref.detach().numpy()) < 8e-3


@pytest.mark.parametrize("act", [1, 2])
def test_gemm_epilogue_act_bias_residual(cuda, act):
    K_ = _k()
    torch.manual_seed(act)
    M, N, Kd = 192, 256, 384
    x = torch.randn(M, Kd).to(BF)
    w = (torch.randn(N, Kd) * 0.05).to(BF)
    bias = torch.randn(N).to(BF)
    res = torch.randn(M, N).to(BF)
    pre = torch.empty(M, N, dtype=BF, device=cuda)
    y = K_.gemm(x.to(cuda), w.to(cuda), bias=bias.to(cuda), act=act, pre_out=pre,
                residual=res.to(cuda))
    h = x.float() @ w.float().t() + bias.float()
    g = O.gelu_tanh(h) if act == 1 else O.gelu_erf(h)
    assert rel_err(pre.float().cpu().numpy(), h.numpy()) < 8e-3
    assert rel_err(y.float().cpu().numpy(), (g + res.float()).numpy()) < 8e-3


@pytest.mark.parametrize("dact", [1, 2])
def test_gemm_dgelu_alpha_ptr(cuda, dact):
    K_ = _k()
    torch.manual_seed(10 + dact)
    M, N, Kd = 128, 192, 256
    dy = torch.randn(M, Kd).to(BF)
    w = (torch.randn(Kd, N) * 0.05).to(BF)  # nn.Linear weight [out=Kd][in=N]
    hpre = torch.randn(M, N).to(BF)
    alpha = torch.tensor([0.37], dtype=torch.float32)
    out = K_.gemm(dy.to(cuda), w.to(cuda), b_mn=True, dact=dact, pre_in=hpre.to(cuda),
                  alpha_ptr=alpha.to(cuda))
    hx = hpre.float().requires_grad_(True)
    (O.gelu_tanh(hx) if dact == 1 else O.gelu_erf(hx)).sum().backward()
    ref = 0.37 * (dy.float() @ w.float()) * hx.grad
    assert rel_err(out.float().cpu().numpy(), ref.numpy()) < 8e-3


def test_gemm_dropout_gate(cuda):
    K_ = _k()
    torch.manual_seed(3)
    M, N, Kd = 96, 128, 64
    x = torch.randn(M, Kd).to(BF)
    w = (torch.randn(N, Kd) * 0.1).to(BF)
    res = torch.randn(M, N).to(BF)
    gate = torch.tensor(0.7).to(BF)
    ybr = torch.empty(M, N, dtype=BF, device=cuda)
    p, seed = 0.1, 987654321
    y = K_.gemm(x.to(cuda), w.to(cuda), residual=res.to(cuda), gate=gate.to(cuda),
                pre_out=ybr, drop_p=p, seed=seed)
    h = x.float() @ w.float().t()
    keep = torch.from_numpy(keep_mask(seed, np.arange(M * N), p).reshape(M, N))
    hd = torch.where(keep, h / (1 - p), torch.zeros_like(h))
    ref = res.float() + math.tanh(float(gate.float())) * hd
    assert rel_err(y.float().cpu().numpy(), ref.numpy()) < 8e-3
    assert rel_err(ybr.float().cpu().numpy(), hd.numpy()) < 8e-3
    frac = 1 - keep.float().mean().item()
    assert 0.08 < frac < 0.12


@pytest.mark.parametrize("M,N,Kd,kern", [(4096, 768, 768, _w4_name(4096, 768, "drop_res", 768)),
                                         (4096, 3072, 768, "gemm_pp3_kernel"),
                                         (200, 136, 72, None), (4096, 768, 3072, None)])
def test_gemm_bias_dropout_residual(cuda, M, N, Kd, kern):
    """Compile-time bias + dropout + residual epilogue (EPI_BIAS_DROP_RES, the Q-Former's
    out_proj / MLP output branches) in the four-wave and persistent kernels, and the same op
    on the generic paths: mask = the counter hash of (m, n), exactly as the numpy restatement."""
    K_ = _k()
    torch.manual_seed(M + N + Kd)
    x = torch.randn(M, Kd).to(BF)
    w = (torch.randn(N, Kd) * 0.05).to(BF)
    bias = torch.randn(N).to(BF)
    res = torch.randn(M, N).to(BF)
    p, seed = 0.1, 123456789
    A, B = x.to(cuda), w.to(cuda)
    if kern is not None:
        name = _kernel_name(A, B, 0, 0, M, N, Kd, epi="drop_res")
        assert name.startswith(kern), name
    y = K_.gemm(A, B, bias=bias.to(cuda), residual=res.to(cuda), drop_p=p, seed=seed)
    h = x.float() @ w.float().t() + bias.float()
    keep = torch.from_numpy(keep_mask(seed, np.arange(M * N), p).reshape(M, N))
    ref = res.float() + torch.where(keep, h / (1 - p), torch.zeros_like(h))
    assert rel_err(y.float().cpu().numpy(), ref.numpy()) < 8e-3
    # every dropped element is exactly the residual
    yd = y.float().cpu()[~keep]
    assert torch.equal(yd, res.float()[~keep])


@pytest.mark.parametrize("count,M,N,K,acc", [(12, 768, 768, 4096, True), (12, 2304, 768, 2048, True),
                                             (3, 3072, 768, 1024, False), (2, 200, 136, 96, True),
                                             (17, 256, 256, 64, True), (12, 768, 768, 16384, True),
                                             (12, 768, 768, 1024, False), (12, 3072, 768, 1024, True),
                                             (12, 768, 3072, 512, True), (12, 1000, 776, 96, True),
                                             (9, 3072, 768, 256, True)])
def test_gemm_batched_wgrad(cuda, count, M, N, K, acc):
    """gvl_gemm_batched: `count` weight-gradient GEMMs dW_i (+)= dY_i^T X_i (both operands
    MN-contiguous, as the deferred GPT-2 block weight gradients) in one persistent launch;
    each equals its own reference.  count 17 (> 16) and a ragged shape exercise the fallback.
    12 x (768, 768) — the LM's attn.c_proj at K = 16384 and shorter — runs as a two-way K
    split combined in-launch, with the fused bias row sums combined through the workspace;
    the second (dbias) launch also checks that the first left the tickets at zero.  Batches of
    accumulating problems whose 256 x 192 tiles fill the chip run on the AGPR four-wave kernel
    (gemm_w4x.hip: MN-contiguous A and B by asm transposed reads, fused bias row sums), incl.
    ragged M / N and a 3-step K."""
    import ctypes as C
    from gvl import _lib
    K_ = _k()
    torch.manual_seed(count + M + N + K)
    dys = [torch.randn(K, M).to(BF) for _ in range(count)]
    xs = [(torch.randn(K, N) * 0.1).to(BF) for _ in range(count)]
    c0 = [torch.randn(M, N).to(BF) for _ in range(count)]
    outs = [c.to(cuda) for c in c0]
    K_.gemm_batched([(dy.to(cuda), x.to(cuda), o, acc) for dy, x, o in zip(dys, xs, outs)],
                    a_mn=True, b_mn=True)
    buf = C.create_string_buffer(128)
    _lib.lib().gvl_gemm_batched_kernel_name(buf, 128)
    if acc and count == 12 and (M, N) in ((2304, 768), (1000, 776)):  # whole rounds of 256 x 192
        assert buf.value.decode().startswith("gemm_w4x_kernel"), buf.value
    for dy, x, c, o in zip(dys, xs, c0, outs):
        ref = dy.float().t() @ x.float() + (c.float() if acc else 0)
        assert rel_err(o.float().cpu().numpy(), ref.numpy()) < 8e-3
    if acc:  # fused bias gradients: db_i += column sums of dY_i, from the same launch
        b0 = [torch.randn(M).to(BF) for _ in range(count)]
        dbs = [b.to(cuda) for b in b0]
        outs = [c.to(cuda) for c in c0]
        fused = K_.gemm_batched([(dy.to(cuda), x.to(cuda), o, True) for dy, x, o in zip(dys, xs, outs)],
                                a_mn=True, b_mn=True, dbias=dbs)
        assert fused == (2 <= count <= 16)
        if fused:
            for dy, x, c, o, b, db in zip(dys, xs, c0, outs, b0, dbs):
                ref = dy.float().t() @ x.float() + c.float()
                assert rel_err(o.float().cpu().numpy(), ref.numpy()) < 8e-3
                assert rel_err(db.float().cpu().numpy(), (dy.float().sum(0) + b.float()).numpy()) < 1e-2


@pytest.mark.parametrize("shapes", [
    [(4096, 768, 768), (4096, 768, 768), (4096, 3072, 768), (4096, 768, 3072), (4224, 768, 1024),
     (96, 200, 136)],
    # the Q-Former step's whole flush incl. the in_proj row slices: 256 x 192 tiles fill better
    [(4096, 768, 768)] * 4 + [(4096, 3072, 768)] * 2 + [(4096, 768, 3072)] * 2 + [(4224, 768, 1024)]
    + [(4096, 2304, 768)] * 2 + [(4096, 768, 768)] * 2 + [(4224, 1536, 768)] * 2,
    # an LM backward flush (12 blocks x c_attn / attn.c_proj / c_fc / mlp.c_proj, 48 problems,
    # the GVL_MAX_GROUP limit) at 1024 of its 16384 tokens
    [(1024, 768, 3072), (1024, 3072, 768), (1024, 768, 768), (1024, 2304, 768)] * 12,
    # one problem: its bias sum is fused too (a grouped launch of one problem used to
    # skip the Db update while reporting success)
    [(4096, 768, 3072)]])
def test_gemm_grouped_wgrad(cuda, shapes):
    """gvl_gemm_grouped: weight gradients of different shapes (the Q-Former bridge's deferred
    out_proj / MLP / projection dW at K = 4096 / 4224 tokens, plus a ragged 200 x 136 one over
    3 K-steps) in one launch of the AGPR four-wave kernel, out += dy^T x, with the bias sums
    fused for some problems and not others; each vs its own fp32 reference."""
    import ctypes as C
    from gvl import _lib
    K_ = _k()
    torch.manual_seed(len(shapes))
    dys = [(torch.randn(k, m) * 0.1).to(BF) for k, m, n in shapes]
    xs = [(torch.randn(k, n) * 0.1).to(BF) for k, m, n in shapes]
    c0 = [torch.randn(m, n).to(BF) for k, m, n in shapes]
    b0 = [torch.randn(m).to(BF) for k, m, n in shapes]
    outs = [c.to(cuda) for c in c0]
    dbs = [(b.to(cuda) if i % 2 == 0 else None) for i, b in enumerate(b0)]
    assert K_.gemm_grouped([(dy.to(cuda), x.to(cuda), o) for dy, x, o in zip(dys, xs, outs)], dbias=dbs)
    buf = C.create_string_buffer(128)
    _lib.lib().gvl_gemm_batched_kernel_name(buf, 128)
    assert buf.value.decode() in ("gemm_w4x_kernel<256, 256, true, true, 6, true>",
                                  "gemm_w4x_kernel<256, 192, true, true, 6, true>"), buf.value
    torch.cuda.synchronize()
    for dy, x, c, o, b, db in zip(dys, xs, c0, outs, b0, dbs):
        ref = dy.float().t() @ x.float() + c.float()
        assert rel_err(o.float().cpu().numpy(), ref.numpy()) < 8e-3
        if db is not None:
            assert rel_err(db.float().cpu().numpy(), (dy.float().sum(0) + b.float()).numpy()) < 1e-2


def test_gemm_grouped_device_scale(cuda):
    """ABI v11: a grouped launch where some problems carry the device scalar (the tied lm_head's
    dW, scaled by dloss / count: a 50304-row problem, shrunk here to 2000 rows) and the others
    none; each vs its fp32 reference.  Two different scale tensors in one call are declined."""
    K_ = _k()
    torch.manual_seed(11)
    shapes = [(1024, 2000, 768), (1024, 768, 3072), (1024, 3072, 768), (1024, 2304, 768)]
    dys = [(torch.randn(k, m) * 0.1).to(BF) for k, m, n in shapes]
    xs = [(torch.randn(k, n) * 0.1).to(BF) for k, m, n in shapes]
    c0 = [torch.randn(m, n).to(BF) for k, m, n in shapes]
    b0 = [torch.randn(m).to(BF) for k, m, n in shapes]
    scale = torch.tensor([0.37], device=cuda)
    outs = [c.to(cuda) for c in c0]
    dbs = [None] + [b.to(cuda) for b in b0[1:]]
    items = [(dy.to(cuda), x.to(cuda), o, scale if i == 0 else None)
             for i, (dy, x, o) in enumerate(zip(dys, xs, outs))]
    assert K_.gemm_grouped(items, dbias=dbs)
    torch.cuda.synchronize()
    for i, (dy, x, c, o, b, db) in enumerate(zip(dys, xs, c0, outs, b0, dbs)):
        a = 0.37 if i == 0 else 1.0
        ref = a * (dy.float().t() @ x.float()) + c.float()
        assert rel_err(o.float().cpu().numpy(), ref.numpy()) < 8e-3, i
        if db is not None:
            assert rel_err(db.float().cpu().numpy(), (dy.float().sum(0) + b.float()).numpy()) < 1e-2
    other = torch.tensor([2.0], device=cuda)
    before = [o.clone() for o in outs]
    assert not K_.gemm_grouped([items[0], items[1][:3] + (other,)])
    torch.cuda.synchronize()
    for o, b in zip(outs, before):
        assert torch.equal(o, b)


def test_gemm_grouped_declines_past_limit(cuda):
    """gvl_gemm_grouped returns -1 (gemm_grouped False) for 49 problems, launching nothing."""
    K_ = _k()
    dy = torch.randn(64, 64, device=cuda).to(BF)
    x = torch.randn(64, 64, device=cuda).to(BF)
    outs = [torch.zeros(64, 64, device=cuda, dtype=BF) for _ in range(49)]
    assert not K_.gemm_grouped([(dy, x, o) for o in outs])
    assert K_.gemm_grouped([(dy, x, o) for o in outs[:48]])
    torch.cuda.synchronize()
    assert float(outs[48].float().abs().max()) == 0.0
    ref = dy.float().t() @ x.float()
    assert rel_err(outs[47].float().cpu().numpy(), ref.cpu().numpy()) < 8e-3


@pytest.mark.parametrize("count,rows,cols", [(12, 16384, 2304), (12, 4096, 768), (3, 1000, 3080),
                                             (1, 37, 8)])
@pytest.mark.parametrize("acc", [False, True])
def test_colsum_batched(cuda, count, rows, cols, acc):
    """gvl_colsum_batched (the deferred bias gradients): out_i (+)= column sums of x_i."""
    K_ = _k()
    torch.manual_seed(count + rows + cols)
    xs = [torch.randn(rows, cols).to(BF) for _ in range(count)]
    o0 = [torch.randn(cols).to(BF) for _ in range(count)]
    outs = [o.to(cuda) for o in o0]
    K_.colsum_batched([x.to(cuda) for x in xs], outs, accumulate=acc)
    for x, o, r in zip(xs, o0, outs):
        ref = x.float().sum(0) + (o.float() if acc else 0)
        assert rel_err(r.float().cpu().numpy(), ref.numpy()) < 1e-2


# ------------------------------------------------------------------------- LayerNorm
@pytest.mark.parametrize("rows,C", [(37, 128), (300, 768), (5, 1024), (20011, 768), (1000, 520)])
def test_layernorm_fwd_bwd(cuda, rows, C):
    K_ = _k()
    torch.manual_seed(rows)
    x = (torch.randn(rows, C) * 2 + 0.5).to(BF)
    w = (1 + 0.1 * torch.randn(C)).to(BF)
    b = (0.1 * torch.randn(C)).to(BF)
    y, mean, rstd = K_.layernorm_fwd(x.to(cuda), w.to(cuda), b.to(cuda))
    xr = x.float().requires_grad_(True)
    wr = w.float().requires_grad_(True)
    br = b.float().requires_grad_(True)
    ref = O.layernorm(xr, wr, br)
    assert rel_err(y.float().cpu().numpy(), ref.detach().numpy()) < 8e-3
    dy = torch.randn(rows, C).to(BF)
    ref.backward(dy.float())
    prev = torch.randn(rows, C).to(BF)
    dx = prev.clone().to(cuda)
    dw = torch.empty(C, dtype=BF, device=cuda)
    db = torch.empty(C, dtype=BF, device=cuda)
    K_.layernorm_bwd(dy.to(cuda), x.to(cuda), w.to(cuda), mean, rstd, dx=dx, accumulate_dx=True,
                     dw=dw, db=db)
    assert rel_err(dx.float().cpu().numpy(), (xr.grad + prev.float()).numpy()) < 1e-2
    assert rel_err(dw.float().cpu().numpy(), wr.grad.numpy()) < 1e-2
    assert rel_err(db.float().cpu().numpy(), br.grad.numpy()) < 1e-2
    # accumulate_wb: dw/db += (fused gradient accumulation)
    dw0, db0 = dw.float().cpu(), db.float().cpu()
    K_.layernorm_bwd(dy.to(cuda), x.to(cuda), w.to(cuda), mean, rstd, dw=dw, db=db,
                     accumulate_wb=True)
    assert rel_err(dw.float().cpu().numpy(), (dw0 + wr.grad).numpy()) < 1e-2
    assert rel_err(db.float().cpu().numpy(), (db0 + br.grad).numpy()) < 1e-2
    # residual read from its own buffer (gvl_layernorm_bwd_res): dx = prev + LN backward,
    # prev untouched
    prev_d = prev.to(cuda)
    dx2 = torch.full((rows, C), float("nan"), dtype=BF, device=cuda)
    K_.layernorm_bwd(dy.to(cuda), x.to(cuda), w.to(cuda), mean, rstd, dx=dx2, residual=prev_d)
    assert rel_err(dx2.float().cpu().numpy(), (xr.grad + prev.float()).numpy()) < 1e-2
    assert torch.equal(prev_d.cpu(), prev)
    # ABI v12: dw / db left as partials, reduced later by the batched finalize (two items: this
    # LayerNorm's and a second one over the first half of the rows, db only), bit-identical to
    # the in-place finalize
    dx3, (ws, nblk) = K_.layernorm_bwd(dy.to(cuda), x.to(cuda), w.to(cuda), mean, rstd,
                                       residual=prev_d, defer_wb=True)
    assert torch.equal(dx3, dx2)
    h = max(rows // 2, 1)
    _, (ws2, nblk2) = K_.layernorm_bwd(dy[:h].to(cuda), x[:h].to(cuda), w.to(cuda), mean[:h], rstd[:h],
                                       defer_wb=True)
    dwb, dbb = dw0.to(BF).to(cuda), db0.to(BF).to(cuda)
    db2 = torch.zeros(C, dtype=BF, device=cuda)
    K_.layernorm_finalize_batched([(ws, nblk, dwb, dbb), (ws2, nblk2, None, db2)], C, accumulate=True)
    dwr, dbr = dw0.to(BF).to(cuda), db0.to(BF).to(cuda)
    K_.layernorm_bwd(dy.to(cuda), x.to(cuda), w.to(cuda), mean, rstd, dw=dwr, db=dbr, accumulate_wb=True)
    assert torch.equal(dwb, dwr) and torch.equal(dbb, dbr)
    assert rel_err(db2.float().cpu().numpy(), dy[:h].float().sum(0).numpy()) < 1e-2


# ------------------------------------------------------------------------- attention
def _attn_case(cuda, B, H, Tq, Tk, causal, packed, drop_p=0.0, seed=0, grad=True):
    K_ = _k()
    torch.manual_seed(B * 100 + Tq + Tk)
    C = H * 64
    q = torch.randn(B, Tq, C).to(BF)
    k = torch.randn(B, Tk, C).to(BF)
    v = torch.randn(B, Tk, C).to(BF)
    if packed:  # q, k, v as column slices of one [B, T, 3C] buffer (c_attn output)
        buf = torch.cat([q, k, v], dim=2).to(cuda)
        qg, kg, vg = buf[:, :, :C], buf[:, :, C:2 * C], buf[:, :, 2 * C:]
    else:
        qg, kg, vg = q.to(cuda), k.to(cuda), v.to(cuda)
    o, lse = K_.attn_fwd(qg, kg, vg, H, causal, drop_p=drop_p, seed=seed)
    qr, kr, vr = (t.float().requires_grad_(True) for t in (q, k, v))
    sq, sk, sv = (O.split_heads(t, H) for t in (qr, kr, vr))
    if drop_p > 0:
        s = (sq @ sk.transpose(-1, -2)) / 8.0
        if causal:
            s = s.masked_fill(~torch.ones(Tq, Tk, dtype=torch.bool).tril(), float("-inf"))
        pr = torch.softmax(s, dim=-1)
        idx = np.arange(B * H * Tq * Tk)
        keep = torch.from_numpy(keep_mask(seed, idx, drop_p).reshape(B, H, Tq, Tk))
        pr = torch.where(keep, pr / (1 - drop_p), torch.zeros_like(pr))
        ref = O.merge_heads(pr @ sv)
    else:
        ref = O.merge_heads(O.attention(sq, sk, sv, causal))
    assert rel_err(o.float().cpu().numpy(), ref.detach().numpy()) < 1.2e-2
    if not grad:
        return
    do = torch.randn(B, Tq, C).to(BF)
    ref.backward(do.float())
    if packed:
        dbuf = torch.empty(B, Tq, 3 * C, dtype=BF, device=cuda)
        dq, dk, dv = dbuf[:, :, :C], dbuf[:, :, C:2 * C], dbuf[:, :, 2 * C:]
    else:
        dq = torch.empty(B, Tq, C, dtype=BF, device=cuda)
        dk = torch.empty(B, Tk, C, dtype=BF, device=cuda)
        dv = torch.empty(B, Tk, C, dtype=BF, device=cuda)
    K_.attn_bwd(do.to(cuda), qg, kg, vg, o, lse, H, causal, dq, dk, dv, drop_p=drop_p, seed=seed)
    for got, want, nm in ((dq, qr.grad, "dq"), (dk, kr.grad, "dk"), (dv, vr.grad, "dv")):
        e = rel_err(got.float().cpu().numpy(), want.numpy())
        assert e < 2.5e-2, f"{nm} rel err {e}"


@pytest.mark.parametrize("B,H,T", [(2, 2, 80), (1, 2, 1024), (2, 2, 300), (3, 12, 63), (2, 3, 64), (1, 1, 7),
                                   (3, 3, 50), (40, 12, 31), (5, 12, 32), (2, 2, 1), (2, 3, 17)])
def test_attention_causal(cuda, B, H, T):
    _attn_case(cuda, B, H, T, T, True, packed=True)


@pytest.mark.parametrize("Tq,Tk", [(31, 33), (32, 32), (32, 33), (100, 257), (40, 130), (130, 1000),
                                   (1, 32), (20, 9), (20, 64), (1, 40)])
def test_attention_noncausal(cuda, Tq, Tk):
    _attn_case(cuda, 2, 2, Tq, Tk, False, packed=False)


@pytest.mark.parametrize("Tq,Tk", [(32, 33), (40, 130), (32, 32), (17, 29), (31, 50)])
def test_attention_dropout_exact_mask(cuda, Tq, Tk):
    _attn_case(cuda, 2, 2, Tq, Tk, False, packed=False, drop_p=0.1, seed=4242)


def test_attention_short_over_nan_filled_memory(cuda):
    """The single-launch short backward (Q / dO fragments and the dO row piece of D read back
    from its LDS tiles) repeated over NaN-filled free memory, causal 63-token and dropout 32 x 33
    cases, and the 32-row kernel's causal 31-token and dropout 32 x 32 cases: any byte read before
    it is written shows up as an intermittent error."""
    for it in range(6):
        junk = torch.full((32 << 20,), float("nan"), device=cuda)
        del junk
        _attn_case(cuda, 4, 6, 63, 63, True, packed=True)
        _attn_case(cuda, 3, 2, 32, 33, False, packed=False, drop_p=0.1, seed=77 + it)
        _attn_case(cuda, 4, 6, 31, 31, True, packed=True)
        _attn_case(cuda, 3, 2, 32, 32, False, packed=False, drop_p=0.1, seed=91 + it)


def test_attention_bwd_repeats_over_nan_filled_memory(cuda):
    """The dropout case (40 queries x 130 keys) 12 times, the caching allocator's free memory
    filled with NaN before each: a backward that reads any byte it did not write, or races,
    shows up as an intermittent dQ / dK / dV error (round 3: a dQ kernel computing D itself
    failed 4 of 40 such repeats; tools/attn_stress.py)."""
    for it in range(12):
        junk = torch.full((32 << 20,), float("nan"), device=cuda)
        del junk
        _attn_case(cuda, 2, 2, 40, 130, False, packed=False, drop_p=0.1, seed=4242 + it)


def test_attention_matches_reference_fixture(cuda, golden):
    """SDPA fixtures produced by the reference's torch path (tools/make_fixtures.py)."""
    K_ = _k()
    fx = golden("ops")
    for name, causal in (("sdpa_causal", True), ("sdpa_cross", False), ("sdpa_self32", False)):
        q, k, v = (torch.from_numpy(fx[f"{name}:{n}"]) for n in "qkv")
        B, H = q.shape[0], q.shape[1]
        to_bt = lambda t: t.transpose(1, 2).reshape(t.shape[0], t.shape[2], -1).to(BF).to(cuda)
        o, _ = K_.attn_fwd(to_bt(q), to_bt(k), to_bt(v), H, causal)
        want = torch.from_numpy(fx[f"{name}:o"]).transpose(1, 2).reshape(B, q.shape[2], -1)
        assert rel_err(o.float().cpu().numpy(), want.numpy()) < 2e-2


# ----------------------------------------------------------------- CE / embed / pool
def test_cross_entropy(cuda, golden):
    K_ = _k()
    fx = golden("ops")
    lg = torch.from_numpy(fx["ce:logits"]).to(BF)
    tg = torch.from_numpy(fx["ce:targets"])
    out, dl = K_.cross_entropy(lg.to(cuda), tg.to(cuda))
    ref = O.cross_entropy(lg.float(), tg)
    assert abs(out[0].item() - float(ref)) / float(ref) < 1e-5
    p = torch.softmax(lg.float(), -1)
    oh = torch.zeros_like(p)
    valid = tg != -100
    oh[valid, tg[valid]] = 1.0
    want = torch.where(valid.unsqueeze(1), p - oh, torch.zeros_like(p))
    assert rel_err(dl.float().cpu().numpy(), want.numpy()) < 8e-3
    assert abs(out[1].item() - 1.0 / valid.sum().item()) < 1e-7
    tg2 = torch.from_numpy(fx["ce:targets2"])
    mk = torch.from_numpy(fx["ce:mask"])
    out2, _ = K_.cross_entropy(lg.to(cuda), tg2.to(cuda), mask=mk.to(cuda), mask_mode=True)
    ref2 = O.masked_cross_entropy(lg.float(), tg2, mk)
    assert abs(out2[0].item() - float(ref2)) / float(ref2) < 1e-5


def test_cross_entropy_row_mapping_fullvocab(cuda):
    """Caption layout: loss rows are logits[:, M:M+T] of a [B, S, V] tensor, V=50304."""
    K_ = _k()
    torch.manual_seed(5)
    B, S, M, T, V = 3, 12, 5, 7, 50304
    lg = (torch.randn(B, S, V) * 3).to(BF)
    tg = torch.randint(0, 50257, (B, T))
    tg[0, 3] = -100
    out, dl = K_.cross_entropy(lg.view(B * S, V).to(cuda), tg.to(cuda), rows_per_group=T,
                               group_stride=S, row_offset=M)
    ref = O.cross_entropy(lg[:, M:M + T].float(), tg)
    assert abs(out[0].item() - float(ref)) / float(ref) < 1e-5


def test_embedding_fwd_bwd(cuda):
    K_ = _k()
    torch.manual_seed(7)
    V, P, C, B, T, M = 300, 64, 128, 3, 20, 4
    wte = torch.randn(V, C).to(BF)
    wpe = torch.randn(P, C).to(BF)
    idx = torch.randint(0, V, (B, T))
    out = torch.zeros(B, M + T, C, dtype=BF, device=cuda)
    K_.embedding_fwd(idx.to(cuda), wte.to(cuda), wpe.to(cuda), out, T, M + T, M)
    want = wte.float()[idx] + wpe.float()[:T]
    assert rel_err(out[:, M:].float().cpu().numpy(), want.numpy()) < 5e-3
    assert out[:, :M].abs().max().item() == 0
    dout = torch.randn(B, M + T, C).to(BF)
    ate = torch.zeros(V, C, device=cuda)
    ape = torch.zeros(P, C, device=cuda)
    K_.embedding_bwd(idx.to(cuda), dout.to(cuda), ate, ape, T, M + T, M, C, V)
    wr = wte.float().requires_grad_(True)
    pr = wpe.float().requires_grad_(True)
    ((wr[idx] + pr[:T]) * dout[:, M:].float()).sum().backward()
    assert rel_err(ate.cpu().numpy(), wr.grad.numpy()) < 1e-5
    assert rel_err(ape.cpu().numpy(), pr.grad.numpy()) < 1e-5


@pytest.mark.parametrize("case", ["small", "lm", "hot", "chunks"])
def test_embedding_bwd_det_bit_exact(cuda, case):
    """gvl_embedding_bwd_det: per-id fp32 sums in token order, one bf16 update per row —
    emulated exactly on the host (np.add.at applies its updates in index order), so the
    result must match BIT FOR BIT, including hot ids (one id repeated thousands of times),
    out-of-range ids (skipped), a token count that is not a whole number of sort tiles and
    inputs longer than one 16,384-token chunk (chunks applied in order)."""
    K_ = _k()
    V, C, G, T, M = {"small": (300, 128, 3, 20, 4), "lm": (50304, 768, 16, 1024, 0),
                     "hot": (1000, 256, 5, 700, 2), "chunks": (4000, 64, 9, 4000, 1)}[case]
    gen = torch.Generator().manual_seed(11)
    idx = torch.randint(0, V, (G, T), generator=gen)
    if case == "hot":
        idx[:, ::2] = 7          # 1,750 copies of id 7, interleaved
        idx[1, 5] = V + 3        # out of range: contributes nothing
        idx[2, 9] = -1
    dout = torch.randn(G, M + T, C, generator=gen).to(BF)
    w0 = torch.randn(V, C, generator=gen).to(BF)
    p0 = torch.randn(T + 5, C, generator=gen).to(BF)
    gte, gpe = w0.to(cuda), p0.to(cuda)
    K_.embedding_bwd_det(idx.to(cuda), dout.to(cuda), gte, gpe, T, M + T, M, C, V)
    # host emulation, chunk by chunk (16,384 tokens) and position by position within a chunk
    ids = idx.reshape(-1).numpy()
    rows = dout[:, M:].reshape(-1, C).float().numpy()
    want = w0.clone()
    for c0 in range(0, ids.size, 16384):
        ci, cr = ids[c0:c0 + 16384], rows[c0:c0 + 16384]
        ok = (ci >= 0) & (ci < V)
        acc = np.zeros((V, C), np.float32)
        np.add.at(acc, ci[ok], cr[ok])
        touched = np.unique(ci[ok])
        upd = want.float().numpy()
        upd[touched] = upd[touched] + acc[touched]
        want = torch.from_numpy(upd).to(BF)
    assert torch.equal(gte.cpu().view(torch.int16), want.view(torch.int16)), case
    pacc = dout[:, M:].float().numpy()
    ps = np.zeros((T, C), np.float32)
    for g in range(G):
        ps += pacc[g]
    wp = p0.float().numpy().copy()
    wp[:T] += ps
    assert torch.equal(gpe.cpu().view(torch.int16), torch.from_numpy(wp).to(BF).view(torch.int16))
    # and run to run
    again = w0.to(cuda)
    K_.embedding_bwd_det(idx.to(cuda), dout.to(cuda), again, None, T, M + T, M, C, V)
    assert torch.equal(again, gte)


@pytest.mark.parametrize("side", [16, 14])
def test_pool_clip(cuda, golden, side):
    K_ = _k()
    fx = golden("ops")
    tok = torch.from_numpy(fx[f"pool{side}:in"])
    out = K_.pool_clip(tok.to(cuda))
    assert rel_err(out.cpu().numpy(), fx[f"pool{side}:out"]) < 1e-5
    outb = K_.pool_clip(tok.to(BF).to(cuda))
    want = O.pool_clip(tok.to(BF).float())
    assert rel_err(outb.float().cpu().numpy(), want.numpy()) < 8e-3


def test_pool_clip_full_size(cuda):
    K_ = _k()
    tok = torch.randn(4, 257, 768)
    out = K_.pool_clip(tok.to(cuda))
    assert rel_err(out.cpu().numpy(), O.pool_clip(tok).numpy()) < 1e-5


# -------------------------------------------------------------------- optimizer path
def test_grad_norm_and_adamw(cuda, golden):
    K_ = _k()
    fx = golden("ops")
    p1 = torch.from_numpy(fx["adam:p1"]).to(BF)
    p2 = torch.from_numpy(fx["adam:p2"]).to(BF)
    g1 = torch.from_numpy(fx["adam:g1"])
    g2 = torch.from_numpy(fx["adam:g2"])
    n1, n2 = p1.numel(), p2.numel()
    P = torch.cat([p1.reshape(-1), p2.reshape(-1)]).to(cuda)
    Mm = torch.zeros_like(P)
    Vv = torch.zeros_like(P)
    refp = [p1.float().clone(), p2.float().clone()]
    st = [(torch.zeros_like(refp[0]), torch.zeros_like(refp[0])),
          (torch.zeros_like(refp[1]), torch.zeros_like(refp[1]))]
    for it in range(2):
        gs = [(g1 * (it + 1)).to(BF), (g2 * (it + 1)).to(BF)]
        G = torch.cat([gs[0].reshape(-1), gs[1].reshape(-1)]).to(cuda)
        out = K_.grad_norm(G, 1.0)
        nrm, coef = O.clip_coef([g.float() for g in gs], 1.0)
        assert abs(out[0].item() - float(nrm)) / float(nrm) < 1e-5
        assert abs(out[1].item() - coef) < 1e-6
        K_.adamw(P[:n1], G[:n1], Mm[:n1], Vv[:n1], n1, 1e-3, 0.9, 0.95, 1e-8, 0.1, it + 1, out[1:2])
        K_.adamw(P[n1:], G[n1:], Mm[n1:], Vv[n1:], n2, 1e-3, 0.9, 0.95, 1e-8, 0.0, it + 1, out[1:2])
        for j in range(2):
            O.adamw_update(refp[j], gs[j].float() * coef, st[j][0], st[j][1], it + 1, 1e-3,
                           wd=0.1 if j == 0 else 0.0)
    got = P.float().cpu()
    assert rel_err(got[:n1].numpy(), refp[0].reshape(-1).numpy()) < 1e-2
    assert rel_err(got[n1:].numpy(), refp[1].reshape(-1).numpy()) < 1e-2


@pytest.mark.parametrize("rows,cols", [(16384, 768), (8064, 3072), (3, 2304), (0, 16), (777, 264)])
def test_colsum_shapes(cuda, rows, cols):
    """Bias-gradient column sums at the model's shapes (split partials + finish), plus the
    accumulate flag used by fused gradient accumulation."""
    K_ = _k()
    torch.manual_seed(rows + cols)
    x = torch.randn(rows, cols).to(BF)
    s = K_.colsum(x.to(cuda))
    want = x.float().sum(0)
    assert rel_err(s.float().cpu().numpy(), want.numpy()) < 8e-3 or rows == 0
    if rows == 0:
        assert s.float().abs().max().item() == 0
    prev = torch.randn(cols).to(BF)
    acc = prev.to(cuda)
    K_.colsum(x.to(cuda), out=acc, accumulate=True)
    assert rel_err(acc.float().cpu().numpy(), (want + prev.float()).numpy()) < 8e-3


def test_colsum_dropout_gate(cuda):
    K_ = _k()
    torch.manual_seed(11)
    x = torch.randn(1000, 96).to(BF)
    s = K_.colsum(x.to(cuda))
    assert rel_err(s.float().cpu().numpy(), x.float().sum(0).numpy()) < 8e-3
    p, seed = 0.1, 77
    d = K_.dropout_mask_apply(x.to(cuda), p, seed)
    keep = torch.from_numpy(keep_mask(seed, np.arange(x.numel()), p).reshape(x.shape))
    want = torch.where(keep, x.float() / (1 - p), torch.zeros_like(x.float()))
    assert rel_err(d.float().cpu().numpy(), want.numpy()) < 8e-3
    y = torch.randn(1000, 96).to(BF)
    gate = torch.tensor(0.3).to(BF)
    acc = torch.zeros(1, device=cuda)
    dy = K_.gate_bwd(x.to(cuda), y.to(cuda), gate.to(cuda), acc)
    t = math.tanh(float(gate.float()))
    assert rel_err(dy.float().cpu().numpy(), (t * x.float()).numpy()) < 8e-3
    want_g = (x.float() * y.float()).sum().item() * (1 - t * t)
    assert abs(acc.item() - want_g) / abs(want_g) < 1e-3
    # 96 columns take the 8-wide kernels (round 5); 45 (and 37 x 45 elements) the scalar ones
    x2, y2 = torch.randn(37, 45).to(BF), torch.randn(37, 45).to(BF)
    d2 = K_.dropout_mask_apply(x2.to(cuda), p, seed)
    keep2 = torch.from_numpy(keep_mask(seed, np.arange(x2.numel()), p).reshape(x2.shape))
    want2 = torch.where(keep2, x2.float() / (1 - p), torch.zeros_like(x2.float()))
    assert rel_err(d2.float().cpu().numpy(), want2.numpy()) < 8e-3
    acc2 = torch.zeros(1, device=cuda)
    dy2 = K_.gate_bwd(x2.to(cuda), y2.to(cuda), gate.to(cuda), acc2)
    assert rel_err(dy2.float().cpu().numpy(), (t * x2.float()).numpy()) < 8e-3
    want_g2 = (x2.float() * y2.float()).sum().item() * (1 - t * t)
    assert abs(acc2.item() - want_g2) / abs(want_g2) < 1e-3
    # ABI v13: the gate gradient added into a bf16 scalar grad with autograd's roundings
    for xx, yy, wg in ((x, y, want_g), (x2, y2, want_g2)):
        gb = torch.tensor(0.75).to(BF).to(cuda)
        dyb = K_.gate_bwd(xx.to(cuda), yy.to(cuda), gate.to(cuda), grad_bf16=gb)
        assert torch.equal(dyb.cpu(), K_.gate_bwd(xx.to(cuda), yy.to(cuda), gate.to(cuda),
                                                  torch.zeros(1, device=cuda)).cpu())
        want_b = (torch.tensor(0.75).to(BF).float() + torch.tensor(wg).to(BF).float()).to(BF)
        assert abs(gb.float().item() - want_b.float().item()) <= 2 ** -7 * abs(want_b.float().item())


@pytest.mark.parametrize("M,N,K", [(4096, 4096, 1024), (2056, 3072, 1024), (300, 136, 72)])
def test_gemm_bias_quick_gelu(cuda, M, N, K):
    """act 5 (ABI v14): C = quick_gelu(A W^T + b) = h * sigmoid(1.702 h), the frozen CLIP tower's
    fc1 (transformers QuickGELUActivation) on the gvl-native feature stage — the persistent
    kernel's compile-time epilogue (EPI_BIAS_QGELU) on the wide shapes, the generic epilogue on a
    ragged small one; quick-GELU with a pre-activation output is refused."""
    K_ = _k()
    torch.manual_seed(M + N + K)
    x = torch.randn(M, K).to(BF)
    w = (torch.randn(N, K) * 0.05).to(BF)
    bias = torch.randn(N).to(BF)
    A, B = x.to(cuda), w.to(cuda)
    name = _kernel_name(A, B, 0, 0, M, N, K, epi="qgelu")
    y = K_.gemm(A, B, bias=bias.to(cuda), act=5)
    torch.cuda.synchronize()
    h = x.float() @ w.float().t() + bias.float()
    ref = h * torch.sigmoid(1.702 * h)
    print(name)
    if M == 4096:  # (2056 rows: too few tiles for the persistent kernel, the ring's generic epilogue)
        assert name.startswith("gemm_pp3_kernel") and ", 14, " in name, name
    assert rel_err(y.float().cpu().numpy(), ref.numpy()) < 8e-3
    with pytest.raises(RuntimeError):
        K_.gemm(A, B, bias=bias.to(cuda), act=5, pre_out=torch.empty(M, N, dtype=BF, device=cuda))
