"""LayerNorm folded across a GEMM pair (fd_gemm_params.ln_out / ln_in), through the C ABI.

The UNet's transformer blocks (diffusers BasicTransformerBlock: norm1 -> attn1 QKV, norm2 -> attn2 Q, norm3 ->
GEGLU) run the residual-stream GEMM as the producer of per-row (sum, sumsq) partials and the next
projection on the raw stream with W * gamma; reference here: torch LayerNorm (fp32) of the SAME bf16 stream,
then an fp32 matmul.  Tolerance rel-L2 < 1e-2 (bf16 W * gamma rounding + one bf16 output rounding).
Both consumer kernels are covered (8-wave 256-row tiles for QKV / GEGLU at M = 2048, the 4-wave kernel for
N = C and for small M), edge tiles (M not a multiple of 64), and the partials themselves.
"""
import pytest
import torch
import torch.nn.functional as F
from parity import rel_l2  # noqa: E402  (records every measured value)

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _dev():
    from fdhip import lib
    lib.require_device()
    torch.manual_seed(0)




def rnd(*shape, dtype=torch.bfloat16, scale=1.0):
    return (torch.randn(*shape, device=DEV) * scale).to(dtype)


def _producer(M, C, K0=640):
    """h = att @ Wo^T + bo + residual, with LN partials; returns (h, stats)."""
    from fdhip import ops
    att, wo = rnd(M, K0), rnd(C, K0, scale=K0 ** -0.5)
    bo = torch.randn(C, device=DEV) * 0.1
    # a residual stream with a row mean well away from zero (as in the UNet's hidden states)
    res = (torch.randn(M, C, device=DEV) * 2.0 + torch.randn(M, 1, device=DEV) * 3.0).to(torch.bfloat16)
    st = torch.full((M, C // 160, 2), float("nan"), device=DEV)
    h = ops.gemm(att, wo, bias=bo, residual=res, out=res.clone(), ln_out=st)
    return h, st


@pytest.mark.parametrize("M", [2048, 8192, 120])
@pytest.mark.parametrize("C", [640, 1280])
def test_partials(M, C):
    h, st = _producer(M, C)
    torch.cuda.synchronize()
    hf = h.float().view(M, C // 160, 160)
    ref = torch.stack([hf.sum(-1), (hf * hf).sum(-1)], -1)
    assert torch.isfinite(st).all()
    assert rel_l2(st, ref) < 1e-5, rel_l2(st, ref)


@pytest.mark.parametrize("M", [2048, 2000])
@pytest.mark.parametrize("C", [640, 1280])
def test_partials_long_k(M, C):
    """K >= 4096 (the ff out, 2048 x 1280 x 5120): the producer is the 8-wave family's 128 x 160 tile with K split
    in two (plan8); its epilogue writes the same per-160-column partials (M = 2000: a ragged last row tile)."""
    h, st = _producer(M, C, K0=5120)
    torch.cuda.synchronize()
    hf = h.float().view(M, C // 160, 160)
    ref = torch.stack([hf.sum(-1), (hf * hf).sum(-1)], -1)
    assert torch.isfinite(st).all()
    assert rel_l2(st, ref) < 1e-5, rel_l2(st, ref)


def test_long_k_producer_output_matches_torch():
    from fdhip import ops
    M, C, K0 = 2048, 1280, 5120
    att, wo = rnd(M, K0), rnd(C, K0, scale=K0 ** -0.5)
    bo = torch.randn(C, device=DEV) * 0.1
    res = rnd(M, C, scale=2.0)
    st = torch.zeros((M, C // 160, 2), device=DEV)
    h = ops.gemm(att, wo, bias=bo, residual=res, out=res.clone(), ln_out=st)
    y = att.float() @ wo.float().T + bo + res.float()
    assert rel_l2(h, y) < 6e-3, rel_l2(h, y)
    h2 = ops.gemm(att, wo, bias=bo, residual=res, out=res.clone())  # no partials: the 3-split 256 x 128 plan
    assert rel_l2(h2, y) < 6e-3, rel_l2(h2, y)


@pytest.mark.parametrize("M", [2048, 120])
@pytest.mark.parametrize("C", [640, 1280])
@pytest.mark.parametrize("K0", [640, 5120])
@pytest.mark.parametrize("kind", ["qkv", "q", "geglu"])
def test_consumer_matches_layer_norm_then_linear(M, C, K0, kind):
    from fdhip import ops
    h, st = _producer(M, C, K0)
    gamma = 1.0 + 0.2 * torch.randn(C, device=DEV)
    beta = 0.2 * torch.randn(C, device=DEV)
    n = {"qkv": 3 * C, "q": C, "geglu": 8 * C}[kind]
    w = rnd(n, C, scale=C ** -0.5)
    b = 0.1 * torch.randn(n, device=DEV) if kind == "geglu" else None
    wp, c, d = ops.fold_layer_norm(w, gamma, beta, b)
    out = ops.gemm(h, wp, bias=d, ln_in=st, ln_c=c, ln_eps=1e-5, act="geglu" if kind == "geglu" else "none")
    y = F.layer_norm(h.float(), (C,), gamma, beta, 1e-5) @ w.float().T
    if b is not None:
        y = y + b
    if kind == "geglu":  # rows packed [16 hidden | 16 gate] per 32 (ops.pack_geglu layout)
        yv = y.view(M, n // 32, 2, 16)
        y = (yv[:, :, 0] * F.gelu(yv[:, :, 1])).reshape(M, n // 2)
    assert rel_l2(out, y) < 1e-2, rel_l2(out, y)


def test_rejects_bad_shapes():
    from fdhip import ops
    st = torch.empty(256, 8, 2, device=DEV)
    with pytest.raises(RuntimeError):
        ops.gemm(rnd(256, 640), rnd(600, 640), ln_out=st)  # N % 160 != 0
    with pytest.raises(RuntimeError):
        ops.gemm(rnd(256, 576), rnd(640, 576), ln_in=st, ln_c=torch.zeros(640, device=DEV))  # K % 160 != 0
