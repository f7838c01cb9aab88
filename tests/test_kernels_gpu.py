"""Per-kernel parity of the HIP library (via the C ABI) against plain fp32 references.

Tolerances (stated per test) follow from bf16/fp16 storage: the kernels accumulate in fp32 and round
once on store, so the relative L2 error vs an fp32 reference computed from the *same* rounded inputs
is ~2^-9 (bf16) / 2^-12 (fp16) per stored value.
"""
import math
import os

import numpy as np
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






TOL = {torch.bfloat16: 6e-3, torch.float16: 1.5e-3}


def rnd(*shape, dtype=torch.bfloat16, scale=1.0):
    return (torch.randn(*shape, device=DEV) * scale).to(dtype)


# ------------------------------------------------------------------------------------------ GEMM
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("M,N,K", [(8192, 640, 640), (2048, 1280, 1280), (2048, 3840, 1280), (77, 1280, 2048),
                                   (2, 1280, 320), (300, 200, 128), (32768, 320, 640), (1000, 4, 2880),
                                   (8192, 32, 1152), (5000, 24, 640)])
def test_gemm_plain(dtype, M, N, K):
    from fdhip import ops
    a, w = rnd(M, K, dtype=dtype), rnd(N, K, dtype=dtype, scale=K ** -0.5)
    b = torch.randn(N, device=DEV)
    out = ops.gemm(a, w, bias=b)
    ref = a.float() @ w.float().T + b
    assert rel_l2(out, ref) < TOL[dtype], rel_l2(out, ref)


@pytest.mark.parametrize("M", [1, 2, 3, 4])
@pytest.mark.parametrize("N,K", [(1280, 320), (13760, 1280), (1282, 2816)])
@pytest.mark.parametrize("odt", [torch.float32, torch.bfloat16])
def test_gemm_few_rows_gemv(M, N, K, odt):
    """M <= 4 (time / add-embedding MLPs at the CFG pair, time_emb_proj, text projection): the weight-streaming
    GEMV path of fd_gemm, with alpha, bias, SiLU and a residual in its epilogue; N not a multiple of 4 included."""
    from fdhip import ops
    a, w = rnd(M, K), rnd(N, K, scale=K ** -0.5)
    bias = torch.randn(N, device=DEV)
    res = torch.randn(M, N, device=DEV).to(odt)
    out = torch.empty(M, N, device=DEV, dtype=odt)
    ops.gemm(a, w, bias=bias, residual=res, act="silu", alpha=0.5, out=out)
    ref = F.silu(0.5 * (a.float() @ w.float().T) + bias) + res.float()
    assert rel_l2(out, ref) < (6e-3 if odt == torch.bfloat16 else 1e-5), rel_l2(out, ref)


def test_gemm_few_rows_batched_tiles_bitwise():
    """The GEMV is chosen by the per-tile row count (m_ref = CFG pair = 2): 13 tiles batched into one launch (M = 26,
    as C3's tile batches) give every row bitwise what one tile's launch gives."""
    from fdhip import ops
    K, N = 1280, 13760
    a, w = rnd(26, K), rnd(N, K, scale=K ** -0.5)
    bias = torch.randn(N, device=DEV)
    with ops.tile_groups(13):
        big = ops.gemm(a, w, bias=bias, act="silu", out_dtype=torch.float32)
    for t in (0, 5, 12):
        one = ops.gemm(a[2 * t:2 * t + 2].contiguous(), w, bias=bias, act="silu", out_dtype=torch.float32)
        assert torch.equal(big[2 * t:2 * t + 2], one)


@pytest.mark.parametrize("act", ["silu", "gelu", "quickgelu"])
def test_gemm_act_residual_rowbias(act):
    from fdhip import ops
    M, N, K = 1024, 640, 1280
    a, w = rnd(M, K), rnd(N, K, scale=K ** -0.5)
    bias = torch.randn(N, device=DEV)
    res = rnd(M, N)
    rowb = torch.randn(4, N, device=DEV)
    out = ops.gemm(a, w, bias=bias, residual=res, rowbias=rowb, rows_per_group=M // 4, act=act)
    v = a.float() @ w.float().T + bias + rowb.repeat_interleave(M // 4, 0)
    v = {"silu": F.silu, "gelu": F.gelu, "quickgelu": lambda x: x * torch.sigmoid(1.702 * x)}[act](v)
    ref = v + res.float()
    assert rel_l2(out, ref) < 6e-3


def test_gemm_geglu_packed():
    from fdhip import ops
    M, C, Fd = 2048, 640, 2560
    x = rnd(M, C)
    w = rnd(2 * Fd, C, scale=C ** -0.5)
    b = torch.randn(2 * Fd, device=DEV) * 0.1
    wp, bp = ops.pack_geglu(w, b)
    out = ops.gemm(x, wp, bias=bp, act="geglu")
    assert out.shape == (M, Fd)
    h, g = (x.float() @ w.float().T + b).chunk(2, dim=-1)
    ref = h * F.gelu(g)
    assert rel_l2(out, ref) < 6e-3


def test_gemm_batched_strided_f32_out():
    from fdhip import ops
    B, T, D = 2, 1000, 512
    q, k = rnd(B, T, D, dtype=torch.float16), rnd(B, T, D, dtype=torch.float16)
    s = ops.gemm(q, k, batch=B, M=T, N=T, K=D, stride_a=T * D, stride_w=T * D, stride_c=T * T, alpha=D ** -0.5,
                 out_dtype=torch.float32)
    ref = torch.einsum("btd,bsd->bts", q.float(), k.float()) * D ** -0.5
    assert rel_l2(s, ref) < 1e-5 * 100


# ------------------------------------------------------------------------------------------ conv
def conv_ref(x_nhwc, w, b, nimg, H, W, stride, pad, upsample=False, vae_pad=False):
    x = x_nhwc.float().reshape(nimg, H, W, -1).permute(0, 3, 1, 2)
    if upsample:
        x = F.interpolate(x, scale_factor=2.0, mode="nearest")
    if vae_pad:
        x = F.pad(x, (0, 1, 0, 1))
    y = F.conv2d(x, w.float(), b, stride=stride, padding=pad)
    return y.permute(0, 2, 3, 1).reshape(-1, w.shape[0])


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("nimg,H,W,Cin,Cout,stride,pad,up", [
    (2, 128, 128, 320, 320, 1, 1, False), (2, 32, 32, 1280, 1280, 1, 1, False), (2, 64, 64, 640, 640, 2, 1, False),
    (1, 33, 47, 128, 256, 1, 1, False), (1, 64, 64, 128, 128, 2, 0, False), (2, 32, 32, 1280, 1280, 1, 1, True),
    (1, 40, 24, 256, 3, 1, 1, False), (2, 16, 16, 320, 4, 1, 1, False),
    # Cout <= 8: the narrow conv kernel (VAE conv_out 128 -> 3, encoder 512 -> 8)
    (1, 256, 192, 128, 3, 1, 1, False), (2, 33, 17, 512, 8, 1, 1, False), (1, 64, 64, 128, 6, 2, 0, False),
    (1, 31, 29, 64, 1, 2, 1, False)])
def test_conv3x3(dtype, nimg, H, W, Cin, Cout, stride, pad, up):
    from fdhip import ops
    x = rnd(nimg * H * W, Cin, dtype=dtype)
    w = (torch.randn(Cout, Cin, 3, 3, device=DEV) / math.sqrt(9 * Cin)).to(dtype)
    b = torch.randn(Cout, device=DEV) * 0.1
    out = ops.conv3x3(x, ops.pack_conv3x3(w), b, nimg, H, W, stride=stride, pad=pad, upsample=up)
    ref = conv_ref(x, w, b, nimg, H, W, stride, pad, up, vae_pad=(stride == 2 and pad == 0))
    assert out.shape == ref.shape
    assert rel_l2(out, ref) < TOL[dtype], rel_l2(out, ref)


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("nimg,H,W,Cin,Cout", [(1, 1024, 1024, 128, 3), (2, 37, 100, 128, 3), (1, 64, 64, 32, 4),
                                               (1, 17, 130, 64, 1), (2, 8, 8, 128, 2)])
def test_conv3x3_narrow(dtype, nimg, H, W, Cin, Cout):
    """fd_conv3x3_narrow (the VAE decoder's conv_out, 128 -> 3 at 1024^2) vs torch conv2d in fp32 on the same
    values, incl. row tails (W % 64 != 0) and image borders; and vs the implicit-GEMM conv it replaces."""
    from fdhip import ops
    x = rnd(nimg * H * W, Cin, dtype=dtype)
    w = torch.randn(Cout, Cin, 3, 3, device=DEV) / math.sqrt(9 * Cin)
    b = torch.randn(Cout, device=DEV) * 0.1
    out = ops.conv3x3_narrow(x, ops.pack_conv3x3(w).float(), b, nimg, H, W)
    ref = conv_ref(x, w, b, nimg, H, W, 1, 1)
    assert out.dtype == dtype and out.shape == (nimg * H * W, Cout)
    assert rel_l2(out, ref) < TOL[dtype]
    if Cin % 64 == 0:  # the implicit-GEMM conv needs Cin % 64 == 0
        gemm = ops.conv3x3(x, ops.pack_conv3x3(w.to(dtype)), b, nimg, H, W)
        assert rel_l2(out, gemm) < 2 * TOL[dtype]
    # the decoder's conv_norm_out + SiLU folded into the staging (fd_conv3x3_narrow_gn): bitwise the same conv of
    # fd_group_norm's stored output (the staged values are those bits, the summation order is unchanged)
    if Cin >= 32:
        gamma = 1 + 0.1 * torch.randn(Cin, device=DEV)
        beta = 0.1 * torch.randn(Cin, device=DEV)
        aff = ops.group_norm_affine(x, gamma, beta, nimg, H * W, Cin, 32, 1e-6)
        fused = ops.conv3x3_narrow(x, ops.pack_conv3x3(w).float(), b, nimg, H, W, gn_in=(aff, True))
        hn = ops.group_norm(x, gamma, beta, nimg, H * W, Cin, 32, 1e-6, silu=True)
        plain = ops.conv3x3_narrow(hn, ops.pack_conv3x3(w).float(), b, nimg, H, W)
        torch.cuda.synchronize()
        assert torch.equal(fused, plain)


def test_conv3x3_concat_temb_residual():
    from fdhip import ops
    nimg, H, W, C1, C2, Cout = 2, 32, 32, 1280, 640, 1280
    x1, x2 = rnd(nimg * H * W, C1), rnd(nimg * H * W, C2)
    w = (torch.randn(Cout, C1 + C2, 3, 3, device=DEV) / math.sqrt(9 * (C1 + C2))).to(torch.bfloat16)
    b = torch.randn(Cout, device=DEV) * 0.1
    temb = torch.randn(nimg, Cout, device=DEV)
    res = rnd(nimg * H * W, Cout)
    out = ops.conv3x3(x1, ops.pack_conv3x3(w), b, nimg, H, W, x2=x2, C1=C1, rowbias=temb, residual=res)
    ref = conv_ref(torch.cat([x1, x2], 1), w, b, nimg, H, W, 1, 1) + temb.repeat_interleave(H * W, 0) + res.float()
    assert rel_l2(out, ref) < 6e-3


@pytest.mark.parametrize("Cin,Cout,k", [(4, 320, 3), (3, 128, 3), (8, 8, 1), (4, 512, 3)])
def test_conv_direct(Cin, Cout, k):
    from fdhip import ops
    nimg, H, W = 2, 37, 29
    x = rnd(nimg * H * W, Cin, dtype=torch.float16)
    w = torch.randn(Cout, Cin, k, k, device=DEV) / math.sqrt(k * k * Cin)
    b = torch.randn(Cout, device=DEV)
    out = ops.conv_direct(x, w.permute(0, 2, 3, 1).contiguous(), b, nimg, H, W, Cin, ksize=k, pad=k // 2,
                          out_dtype=torch.float32)
    ref = conv_ref(x, w, b, nimg, H, W, 1, k // 2)
    assert rel_l2(out, ref) < 1e-5


# ------------------------------------------------------------------------------------------ norms
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("nimg,HW,C", [(2, 16384, 320), (2, 4096, 640), (2, 1024, 2560), (2, 1024, 1920),
                                       (1, 65536, 128), (1, 16384, 512), (2, 4096, 960), (1, 100, 256)])
@pytest.mark.parametrize("silu", [False, True])
def test_group_norm(dtype, nimg, HW, C, silu):
    from fdhip import ops
    x = (torch.randn(nimg * HW, C, device=DEV) * 2 + 0.5).to(dtype)
    g, b = torch.rand(C, device=DEV) + 0.5, torch.randn(C, device=DEV) * 0.1
    out = ops.group_norm(x, g, b, nimg, HW, C, 32, 1e-5, silu)
    xr = x.float().reshape(nimg, HW, C).permute(0, 2, 1)
    ref = F.group_norm(xr, 32, g, b, 1e-5)
    if silu:
        ref = F.silu(ref)
    ref = ref.permute(0, 2, 1).reshape(-1, C)
    assert rel_l2(out, ref) < TOL[dtype]


def test_group_norm_deterministic():
    from fdhip import ops
    x = rnd(2 * 4096, 640)
    g, b = torch.ones(640, device=DEV), torch.zeros(640, device=DEV)
    a1 = ops.group_norm(x, g, b, 2, 4096, 640)
    a2 = ops.group_norm(x, g, b, 2, 4096, 640)
    assert torch.equal(a1, a2)


@pytest.mark.parametrize("C", [640, 1280])
def test_layer_norm(C):
    from fdhip import ops
    x = rnd(4099, C)
    g, b = torch.rand(C, device=DEV) + 0.5, torch.randn(C, device=DEV) * 0.1
    out = ops.layer_norm(x, g, b, 1e-5)
    ref = F.layer_norm(x.float(), (C,), g, b, 1e-5)
    assert rel_l2(out, ref) < 6e-3


# ------------------------------------------------------------------------------------------ attention
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("B,heads,Lq,Lk,kv_mod", [(2, 10, 4096, 4096, 0), (2, 20, 1024, 1024, 0), (4, 10, 4096, 77, 2),
                                                  (1, 3, 200, 333, 0), (2, 20, 1024, 77, 2)])
def test_flash_attn(dtype, B, heads, Lq, Lk, kv_mod):
    from fdhip import ops
    C = heads * 64
    q = rnd(B, Lq, C, dtype=dtype)
    nkv = kv_mod if kv_mod else B
    kv = rnd(nkv, Lk, 2 * C, dtype=dtype)
    k, v = kv[..., :C], kv[..., C:]
    o = torch.empty(B, Lq, C, dtype=dtype, device=DEV)
    ops.flash_attn(q, k, v, o, B, heads, Lq, Lk, C, 2 * C, 2 * C, C, Lq * C, Lk * 2 * C, Lk * 2 * C, Lq * C,
                   kv_mod=kv_mod, scale=0.125)
    idx = torch.arange(B, device=DEV) % nkv
    qh = q.float().view(B, Lq, heads, 64).transpose(1, 2)
    kh = k.float()[idx].reshape(B, Lk, heads, 64).transpose(1, 2)
    vh = v.float()[idx].reshape(B, Lk, heads, 64).transpose(1, 2)
    ref = F.scaled_dot_product_attention(qh, kh, vh).transpose(1, 2).reshape(B, Lq, C)
    assert rel_l2(o, ref) < 1.5 * TOL[dtype], rel_l2(o, ref)


@pytest.mark.parametrize("Lk", [1024, 77])
def test_flash_attn_query_split_bitwise(Lk):
    """A 2-image launch (16 queries per wave) and the same images inside a 26-image launch (32 per wave, the
    CFG-batched TLC tiles of C3) give the same bits: the kernel form is chosen by launch size."""
    from fdhip import ops
    B, heads, Lq = 26, 20, 1024
    C = heads * 64
    q = rnd(B, Lq, C)
    kv = rnd(B, Lk, 2 * C)
    k, v = kv[..., :C], kv[..., C:]
    big = torch.empty(B, Lq, C, dtype=torch.bfloat16, device=DEV)
    ops.flash_attn(q, k, v, big, B, heads, Lq, Lk, C, 2 * C, 2 * C, C, Lq * C, Lk * 2 * C, Lk * 2 * C, Lq * C,
                   kv_mod=0, scale=0.125)
    for b0 in (0, 12, 24):
        small = torch.empty(2, Lq, C, dtype=torch.bfloat16, device=DEV)
        ops.flash_attn(q[b0:b0 + 2], k[b0:b0 + 2], v[b0:b0 + 2], small, 2, heads, Lq, Lk, C, 2 * C, 2 * C, C,
                       Lq * C, Lk * 2 * C, Lk * 2 * C, Lq * C, kv_mod=0, scale=0.125)
        assert torch.equal(small, big[b0:b0 + 2])


@pytest.mark.parametrize("same", [True, False])
def test_mha_seq_axis(same):
    from fdhip import ops
    G, Lx, N, E, H = 3, 2, 500, 640, 8
    qkv = rnd(G * Lx, N, 3 * E)
    if same:
        qkv.view(G, Lx, N, 3 * E)[:, 1] = qkv.view(G, Lx, N, 3 * E)[:, 0]
    o = torch.empty(G * Lx, N, E, dtype=torch.bfloat16, device=DEV)
    ops.mha_seq_axis(qkv, o, Lx, G, N, E, H)
    x = qkv.float().view(G, Lx, N, 3, H, E // H)
    q, k, v = x[:, :, :, 0], x[:, :, :, 1], x[:, :, :, 2]  # G, L, N, H, d
    s = torch.einsum("glnhd,gmnhd->gnhlm", q, k) / math.sqrt(E // H)
    p = s.softmax(-1)
    ref = torch.einsum("gnhlm,gmnhd->glnhd", p, v).reshape(G * Lx, N, E)
    assert rel_l2(o, ref) < 6e-3
    if same:
        torch.testing.assert_close(o.float(), v[:, :1].expand(G, Lx, N, H, E // H).reshape(G * Lx, N, E),
                                   rtol=1e-2, atol=2e-2)


def test_softmax_rows():
    from fdhip import ops
    R, C = 333, 16384
    s = torch.randn(R, C, device=DEV) * 3
    p = torch.empty(R, C, dtype=torch.float16, device=DEV)
    ops.softmax_rows(s, p, R, C, 0.5)
    ref = (s * 0.5).softmax(-1)
    assert rel_l2(p, ref) < 2e-3


# ------------------------------------------------------------------------------------------ elementwise / loop
def test_layouts_concat_time_features():
    from fdhip import ops
    from oracle.unet import timestep_embedding
    x = torch.randn(2, 4, 37 * 29, device=DEV)
    y = torch.empty(2, 37 * 29, 4, dtype=torch.bfloat16, device=DEV)
    ops.nchw_to_nhwc(x, y, 2, 4, 37 * 29, 0.5)
    assert torch.equal(y, (x * 0.5).transpose(1, 2).to(torch.bfloat16))
    z = torch.empty(2, 4, 37 * 29, device=DEV)
    ops.nhwc_to_nchw(y, z, 2, 4, 37 * 29, 2.0)
    torch.testing.assert_close(z, (y.float() * 2).transpose(1, 2))
    a, b = rnd(1000, 320), rnd(1000, 640)
    c = torch.empty(1000, 960, dtype=torch.bfloat16, device=DEV)
    ops.concat_channels(a, 320, b, 640, c, 1000)
    assert torch.equal(c, torch.cat([a, b], 1))
    t = torch.tensor([951.0, 951.0], device=DEV)
    tid = torch.tensor([[1024, 1024, 0, 64, 1024, 1024]] * 2, dtype=torch.float32, device=DEV)
    text = torch.randn(2, 1280, device=DEV)
    tf = torch.empty(2, 320, device=DEV)
    af = torch.empty(2, 2816, device=DEV)
    ops.time_features(t, tid, text, tf, af, 2)
    torch.testing.assert_close(tf.cpu(), timestep_embedding(t.cpu(), 320), rtol=1e-4, atol=2e-4)
    ref_a = torch.cat([text.cpu(), timestep_embedding(tid.cpu().flatten(), 256).reshape(2, -1)], -1)
    torch.testing.assert_close(af.cpu(), ref_a, rtol=1e-4, atol=2e-4)


def test_tlc_blend_bitexact_vs_reference_golden(golden):
    """fd_tlc_blend reproduces the reference's grids_inverse bit for bit (golden from the reference)."""
    from fdhip import ops
    from _det import det_tensor
    from oracle import tlc
    for h, w in [(64, 64), (128, 128), (128, 192), (200, 136)]:
        idx, (k1, k2) = tlc.tile_origins(h, w, (128, 128), 0.5)
        rows = sorted({i for i, _ in idx})
        cols = sorted({j for _, j in idx})
        assert idx == [(r, c) for r in rows for c in cols]
        x = det_tensor((1, 4, h, w), 1000 + h * 7 + w)
        tiles = torch.cat([x[:, :, i:i + k1, j:j + k2] for i, j in idx], 0)
        outs = tiles * (1.0 + 0.01 * torch.arange(tiles.shape[0]).view(-1, 1, 1, 1)) + 0.05
        wts = tlc.gaussian_weights(k2, k1)[0].contiguous()
        canvas = torch.empty(4, h, w, device=DEV)
        ops.tlc_blend(outs.to(DEV).contiguous(), wts.to(DEV), torch.tensor(rows, dtype=torch.int32, device=DEV),
                      torch.tensor(cols, dtype=torch.int32, device=DEV), 4, h, w, k1, k2, canvas)
        np.testing.assert_array_equal(canvas.cpu().numpy()[None], golden[f"tlc_{h}x{w}_inv"])


def test_tlc_scale_input_and_euler_step():
    from fdhip import ops
    from oracle import schedulers as S
    H, W, k = 200, 136, 128
    canvas = torch.randn(4, H, W, device=DEV) * 5
    rows = torch.tensor([0, 64, 72], dtype=torch.int32, device=DEV)
    cols = torch.tensor([0, 8], dtype=torch.int32, device=DEV)
    nt = 6
    sig, sig_n, g = 11.02834, 10.1, 5.0
    xin = torch.empty(nt * 2, k * k, 4, dtype=torch.bfloat16, device=DEV)
    ops.tlc_scale_input(canvas, rows, cols, H, W, k, k, 0, nt, 2, sig, xin)
    tiles = torch.stack([canvas[:, r:r + k, c:c + k] for r in rows.tolist() for c in cols.tolist()])
    # reference on the host: tensor / tensor true division (a device tensor / python scalar multiplies by the
    # reciprocal, which is not what scale_model_input computes)
    ref_in = (tiles.cpu() / ((torch.tensor(sig) ** 2 + 1) ** 0.5)).permute(0, 2, 3, 1).reshape(nt, k * k, 4).to(DEV)
    assert torch.equal(xin.view(nt, 2, k * k, 4)[:, 0], ref_in.to(torch.bfloat16))
    assert torch.equal(xin.view(nt, 2, k * k, 4)[:, 1], ref_in.to(torch.bfloat16))
    eps = rnd(nt * 2, k * k, 4)
    out = torch.empty(nt, 4, k, k, device=DEV)
    ops.tlc_cfg_euler_step(eps, canvas, rows, cols, H, W, k, k, 0, nt, 2, g, 0.0, sig, sig_n, out)
    e = eps.float().view(nt, 2, k, k, 4).permute(0, 1, 4, 2, 3)
    ec = e[:, 0] + g * (e[:, 1] - e[:, 0])
    ref = S.euler_step(ec, tiles, sig, sig_n)
    torch.testing.assert_close(out, ref, rtol=1e-5, atol=1e-4)
    # guidance_rescale > 0 path (rescale_noise_cfg)
    from oracle.pipeline import rescale_noise_cfg
    out2 = torch.empty_like(out)
    ops.tlc_cfg_euler_step(eps, canvas, rows, cols, H, W, k, k, 0, nt, 2, g, 0.7, sig, sig_n, out2)
    ref2 = torch.stack([S.euler_step(rescale_noise_cfg(ec[i:i + 1], e[i:i + 1, 1], 0.7)[0], tiles[i], sig, sig_n)
                        for i in range(nt)])
    torch.testing.assert_close(out2, ref2, rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("t_n", [2, 256, 600])
def test_tlc_scale_input_writes_every_timestep_row(t_n):
    """fd_tlc_scale_input_t fills t_out[0 .. t_n) from the same launch for any t_n (only block 0 wrote it,
    so more than 256 UNet rows -- FD_TILE_BATCH > 128 with CFG -- were refused); the tiles equal the plain launch's."""
    from fdhip import ops
    H, W, k, nt = 200, 136, 64, 6
    canvas = torch.randn(4, H, W, device=DEV) * 5
    rows = torch.tensor([0, 64, 136], dtype=torch.int32, device=DEV)
    cols = torch.tensor([0, 72], dtype=torch.int32, device=DEV)
    a = torch.empty(nt * 2, k * k, 4, dtype=torch.bfloat16, device=DEV)
    b = torch.empty_like(a)
    t_out = torch.full((t_n,), -1.0, device=DEV)
    ops.tlc_scale_input(canvas, rows, cols, H, W, k, k, 0, nt, 2, 11.0, a)
    ops.tlc_scale_input(canvas, rows, cols, H, W, k, k, 0, nt, 2, 11.0, b, t_out=t_out, timestep=961.0)
    torch.cuda.synchronize()
    assert torch.equal(a, b)
    assert bool((t_out == 961.0).all())


def test_tlc_grids_nhwc():
    from fdhip import ops
    H, W, C, k = 200, 136, 512, 128
    canvas = rnd(H * W, C, dtype=torch.float16)
    rows = torch.tensor([0, 64, 72], dtype=torch.int32, device=DEV)
    cols = torch.tensor([0, 8], dtype=torch.int32, device=DEV)
    out = torch.empty(2 * 2, k, k, C, dtype=torch.float16, device=DEV)
    ops.tlc_grids_nhwc(canvas, rows, cols, H, W, C, k, k, 3, 2, 2, out)
    cv = canvas.view(H, W, C)
    for t, tid in enumerate([3, 4]):
        r, c = rows[tid // 2].item(), cols[tid % 2].item()
        assert torch.equal(out[2 * t], cv[r:r + k, c:c + k])
        assert torch.equal(out[2 * t + 1], cv[r:r + k, c:c + k])


def _d512_ref(qkv, n, T, C=512):
    x = qkv.float()
    q, k, v = x[..., :C], x[..., C:2 * C], x[..., 2 * C:]
    return F.scaled_dot_product_attention(q[:, None], k[:, None], v[:, None])[:, 0].reshape(n * T, C)


@pytest.mark.parametrize("split", [False, True])
@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("n,T", [(1, 4096), (2, 1000), (1, 77), (1, 16384)])
def test_flash_attn_d512(dtype, n, T, split):
    """fd_flash_attn_d512 (the VAE mid-block attention, one head of 512 channels; split: the 8-wave split-key form
    fd_flash_attn_d512_split at the planned ks) against fp32 SDPA on the same qkv projection rows [q | k | v]
    (ld 1536), incl. ragged tails (T = 1000, 77) and the 1024^2 size (16384)."""
    from fdhip import ops
    C = 512
    scale = 1.0 if T > 4096 else 2.0  # score spread: keep the softmax peaked enough to be a real test
    qkv = (rnd(n, T, 3 * C, dtype=torch.float32) * scale).to(dtype)
    o = torch.empty(n * T, C, dtype=dtype, device=DEV)
    ops.flash_attn_d512(qkv.view(n * T, 3 * C), o, n, T, split=split)
    assert rel_l2(o, _d512_ref(qkv, n, T)) < 1.5 * TOL[dtype], rel_l2(o, _d512_ref(qkv, n, T))


@pytest.mark.parametrize("ks", [1, 2, 3, 5, 64])
def test_flash_attn_d512_key_splits(ks):
    """Every split count through the C ABI, incl. splits with no key tile (T = 300: 10 tiles, ks = 64 leaves most
    splits empty: log2-sum-exp -inf, weight 0 in the merge), against fp32 SDPA; an undersized scratch is refused."""
    from fdhip import lib as L
    n, T, C = 2, 300, 512
    qkv = (rnd(n, T, 3 * C, dtype=torch.float32) * 2.0).to(torch.float16)
    o = torch.empty(n * T, C, dtype=torch.float16, device=DEV)
    nfl = n * ks * T * 513
    part = torch.empty(max(nfl, 4), dtype=torch.float32, device=DEV)
    args = lambda nf: (L.ptr(qkv), L.ptr(qkv[..., 512:]), L.ptr(qkv[..., 1024:]), 3 * C, T * 3 * C, L.ptr(o), C,
                       T * C, n, T, C ** -0.5, L.dtype_code(qkv.dtype), L.ptr(part), nf, ks, L.stream())
    L.check(L.load().fd_flash_attn_d512_split(*args(nfl)), "fd_flash_attn_d512_split")
    torch.cuda.synchronize()
    assert rel_l2(o, _d512_ref(qkv, n, T)) < 1.5 * TOL[torch.float16]
    if ks > 1:
        assert L.load().fd_flash_attn_d512_split(*args(nfl - 1)) == -1  # FD_ERR_SHAPE
    assert 1 <= L.load().fd_flash_attn_d512_ksplit(1, 16384) <= 8


@pytest.mark.parametrize("nimg,H,W,Cin,Cout,up,expect", [
    (1, 128, 128, 256, 512, False, True),   # gemm8 256x128 (the 512-ch VAE level), cpg 16
    (1, 128, 128, 128, 256, True, True),    # gemm256 upsample conv (256^2 out), cpg 8
    (2, 128, 128, 128, 256, False, True),   # gemm256, two images
    (1, 256, 256, 128, 128, False, True),   # gemm8 256x128, cpg 4 (chunks straddle groups)
    (1, 512, 512, 128, 128, False, True),   # 128-channel conv on a 512^2 image
    (1, 1024, 1024, 128, 128, False, True),  # the VAE decoder's 1024^2 level: 4096 partial blocks (wide finalize)
    (2, 128, 128, 320, 320, False, True),   # gemm8 256x160 (the UNet's 128^2 level), cpg 10
    (2, 64, 64, 640, 640, False, None),     # the 64^2 level, cpg 20 (256x160 when the planner takes it)
    (2, 16, 16, 320, 320, False, None),     # small M: whichever tile the planner picks
    (1, 24, 20, 128, 128, False, False)])   # H*W % 256 != 0
def test_conv_groupnorm_statistics_from_epilogue(nimg, H, W, Cin, Cout, up, expect):
    """A conv asked for its output's GroupNorm statistics (ops.GnStats -> fd_gemm_params.gn_part) + group_norm
    from them (fd_group_norm_partials) == group_norm computing its own statistics, up to the summation order.
    expect None: either way (the planner's tile choice), the result must match."""
    from fdhip import ops
    dt = torch.bfloat16 if Cout % 320 == 0 else torch.float16  # the UNet's (bf16) and the VAE's (fp16) convs
    x = rnd(nimg * H * W, Cin, dtype=dt)
    w = (torch.randn(Cout, Cin, 3, 3, device=DEV) / math.sqrt(9 * Cin)).to(dt)
    b = torch.randn(Cout, device=DEV) * 0.3
    res = rnd(nimg * H * W * (4 if up else 1), Cout, dtype=dt)
    Ho, Wo = (2 * H, 2 * W) if up else (H, W)
    st = ops.GnStats(nimg, Ho * Wo, 32, DEV)
    wp = ops.pack_conv3x3(w)
    halo = ops.halo_conv_rows(x, wp, nimg, H, W, upsample=up)  # the halo-staged conv's block rows (256 / 128), or 0
    y = ops.conv3x3(x, wp, b, nimg, H, W, upsample=up, residual=res, gn=st)
    if expect is not None:
        assert st.done == expect
    if st.done:
        assert st.rows == (halo if halo else 256)
    g, be = torch.randn(Cout, device=DEV), torch.randn(Cout, device=DEV)
    got = ops.group_norm(y, g, be, nimg, Ho * Wo, Cout, 32, 1e-6, silu=True, stats=st)
    want = ops.group_norm(y, g, be, nimg, Ho * Wo, Cout, 32, 1e-6, silu=True)
    ref = F.silu(F.group_norm(y.float().view(nimg, Ho * Wo, Cout).permute(0, 2, 1), 32, g, be, 1e-6)).permute(0, 2, 1)
    assert rel_l2(got, want) < 2e-3
    assert rel_l2(got, ref.reshape(-1, Cout)) < 6e-3


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("nimg,HW,C,silu", [(2, 16384, 320, True), (2, 4096, 640, False), (2, 1024, 1280, True),
                                            (2, 1024, 2560, False), (1, 256, 64, True)])
def test_groupnorm_partials_fold_matches_affine_fold_bitwise(dtype, nimg, HW, C, silu):
    """fd_group_norm_partials' (mean, rstd) from the producer's partials -- written to the caller's stats by
    gn_finalize_kernel -- are bit for bit the fold of fd_group_norm_affine's fused finalize + affine launch (the same
    fp64 order): with gamma = 1, beta = 0 the affine is exactly (rstd, -mean * rstd).  The output is x * scale + shift
    (+ SiLU) of those statistics."""
    import ctypes

    from fdhip import lib as L
    from fdhip import ops
    x = rnd(nimg * HW, C, dtype=dtype)
    st = ops.GnStats(nimg, HW, 32, DEV)
    nblk = HW // 256
    xs = x.float().view(nimg, nblk, 256, 32, C // 32)
    part = torch.stack([xs.sum((2, 4)), (xs * xs).sum((2, 4))], -1)  # (sum, sumsq) per (image, block, group)
    part = part * (1 + 1e-3 * torch.randn_like(part))  # not exactly the data's: the fold, not the data, is tested
    st.part[:part.numel()] = part.reshape(-1)
    st.done, st.rows = True, 256
    one, zero = torch.ones(C, device=DEV), torch.zeros(C, device=DEV)
    y = torch.empty_like(x)
    stats = torch.zeros(nimg * 32 * 2, device=DEV)
    L.check(L.load().fd_group_norm_partials(L.ptr(x), L.ptr(y), L.ptr(one), L.ptr(zero), nimg, HW, C, 32, 1e-6,
                                            int(silu), L.ptr(st.part), 256, L.ptr(stats), L.dtype_code(dtype),
                                            L.stream()), "fd_group_norm_partials")
    aff = ops.group_norm_affine(x, one, zero, nimg, HW, C, 32, 1e-6, stats=st)[:nimg * C].view(nimg, C, 2)
    torch.cuda.synchronize()
    mean, rstd = stats.view(nimg, 32, 2).unbind(-1)
    cpg = C // 32
    assert torch.equal(aff[..., 0], rstd.repeat_interleave(cpg, 1))
    assert torch.equal(aff[..., 1], (-mean * rstd).repeat_interleave(cpg, 1))
    ref = x.double().view(nimg, HW, C) * aff[..., 0].double()[:, None] + aff[..., 1].double()[:, None]
    if silu:
        ref = ref * torch.sigmoid(ref)
    assert rel_l2(y.view(nimg, HW, C), ref) < 4e-3


@pytest.mark.parametrize("nimg,HW,C1,C2", [(2, 1024, 1280, 1280), (2, 1024, 1280, 640), (2, 4096, 1280, 640),
                                           (2, 4096, 640, 320), (2, 16384, 640, 320), (2, 16384, 320, 320),
                                           (1, 100, 64, 32), (1, 1001, 64, 32)])
def test_concat_with_groupnorm_statistics_bitwise(nimg, HW, C1, C2):
    """fd_concat_channels_gn: the up-block concat writes its GroupNorm consumer's statistics partials (fd_group_norm's
    own pass, fused into the copy).  The concat is torch.cat exactly; the GroupNorm (+ SiLU) and the halo conv's
    affine from those partials are bit for bit the ones computed from the concat by their own statistics pass.
    HW = 1001 is not a multiple of its chunk rows (4): no partials (done False), the plain concat."""
    from fdhip import lib as L
    from fdhip import ops
    a, b = rnd(nimg * HW, C1), rnd(nimg * HW, C2)
    C = C1 + C2
    st = ops.GnStats(nimg, HW, 32, DEV)
    out = torch.empty((nimg * HW, C), dtype=torch.bfloat16, device=DEV)
    ops.concat_channels(a, C1, b, C2, out, nimg * HW, gn=st)
    assert torch.equal(out, torch.cat([a, b], 1))
    assert st.done == (HW % L.load().fd_group_norm_chunk_rows(nimg, HW) == 0)
    if not st.done:
        return
    g, be = torch.randn(C, device=DEV), torch.randn(C, device=DEV)
    assert torch.equal(ops.group_norm(out, g, be, nimg, HW, C, 32, 1e-5, silu=True, stats=st),
                       ops.group_norm(out, g, be, nimg, HW, C, 32, 1e-5, silu=True))
    assert torch.equal(ops.group_norm_affine(out, g, be, nimg, HW, C, 32, 1e-5, stats=st),
                       ops.group_norm_affine(out, g, be, nimg, HW, C, 32, 1e-5))


@pytest.mark.parametrize("B,HW,C", [(2, 16384, 320), (2, 4096, 640), (4, 1024, 1280)])
def test_gemm_groupnorm_statistics_from_epilogue(B, HW, C):
    """The UNet's transformer proj_out (GEMM + residual) asked for its output's GroupNorm statistics: group_norm from
    them == group_norm computing its own (summation order aside), == torch GroupNorm."""
    from fdhip import ops
    x, res = rnd(B * HW, C), rnd(B * HW, C)
    w = (torch.randn(C, C, device=DEV) / math.sqrt(C)).to(torch.bfloat16)
    b = torch.randn(C, device=DEV) * 0.3
    st = ops.GnStats(B, HW, 32, DEV)
    y = ops.gemm(x, w, bias=b, residual=res, gn=st)
    g, be = torch.randn(C, device=DEV), torch.randn(C, device=DEV)
    got = ops.group_norm(y, g, be, B, HW, C, 32, 1e-6, stats=st)
    want = ops.group_norm(y, g, be, B, HW, C, 32, 1e-6)
    ref = F.group_norm(y.float().view(B, HW, C).permute(0, 2, 1), 32, g, be, 1e-6).permute(0, 2, 1)
    assert rel_l2(got, want) < 2e-3
    assert rel_l2(got, ref.reshape(-1, C)) < 6e-3
