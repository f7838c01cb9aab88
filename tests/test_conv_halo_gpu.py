"""The halo-staged 3x3 conv (csrc/conv_halo.hip; fd_gemm takes it for eligible stride-1 convs) and the consumer
GroupNorm (+ SiLU) folded into its staging pass (fd_gemm_params.gi_affine, group_norm_affine).

Bars: against torch fp32 (CPU) on the same bf16 / fp16 inputs, rel-L2 < 6e-3 (the implicit-GEMM conv's bar,
tests/test_kernels_gpu.py); GroupNorm folded into the conv BITWISE equal to fd_group_norm followed by the same conv
(the staging pass stores exactly the values fd_group_norm stores); two images in one launch bitwise equal to one
launch per image; TH = 8 and TH = 16 tiles bitwise equal (same per-element K order).  Ragged edges (62 x 46, the
forward_upsample_size latent), nearest x2 and odd-size upsample, residual + per-image row bias + activation, and the
GroupNorm statistics the epilogue writes for the next GroupNorm are covered.  Reference call sites: diffusers
ResnetBlock2D (norm1 -> SiLU -> conv1, norm2 -> SiLU -> conv2) from unet_2d_condition_vae_extension.py:611-690 and
the VAE decode (pipeline_FaithDiff_tlc.py:1438)."""
import pytest
import torch
import torch.nn.functional as F

from parity import rel_l2  # noqa: E402  (records every measured value)

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _knobs(**kw):
    from fdhip import knobs
    return knobs.override(**kw)


def _inputs(nimg, H, W, Cin, Cout, dtype, seed=0, up=None):
    g = torch.Generator().manual_seed(seed)
    Hi, Wi = (H, W) if up is None else up
    x = torch.randn(nimg, Cin, Hi, Wi, generator=g).to(dtype)
    w = (torch.randn(Cout, Cin, 3, 3, generator=g) / (9 * Cin) ** 0.5).to(dtype)
    b = torch.randn(Cout, generator=g) * 0.1
    return x, w, b


def _nhwc(x):
    n, c, h, w = x.shape
    return x.permute(0, 2, 3, 1).reshape(n * h * w, c).contiguous()


def _nchw(y, n, h, w):
    return y.reshape(n, h, w, -1).permute(0, 3, 1, 2)


def _hip_conv(x, w, b, nimg, H, W, **kw):
    from fdhip import ops
    wp = ops.pack_conv3x3(w.float()).to(DEV, x.dtype)
    xs = _nhwc(x).to(DEV)
    return ops.conv3x3(xs, wp, b.float().to(DEV), nimg, H, W, **kw), xs, wp


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("nimg,H,W,Cin,Cout", [(2, 64, 64, 320, 320), (1, 62, 46, 640, 640), (1, 48, 32, 128, 128),
                                               (2, 32, 48, 256, 512)])
def test_halo_conv_matches_torch(dtype, nimg, H, W, Cin, Cout):
    from fdhip import ops
    x, w, b = _inputs(nimg, H, W, Cin, Cout, dtype)
    with _knobs(FD_CONV_HALO_MIN_TILES=1):
        wp = ops.pack_conv3x3(w.float()).to(DEV, dtype)
        xs = _nhwc(x).to(DEV)
        assert ops.halo_conv_rows(xs, wp, nimg, H, W) > 0
        y = ops.conv3x3(xs, wp, b.float().to(DEV), nimg, H, W)
    torch.cuda.synchronize()
    ref = F.conv2d(x.float(), w.float(), b, padding=1)
    rel = rel_l2(_nchw(y.float().cpu(), nimg, H, W), ref)
    assert rel < 6e-3, rel


@pytest.mark.parametrize("silu", [True, False])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_groupnorm_folded_into_conv_is_bitwise_groupnorm_then_conv(silu, dtype):
    from fdhip import ops
    nimg, H, W, Cin, Cout = 2, 64, 48, 640, 320
    x, w, b = _inputs(nimg, H, W, Cin, Cout, dtype, seed=3)
    g = torch.Generator().manual_seed(4)
    gamma = (1 + 0.1 * torch.randn(Cin, generator=g)).to(DEV)
    beta = (0.1 * torch.randn(Cin, generator=g)).to(DEV)
    with _knobs(FD_CONV_HALO_MIN_TILES=1):
        wp = ops.pack_conv3x3(w.float()).to(DEV, dtype)
        xs = _nhwc(x).to(DEV)
        bd = b.float().to(DEV)
        aff = ops.group_norm_affine(xs, gamma, beta, nimg, H * W, Cin, 32, 1e-5)
        fused = ops.conv3x3(xs, wp, bd, nimg, H, W, gn_in=(aff, silu))
        hn = ops.group_norm(xs, gamma, beta, nimg, H * W, Cin, 32, 1e-5, silu=silu)
        plain = ops.conv3x3(hn, wp, bd, nimg, H, W)
    torch.cuda.synchronize()
    assert torch.equal(fused, plain)
    xr = F.group_norm(x.float(), 32, gamma.cpu(), beta.cpu(), 1e-5)
    if silu:
        xr = F.silu(xr)
    ref = F.conv2d(xr.to(dtype).float(), w.float(), b, padding=1)
    rel = rel_l2(_nchw(fused.float().cpu(), nimg, H, W), ref)
    assert rel < 6e-3, rel


def test_halo_conv_batch_and_tile_shape_invariant():
    """Two images in one launch == one launch per image, and 8-row tiles == 16-row tiles, bitwise."""
    from fdhip import ops
    nimg, H, W, C = 2, 64, 64, 320
    x, w, b = _inputs(nimg, H, W, C, C, torch.bfloat16, seed=5)
    wp = ops.pack_conv3x3(w.float()).to(DEV, torch.bfloat16)
    xs = _nhwc(x).to(DEV)
    bd = b.float().to(DEV)
    with _knobs(FD_CONV_HALO_MIN_TILES=1):
        both = ops.conv3x3(xs, wp, bd, nimg, H, W)
        one = torch.cat([ops.conv3x3(xs[i * H * W:(i + 1) * H * W].contiguous(), wp, bd, 1, H, W) for i in range(2)])
        assert ops.halo_conv_rows(xs, wp, nimg, H, W) == 256
    with _knobs(FD_CONV_HALO_MIN_TILES=100000):
        assert ops.halo_conv_rows(xs, wp, nimg, H, W) == 0  # the implicit GEMM
    # TH = 8 tiles: a threshold between the two tile counts (16-row: 2 x 4 x 4 x 2 = 64 tiles; 8-row: 128)
    with _knobs(FD_CONV_HALO_MIN_TILES=100, FD_CONV_HALO_SPLIT16=0):
        assert ops.halo_conv_rows(xs, wp, nimg, H, W) == 128
        th8 = ops.conv3x3(xs, wp, bd, nimg, H, W)
    torch.cuda.synchronize()
    assert torch.equal(both, one)
    assert torch.equal(both, th8)


def test_halo_conv_split16():
    """From 640 input channels the planner prefers 16-row tiles with the input channels split over two workgroups
    (2 x 64 tiles >= 100) to 8-row tiles: a different K association (the halves are summed last), so compared with
    fp32; below 640 channels it keeps the 8-row tiles."""
    from fdhip import ops
    nimg, H, W, C = 2, 64, 64, 640
    x, w, b = _inputs(nimg, H, W, C, 320, torch.bfloat16, seed=6)
    wp = ops.pack_conv3x3(w.float()).to(DEV, torch.bfloat16)
    xs = _nhwc(x).to(DEV)
    with _knobs(FD_CONV_HALO_MIN_TILES=100):
        assert ops.halo_conv_rows(xs, wp, nimg, H, W) == 256
        sk16 = ops.conv3x3(xs, wp, b.float().to(DEV), nimg, H, W)
        assert ops.halo_conv_rows(xs[:, :320].contiguous(), wp[:, :9 * 320].contiguous(), nimg, H, W) == 128
    torch.cuda.synchronize()
    ref = F.conv2d(x.float(), w.float(), b, padding=1)
    assert rel_l2(_nchw(sk16.float().cpu(), nimg, H, W), ref) < 6e-3


@pytest.mark.parametrize("up", [(32, 32), (31, 23)])
def test_halo_conv_upsample(up):
    """Upsample2D: nearest x2, and diffusers' upsample_size path (31 x 23 -> 62 x 46)."""
    from fdhip import ops
    H, W = (64, 64) if up == (32, 32) else (62, 46)
    x, w, b = _inputs(1, H, W, 640, 640, torch.bfloat16, seed=7, up=up)
    with _knobs(FD_CONV_HALO_MIN_TILES=1):
        wp = ops.pack_conv3x3(w.float()).to(DEV, torch.bfloat16)
        xs = _nhwc(x).to(DEV)
        assert ops.halo_conv_rows(xs, wp, 1, up[0], up[1], upsample=True, upsample_size=(H, W)) > 0
        y = ops.conv3x3(xs, wp, b.float().to(DEV), 1, up[0], up[1], upsample=True, upsample_size=(H, W))
    torch.cuda.synchronize()
    ref = F.conv2d(F.interpolate(x.float(), size=(H, W), mode="nearest"), w.float(), b, padding=1)
    rel = rel_l2(_nchw(y.float().cpu(), 1, H, W), ref)
    assert rel < 6e-3, rel


def test_halo_conv_epilogue_residual_rowbias_act_and_groupnorm_statistics():
    """conv1 of a ResnetBlock2D (+ per-image time-embedding row bias) and conv2 (+ residual), the epilogue's
    GroupNorm statistics feeding the next GroupNorm (GnStats) -- against torch and against a statistics pass."""
    from fdhip import ops
    nimg, H, W, C = 2, 32, 32, 640
    x, w, b = _inputs(nimg, H, W, C, C, torch.bfloat16, seed=9)
    g = torch.Generator().manual_seed(10)
    temb = torch.randn(nimg, C, generator=g)
    res = torch.randn(nimg, C, H, W, generator=g).to(torch.bfloat16)
    gamma = (1 + 0.1 * torch.randn(C, generator=g)).to(DEV)
    beta = (0.1 * torch.randn(C, generator=g)).to(DEV)
    with _knobs(FD_CONV_HALO_MIN_TILES=1):
        wp = ops.pack_conv3x3(w.float()).to(DEV, torch.bfloat16)
        xs = _nhwc(x).to(DEV)
        st = ops.GnStats(nimg, H * W, 32, DEV)
        y = ops.conv3x3(xs, wp, b.float().to(DEV), nimg, H, W, rowbias=temb.to(DEV), residual=_nhwc(res).to(DEV),
                        act="silu", gn=st)
        assert st.done and st.rows == 256
        a1 = ops.group_norm_affine(y, gamma, beta, nimg, H * W, C, 32, 1e-5, stats=st)
        a2 = ops.group_norm_affine(y, gamma, beta, nimg, H * W, C, 32, 1e-5)
    torch.cuda.synchronize()
    ref = F.silu(F.conv2d(x.float(), w.float(), b, padding=1) + temb[:, :, None, None]) + res.float()
    rel = rel_l2(_nchw(y.float().cpu(), nimg, H, W), ref)
    assert rel < 6e-3, rel
    # statistics from the epilogue vs from a pass over y: same (scale, shift) up to fp32 summation order
    assert rel_l2(a1[:nimg * C].cpu(), a2[:nimg * C].cpu()) < 1e-5


@pytest.mark.parametrize("fold_gn", [False, True])
def test_halo_conv_ragged_rowbias_residual_silu(fold_gn):
    """The r04 fault's class (profiles/r04zc_serialized_fault.log): rows of a ragged tile past the last image must not
    read the per-image row bias or the residual.  23 x 33 images (neither a multiple of the 8 / 16 tile rows nor of
    the 16 tile columns), two images, a time-embedding table of EXACTLY nimg rows and a residual of exactly M rows in
    their own allocations, SiLU, with and without the consumer GroupNorm folded into the staging pass -- against
    torch.  The halo kernel must be the one that runs (fd_conv_halo_plan > 0)."""
    from fdhip import ops
    nimg, H, W, C = 2, 23, 33, 320
    x, w, b = _inputs(nimg, H, W, C, C, torch.bfloat16, seed=21)
    g = torch.Generator().manual_seed(22)
    temb = torch.randn(nimg, C, generator=g)
    res = torch.randn(nimg, C, H, W, generator=g).to(torch.bfloat16)
    gamma = 1 + 0.1 * torch.randn(C, generator=g)
    beta = 0.1 * torch.randn(C, generator=g)
    with _knobs(FD_CONV_HALO_MIN_TILES=1):
        wp = ops.pack_conv3x3(w.float()).to(DEV, torch.bfloat16)
        xs, tb, rs = _nhwc(x).to(DEV), temb.to(DEV).contiguous(), _nhwc(res).to(DEV)
        assert tb.shape == (nimg, C) and rs.shape == (nimg * H * W, C)
        assert ops.halo_conv_rows(xs, wp, nimg, H, W, residual=rs, rowbias=tb) > 0
        kw = dict(rowbias=tb, residual=rs, act="silu")
        if fold_gn:
            aff = ops.group_norm_affine(xs, gamma.to(DEV), beta.to(DEV), nimg, H * W, C, 32, 1e-5)
            y = ops.conv3x3(xs, wp, b.float().to(DEV), nimg, H, W, gn_in=(aff, True), **kw)
        else:
            y = ops.conv3x3(xs, wp, b.float().to(DEV), nimg, H, W, **kw)
    torch.cuda.synchronize()
    xin = x.float()
    if fold_gn:
        xin = F.silu(F.group_norm(xin, 32, gamma, beta, 1e-5)).to(torch.bfloat16).float()
    ref = F.silu(F.conv2d(xin, w.float(), b, padding=1) + temb[:, :, None, None]) + res.float()
    rel = rel_l2(_nchw(y.float().cpu(), nimg, H, W), ref)
    assert torch.isfinite(y).all() and rel < 6e-3, rel


@pytest.mark.parametrize("Cin,Cout", [(1280, 1280), (2560, 1280), (640, 640)])
def test_halo_conv_channel_split(Cin, Cout):
    """The 32^2 level (C2: 2 x 32 x 32): too few tiles, so the input channels are split over two workgroups combined
    pairwise (SK) -- vs torch, bitwise batch-invariant (the split follows m_ref), GroupNorm folded bitwise.  Cout =
    640 has 64 tiles, under the default floor even split: the floor is lowered to reach the SK kernel with 4 n tiles."""
    from fdhip import knobs
    with knobs.override(**({"FD_CONV_HALO_MIN_TILES": 128} if Cout == 640 else {})):
        _channel_split(Cin, Cout)


def _channel_split(Cin, Cout):
    from fdhip import ops
    nimg, H, W = 2, 32, 32
    x, w, b = _inputs(nimg, H, W, Cin, Cout, torch.bfloat16, seed=11)
    g = torch.Generator().manual_seed(12)
    gamma = (1 + 0.1 * torch.randn(Cin, generator=g)).to(DEV)
    beta = (0.1 * torch.randn(Cin, generator=g)).to(DEV)
    wp = ops.pack_conv3x3(w.float()).to(DEV, torch.bfloat16)
    xs = _nhwc(x).to(DEV)
    bd = b.float().to(DEV)
    assert ops.halo_conv_rows(xs, wp, nimg, H, W) == 128
    y = ops.conv3x3(xs, wp, bd, nimg, H, W)
    one = torch.cat([ops.conv3x3(xs[i * H * W:(i + 1) * H * W].contiguous(), wp, bd, 1, H, W) for i in range(2)]) \
        if ops.halo_conv_rows(xs[:H * W].contiguous(), wp, 1, H, W) == 128 else None
    aff = ops.group_norm_affine(xs, gamma, beta, nimg, H * W, Cin, 32, 1e-5)
    fused = ops.conv3x3(xs, wp, bd, nimg, H, W, gn_in=(aff, True))
    plain = ops.conv3x3(ops.group_norm(xs, gamma, beta, nimg, H * W, Cin, 32, 1e-5, silu=True), wp, bd, nimg, H, W)
    torch.cuda.synchronize()
    ref = F.conv2d(x.float(), w.float(), b, padding=1)
    rel = rel_l2(_nchw(y.float().cpu(), nimg, H, W), ref)
    assert rel < 6e-3, rel
    assert torch.equal(fused, plain)
    if one is not None:
        assert torch.equal(y, one)


@pytest.mark.parametrize("case", ["vae1024_like", "cin256_gn_res", "n256_upsample"])
def test_halo_conv_persistent_form_is_bitwise_the_per_tile_form(case):
    """The persistent form (FD_CONV_HALO_PT: one workgroup per CU walking 256 x 128 tiles, the next tile's DMA under
    this tile's epilogue, 32-row epilogue passes) against the one-workgroup-per-tile form: outputs and the epilogue's
    GroupNorm statistics bitwise equal, with the GroupNorm + SiLU folded into the staging, a residual and fp16 (the
    VAE decoder's 1024^2 level at a quarter of its pixels), 4 input-channel chunks (a patch DMA issued inside the
    K loop), and a nearest x2 upsample with 2 output-channel tiles (FD_CONV_HALO_PT = 2 takes it from gemm256).
    One case against torch fp32 as well."""
    from fdhip import ops
    nimg, H, W, Cin, Cout, up, dt = {"vae1024_like": (1, 512, 256, 128, 128, None, torch.float16),
                                     "cin256_gn_res": (2, 256, 256, 256, 128, None, torch.bfloat16),
                                     "n256_upsample": (1, 512, 256, 256, 256, (256, 128), torch.float16)}[case]
    x, w, b = _inputs(nimg, H, W, Cin, Cout, dt, seed=21, up=up)
    Hi, Wi = up if up else (H, W)
    g = torch.Generator().manual_seed(22)
    gamma = (1 + 0.1 * torch.randn(Cin, generator=g)).to(DEV)
    beta = (0.1 * torch.randn(Cin, generator=g)).to(DEV)
    res = _nhwc(torch.randn(nimg, Cout, H, W, generator=g).to(dt)).to(DEV)
    wp = ops.pack_conv3x3(w.float()).to(DEV, dt)
    xs = _nhwc(x).to(DEV)
    bd = b.float().to(DEV)
    kw = dict(upsample=True) if up else dict(residual=res)
    outs = {}
    for pt in (0, 2):
        with _knobs(FD_CONV_HALO_PT=pt, FD_CONV_HALO=2):
            npt = ops.halo_conv_pt(xs, wp, nimg, Hi, Wi, upsample=bool(up), residual=not up)
            assert (npt > 0) == (pt > 0), npt
            st = ops.GnStats(nimg, H * W, 32, DEV)
            if up:
                y = ops.conv3x3(xs, wp, bd, nimg, Hi, Wi, gn=st, **kw)
            else:
                aff = ops.group_norm_affine(xs, gamma, beta, nimg, H * W, Cin, 32, 1e-5)
                y = ops.conv3x3(xs, wp, bd, nimg, H, W, gn_in=(aff, True), gn=st, **kw)
            assert st.done and st.rows == 256
            torch.cuda.synchronize()
            outs[pt] = (y.clone(), st.part[:nimg * (H * W // 256) * 32 * 2].clone())  # 256-row blocks written
    assert torch.equal(outs[0][0], outs[2][0])
    assert torch.equal(outs[0][1], outs[2][1])
    if case == "vae1024_like":
        xr = F.silu(F.group_norm(x.float(), 32, gamma.cpu(), beta.cpu(), 1e-5)).to(dt).float()
        ref = F.conv2d(xr, w.float(), b, padding=1) + _nchw(res.float().cpu(), nimg, H, W)
        rel = rel_l2(_nchw(outs[2][0].float().cpu(), nimg, H, W), ref)
        assert rel < 6e-3, rel


def test_halo_conv_persistent_form_default_takes_gn_convs_without_residual():
    """FD_CONV_HALO_PT's default (3): the persistent form only for GroupNorm-folded convs without a residual (the VAE
    1024^2 resnet conv1s); the residual convs and the plain ones keep one workgroup per tile."""
    from fdhip import ops
    nimg, H, W, C = 1, 512, 256, 128
    xs = torch.zeros(nimg * H * W, C, dtype=torch.float16, device=DEV)
    wp = torch.zeros(C, 9 * C, dtype=torch.float16, device=DEV)
    assert ops.halo_conv_pt(xs, wp, nimg, H, W, gn_in=True) > 0
    assert ops.halo_conv_pt(xs, wp, nimg, H, W, gn_in=True, residual=True) == 0
    assert ops.halo_conv_pt(xs, wp, nimg, H, W) == 0


@pytest.mark.parametrize("nimg,H,W,C,Cout,dt", [(1, 64, 64, 512, 512, torch.float16), (1, 32, 48, 256, 256, torch.float16),
                                                (2, 32, 32, 1280, 1280, torch.bfloat16),
                                                (2, 64, 64, 640, 640, torch.bfloat16),
                                                (1, 8, 32, 128, 128, torch.float16),
                                                (1, 23, 17 + 16, 320, 320, torch.bfloat16)])
def test_upsample_conv_in_four_phases(nimg, H, W, C, Cout, dt):
    """Upsample2D in the phase form (fd_gemm_params.up_phase, pack_conv3x3_up2): against torch fp32 nearest x2 +
    conv3x3 on the same inputs and the original weights (rel-L2 < 6e-3: the summed weights are rounded once to
    the conv dtype), against the one-workgroup-per-tap upsample conv, bitwise batch invariant (two images in one
    launch == one launch per image), and its epilogue GroupNorm statistics equal to a pass over the output
    (fp32 summation order).  VAE decoder levels (fp16, 256 / 512 ch), the UNet's (bf16, 1280 / 640 ch, 2 images),
    a 128-row tile case (H = 8) and a ragged one (23 x 33)."""
    from fdhip import ops
    x, w, b = _inputs(nimg, 2 * H, 2 * W, C, Cout, dt, seed=31, up=(H, W))
    xs = _nhwc(x).to(DEV)
    bd = b.float().to(DEV)
    wph = ops.pack_conv3x3_up2(w.float()).to(DEV, dt)
    assert ops.up2_phase_ok(xs, wph, nimg, H, W)
    st = ops.GnStats(nimg, 4 * H * W, 32, DEV)
    y = ops.conv3x3_up2(xs, wph, bd, nimg, H, W, gn=st)
    with _knobs(FD_CONV_HALO_MIN_TILES=1):
        wp = ops.pack_conv3x3(w.float()).to(DEV, dt)
        y9 = ops.conv3x3(xs, wp, bd, nimg, H, W, upsample=True)
    one = None
    if nimg == 2:
        one = torch.cat([ops.conv3x3_up2(xs[i * H * W:(i + 1) * H * W].contiguous(), wph, bd, 1, H, W)
                         for i in range(2)])
    torch.cuda.synchronize()
    ref = F.conv2d(F.interpolate(x.float(), scale_factor=2, mode="nearest"), w.float(), b, padding=1)
    rel = rel_l2(_nchw(y.float().cpu(), nimg, 2 * H, 2 * W), ref)
    assert rel < 6e-3, rel
    assert rel_l2(y.float().cpu(), y9.float().cpu()) < 6e-3
    if one is not None:
        assert torch.equal(y, one)
    if st.done:
        g = torch.Generator().manual_seed(32)
        gamma = (1 + 0.1 * torch.randn(Cout, generator=g)).to(DEV)
        beta = (0.1 * torch.randn(Cout, generator=g)).to(DEV)
        a1 = ops.group_norm_affine(y, gamma, beta, nimg, 4 * H * W, Cout, 32, 1e-5, stats=st)
        a2 = ops.group_norm_affine(y, gamma, beta, nimg, 4 * H * W, Cout, 32, 1e-5)
        torch.cuda.synchronize()
        assert rel_l2(a1[:nimg * Cout].cpu(), a2[:nimg * Cout].cpu()) < 1e-5
    else:
        assert H % 16 or W % 16  # statistics are written for whole tiles


def test_short_rowbias_or_residual_is_refused_on_the_device_path():
    """fd_gemm_params.rowbias_rows / residual_rows through the product host layer (ops.conv3x3 / ops.gemm fill them
    from the tensors' extents): a time-embedding table with fewer rows than images, or a residual one row short, is
    FD_ERR_SHAPE -> RuntimeError before any launch; the exact-size tables run."""
    from fdhip import ops
    nimg, H, W, C = 2, 23, 33, 320
    x, w, b = _inputs(nimg, H, W, C, C, torch.bfloat16, seed=31)
    with _knobs(FD_CONV_HALO_MIN_TILES=1):
        wp = ops.pack_conv3x3(w.float()).to(DEV, torch.bfloat16)
        xs, bd = _nhwc(x).to(DEV), b.float().to(DEV)
        temb = torch.randn(nimg, C, device=DEV)
        res = torch.randn(nimg * H * W, C, device=DEV).to(torch.bfloat16)
        with pytest.raises(RuntimeError):
            ops.conv3x3(xs, wp, bd, nimg, H, W, rowbias=temb[:1].contiguous())
        with pytest.raises(RuntimeError):
            ops.conv3x3(xs, wp, bd, nimg, H, W, residual=res[:-1])
        a = torch.randn(64, 128, device=DEV).to(torch.bfloat16)
        wt = torch.randn(160, 128, device=DEV).to(torch.bfloat16)
        with pytest.raises(RuntimeError):
            ops.gemm(a, wt, residual=torch.zeros(63, 160, device=DEV, dtype=torch.bfloat16))
        y = ops.conv3x3(xs, wp, bd, nimg, H, W, rowbias=temb, residual=res)
        g = ops.gemm(a, wt, residual=torch.zeros(64, 160, device=DEV, dtype=torch.bfloat16))
    torch.cuda.synchronize()
    assert torch.isfinite(y.float()).all() and g.shape == (64, 160)


@pytest.mark.parametrize("case", ["th16_n160", "gn_res_rowbias_stats", "th8", "split_k", "phase_f16", "phase_bf16",
                                  "ragged_gn", "f16_n128_ns4"])
def test_ping_pong_loop_is_bitwise_the_one_barrier_loop(case):
    """The two-group ping-pong K loop (FD_CONV_HALO_PP = 1, the default) against the round-5 one-barrier loop
    (FD_CONV_HALO_PP = 0): the per-element K order is the same (chunk by chunk, tap by tap, half 0 then half 1), so
    the outputs and the epilogue's GroupNorm statistics must be bitwise equal -- 256 x 160 and 256 x 128 tiles, 128-row
    tiles, the pairwise channel split, the Upsample2D phase form, the GroupNorm folded into the staging (its patch
    transformed in the ping-pong LOAD segments), residual + row bias + SiLU, a ragged 23 x 33 image, fp16 with the
    4-deep weight ring."""
    from fdhip import ops
    nimg, H, W, Cin, Cout, dt, knob = {
        "th16_n160": (2, 64, 64, 320, 320, torch.bfloat16, dict(FD_CONV_HALO_MIN_TILES=1)),
        "gn_res_rowbias_stats": (2, 64, 48, 640, 320, torch.bfloat16, dict(FD_CONV_HALO_MIN_TILES=1)),
        "th8": (2, 64, 64, 320, 320, torch.bfloat16, dict(FD_CONV_HALO_MIN_TILES=100, FD_CONV_HALO_SPLIT16=0)),
        "split_k": (2, 32, 32, 1280, 1280, torch.bfloat16, {}),
        "phase_f16": (1, 32, 48, 256, 256, torch.float16, {}),
        "phase_bf16": (2, 32, 32, 1280, 1280, torch.bfloat16, {}),
        "ragged_gn": (2, 23, 33, 320, 320, torch.bfloat16, dict(FD_CONV_HALO_MIN_TILES=1)),
        "f16_n128_ns4": (1, 128, 64, 256, 128, torch.float16, dict(FD_CONV_HALO_MIN_TILES=1, FD_CONV_HALO_NS16=4)),
    }[case]
    phase = case.startswith("phase")
    g = torch.Generator().manual_seed(41)
    x, w, b = _inputs(nimg, 2 * H if phase else H, 2 * W if phase else W, Cin, Cout, dt, seed=40,
                      up=(H, W) if phase else None)
    xs, bd = _nhwc(x).to(DEV), b.float().to(DEV)
    gn_in = case in ("gn_res_rowbias_stats", "ragged_gn", "split_k", "f16_n128_ns4")
    epi = case in ("gn_res_rowbias_stats", "ragged_gn")
    gamma = (1 + 0.1 * torch.randn(Cin, generator=g)).to(DEV)
    beta = (0.1 * torch.randn(Cin, generator=g)).to(DEV)
    temb = torch.randn(nimg, Cout, generator=g).to(DEV)
    res = _nhwc(torch.randn(nimg, Cout, H, W, generator=g).to(dt)).to(DEV)
    outs = []
    for pp in (0, 1):
        with _knobs(FD_CONV_HALO_PP=pp, **knob):
            st = ops.GnStats(nimg, (4 if phase else 1) * H * W, 32, DEV)
            if phase:
                wph = ops.pack_conv3x3_up2(w.float()).to(DEV, dt)
                y = ops.conv3x3_up2(xs, wph, bd, nimg, H, W, gn=st)
            else:
                wp = ops.pack_conv3x3(w.float()).to(DEV, dt)
                assert ops.halo_conv_rows(xs, wp, nimg, H, W) > 0
                kw = dict(rowbias=temb, residual=res, act="silu") if epi else {}
                if gn_in:
                    kw["gn_in"] = (ops.group_norm_affine(xs, gamma, beta, nimg, H * W, Cin, 32, 1e-5), True)
                y = ops.conv3x3(xs, wp, bd, nimg, H, W, gn=st, **kw)
            torch.cuda.synchronize()
            hw = (4 if phase else 1) * H * W  # the written partial blocks: [nimg][hw / rows][32] float2
            outs.append((y.clone(), st.part[:nimg * (hw // st.rows) * 32 * 2].clone() if st.done else None))
    assert torch.isfinite(outs[1][0].float()).all()
    assert torch.equal(outs[0][0], outs[1][0])
    if outs[0][1] is not None:
        assert torch.equal(outs[0][1], outs[1][1])
