"""Eight-wave 256-row-tile GEMM with in-launch split-K (csrc/gemm8.hip), through the C ABI.

Tolerance as test_kernels_gpu.py (fp32 accumulation, one bf16 rounding on store: rel-L2 < 6e-3 vs an fp32
reference on the same rounded inputs).  Split-K specifics checked here:
  * every split count the planner can pick (driven through m_ref = M / tile_groups) matches fp32;
  * the slab combine is deterministic (repeat launches bitwise equal) and leaves the tile counters zero;
  * a forward that batches n tiles along M is bitwise equal to n single-tile launches (m_ref invariance).
"""
import math

import pytest
import torch
import torch.nn.functional as F
from parity import rel_l2  # noqa: E402  (records every measured value)

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _implicit_gemm_convs():
    """These tests pin the implicit-GEMM conv kernels (the halo-staged conv has its own, tests/test_conv_halo_gpu.py)."""
    from fdhip import knobs
    with knobs.override(FD_CONV_HALO=0):
        yield
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _dev():
    from fdhip import lib
    lib.require_device()
    torch.manual_seed(0)




def rnd(*shape, dtype=torch.bfloat16, scale=1.0):
    return (torch.randn(*shape, device=DEV) * scale).to(dtype)


@pytest.mark.parametrize("groups", [1, 2, 4, 8])
@pytest.mark.parametrize("M,N,K", [(2048, 1280, 1280), (2048, 3840, 1280), (2048, 640, 1920), (4096, 1280, 11520),
                                   (2048, 1280, 23040)])
def test_split_counts_match_fp32(groups, M, N, K):
    from fdhip import ops
    a, w = rnd(M, K), rnd(N, K, scale=K ** -0.5)
    b = torch.randn(N, device=DEV)
    r = rnd(M, N)
    with ops.tile_groups(groups):
        out = ops.gemm(a, w, bias=b, residual=r)
    ref = a.float() @ w.float().T + b + r.float()
    assert rel_l2(out, ref) < 6e-3, rel_l2(out, ref)


def test_split_deterministic_and_counters_reset():
    from fdhip import ops
    M, N, K = 2048, 1280, 11520  # split-K (S = 3) on the 8-wave kernel
    a, w = rnd(M, K), rnd(N, K, scale=K ** -0.5)
    outs = [ops.gemm(a, w) for _ in range(4)]
    torch.cuda.synchronize()
    for o in outs[1:]:
        assert torch.equal(o, outs[0])
    ws = ops._GEMM_WS[torch.device(DEV, torch.cuda.current_device())]
    assert int(ws[:65536 * 4].view(torch.int32).abs().sum().item()) == 0


@pytest.mark.parametrize("act,N,K", [("none", 3840, 1280), ("silu", 1280, 1280), ("geglu", 10240, 1280),
                                     ("none", 1280, 11520)])
def test_tile_batching_bitwise(act, N, K):
    """4 tiles batched along M (m_ref = M/4) == 4 separate single-tile launches, bit for bit (covers the
    8-wave kernel unsplit and split, and the 4-wave kernel)."""
    from fdhip import ops
    Mt = 2048
    a = rnd(4 * Mt, K)
    w = rnd(N, K, scale=K ** -0.5)
    b = torch.randn(N, device=DEV) * 0.1
    if act == "geglu":
        w, b = ops.pack_geglu(w, b)
    with ops.tile_groups(4):
        big = ops.gemm(a, w, bias=b, act=act)
    parts = [ops.gemm(a[i * Mt:(i + 1) * Mt], w, bias=b, act=act) for i in range(4)]
    assert torch.equal(big, torch.cat(parts, 0))


def test_conv_split_and_batching():
    from fdhip import ops
    nimg, H, W, Cin, Cout = 2, 32, 32, 1280, 1280
    x = rnd(2 * nimg * H * W, Cin)
    wt = (torch.randn(Cout, Cin, 3, 3, device=DEV) / math.sqrt(9 * Cin)).to(torch.bfloat16)
    b = torch.randn(Cout, device=DEV) * 0.1
    wp = ops.pack_conv3x3(wt)
    with ops.tile_groups(2):
        big = ops.conv3x3(x, wp, b, 2 * nimg, H, W)
    one = ops.conv3x3(x[:nimg * H * W], wp, b, nimg, H, W)
    assert torch.equal(big[:nimg * H * W], one)
    xr = x[:nimg * H * W].float().reshape(nimg, H, W, Cin).permute(0, 3, 1, 2)
    ref = F.conv2d(xr, wt.float(), b, padding=1).permute(0, 2, 3, 1).reshape(-1, Cout)
    assert rel_l2(one, ref) < 6e-3


@pytest.mark.parametrize("H,W,Cin,Cout,up", [(32, 32, 1280, 1280, True),    # 8192 x 1280 upsample conv: 256 x 160
                                             (64, 64, 1920, 640, False),    # 8192 x 640, K = 17280: 160 wide, S = 2
                                             (64, 64, 320, 320, False)])    # N = 320 (W160 & 2 only)
def test_conv_160_wide_tiles(H, W, Cin, Cout, up):
    """256 x 160 tiles (gemm8 planner, FD_GEMM8_W160): conv vs fp32, tile batching bitwise."""
    from fdhip import ops
    nimg = 2
    x = rnd(2 * nimg * H * W, Cin)
    wt = (torch.randn(Cout, Cin, 3, 3, device=DEV) / math.sqrt(9 * Cin)).to(torch.bfloat16)
    b = torch.randn(Cout, device=DEV) * 0.1
    wp = ops.pack_conv3x3(wt)
    with ops.tile_groups(2):
        big = ops.conv3x3(x, wp, b, 2 * nimg, H, W, upsample=up)
    one = ops.conv3x3(x[:nimg * H * W], wp, b, nimg, H, W, upsample=up)
    Ho = 2 * H if up else H
    assert torch.equal(big[:nimg * Ho * Ho], one)
    xr = x[:nimg * H * W].float().reshape(nimg, H, W, Cin).permute(0, 3, 1, 2)
    if up:
        xr = F.interpolate(xr, scale_factor=2, mode="nearest")
    ref = F.conv2d(xr, wt.float(), b, padding=1).permute(0, 2, 3, 1).reshape(-1, Cout)
    assert rel_l2(one, ref) < 6e-3, rel_l2(one, ref)
