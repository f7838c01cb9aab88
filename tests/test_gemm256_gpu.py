"""The 256 x 256-tile GEMM / implicit-GEMM conv (csrc/gemm256.hip) that fd_gemm takes for large-M launches with
N % 256 == 0 (the VAE's 256- / 512-channel convs): against fp32 torch, and bitwise against the 256 x 128 kernel
(gemm8, one split) on the same launch (knob FD_GEMM256 = 0) -- both sum K in the same 32-deep order."""

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




def both(fn):
    from fdhip import knobs
    a = fn().clone()
    with knobs.override(FD_GEMM256=0):
        b = fn().clone()
    torch.cuda.synchronize()
    return a, b


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("M,N,K,act,res", [(65536, 512, 1152, "none", False), (65536 + 100, 256, 512, "silu", True),
                                           (49152, 768, 2048, "none", True)])
def test_gemm256_matches_torch_and_gemm8(dtype, M, N, K, act, res):
    from fdhip import ops
    g = torch.Generator(device=DEV).manual_seed(M + N + K)
    a = torch.randn(M, K, generator=g, device=DEV).to(dtype)
    w = (torch.randn(N, K, generator=g, device=DEV) / K ** 0.5).to(dtype)
    bias = torch.randn(N, generator=g, device=DEV) * 0.1
    r = torch.randn(M, N, generator=g, device=DEV).to(dtype) if res else None
    out = torch.empty(M, N, device=DEV, dtype=dtype)
    got, ref8 = both(lambda: ops.gemm(a, w, out=out, bias=bias, residual=r, act=act))
    want = a.float() @ w.float().T + bias
    if act == "silu":
        want = F.silu(want)
    if res:
        want = want + r.float()
    assert rel_l2(got, want) < 6e-3
    assert torch.equal(got, ref8), "gemm256 and gemm8 (S = 1) must agree bitwise"


def conv_ref(x, wp, b, n, H, W, Cin, stride=1, pad=1, up=False, x2=None):
    xi = x.float().view(n, H, W, -1).permute(0, 3, 1, 2)
    if x2 is not None:
        xi = torch.cat([xi, x2.float().view(n, H, W, -1).permute(0, 3, 1, 2)], 1)
    if up:
        xi = F.interpolate(xi, scale_factor=2, mode="nearest")
    w = wp.float().view(wp.shape[0], 3, 3, Cin).permute(0, 3, 1, 2)
    if stride == 2 and pad == 0:
        xi = F.pad(xi, (0, 1, 0, 1))
    y = F.conv2d(xi, w, b, stride=stride, padding=pad)
    return y.permute(0, 2, 3, 1).reshape(-1, w.shape[0])


@pytest.mark.parametrize("case", ["plain", "upsample", "concat", "down", "two_images"])
def test_gemm256_conv(case):
    from fdhip import ops
    dt = torch.float16
    g = torch.Generator(device=DEV).manual_seed(7)
    n, H, W, Cin, Cout, stride, pad, up, C1 = {
        "plain": (1, 256, 256, 256, 512, 1, 1, False, None),
        "upsample": (1, 128, 128, 512, 512, 1, 1, True, None),
        "concat": (1, 256, 256, 512, 256, 1, 1, False, 256),
        "down": (1, 512, 512, 256, 256, 2, 0, False, None),
        "two_images": (2, 192, 160, 128, 256, 1, 1, False, None),
    }[case]
    x = torch.randn(n * H * W, C1 or Cin, generator=g, device=DEV).to(dt)
    x2 = torch.randn(n * H * W, Cin - C1, generator=g, device=DEV).to(dt) if C1 else None
    wp = (torch.randn(Cout, 9 * Cin, generator=g, device=DEV) / (9 * Cin) ** 0.5).to(dt)
    b = torch.randn(Cout, generator=g, device=DEV) * 0.1
    got, ref8 = both(lambda: ops.conv3x3(x, wp, b, n, H, W, stride=stride, pad=pad, upsample=up, x2=x2, C1=C1))
    want = conv_ref(x, wp, b, n, H, W, Cin, stride, pad, up, x2)
    assert got.shape == want.shape
    assert rel_l2(got, want) < 3e-3, rel_l2(got, want)
    assert torch.equal(got, ref8)
