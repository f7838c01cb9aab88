"""Split-K hand-off health: the pairwise split-K forms -- gemm8's S = 2 (the LN-fold ff-out
producer, 2048 x 1280 x 5120) and the halo conv's channel split (the 32^2 level's 1280-channel convs) -- hand one
split's fp32 partial to its partner through a flag with a bounded wait.  A timed-out wait must (1) poison its tile
with NaN instead of hanging, (2) be counted (fd_splitk_health), and (3) leave nothing stale behind once the host has
checked: ops.split_k_health() raises, re-zeroes every split-K workspace's counters, and the next launches are
bitwise the launches before the fault.  fd_splitk_test_drop(1) (a test hook) makes every publisher skip its flag;
each waiting wave then times out after ~2^24 short sleeps (~1-2 s).  Reference call sites: the ff out
(unet_2d_condition_vae_extension.py BasicTransformerBlock, pipeline_FaithDiff_tlc.py:1350) and the resnet convs."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _drop(on):
    from fdhip import lib as L
    L.check(L.load().fd_splitk_test_drop(1 if on else 0), "fd_splitk_test_drop")


def _halo_sk():
    from fdhip import ops
    g = torch.Generator(device=DEV).manual_seed(50)
    nimg, H, W, C = 2, 32, 32, 1280
    x = torch.randn(nimg * H * W, C, device=DEV, generator=g).to(torch.bfloat16)
    wp = (torch.randn(C, 9 * C, device=DEV, generator=g) / (9 * C) ** 0.5).to(torch.bfloat16)
    b = torch.randn(C, device=DEV, generator=g) * 0.1
    assert ops.halo_conv_rows(x, wp, nimg, H, W) == 128  # the channel-split (SK) form
    return lambda: ops.conv3x3(x, wp, b, nimg, H, W)


def _gemm8_pairwise():
    from fdhip import ops
    g = torch.Generator(device=DEV).manual_seed(51)
    M, C, K0 = 2048, 1280, 5120
    att = torch.randn(M, K0, device=DEV, generator=g).to(torch.bfloat16)
    wo = (torch.randn(C, K0, device=DEV, generator=g) * K0 ** -0.5).to(torch.bfloat16)
    res = torch.randn(M, C, device=DEV, generator=g).to(torch.bfloat16)
    st = torch.zeros((M, C // 160, 2), device=DEV)
    return lambda: ops.gemm(att, wo, residual=res, out=res.clone(), ln_out=st)


@pytest.mark.parametrize("form", ["halo_channel_split", "gemm8_pairwise"])
def test_timed_out_split_k_handoff_is_poisoned_counted_and_reset(form):
    from fdhip import ops
    run = {"halo_channel_split": _halo_sk, "gemm8_pairwise": _gemm8_pairwise}[form]()
    assert ops.split_k_health() == 0
    ref = run().clone()
    torch.cuda.synchronize()
    assert torch.isfinite(ref.float()).all()
    _drop(True)
    try:
        bad = run().clone()
        torch.cuda.synchronize()
    finally:
        _drop(False)
    assert not torch.isfinite(bad.float()).all()  # poisoned, not silently wrong
    with pytest.raises(RuntimeError, match="timed out"):
        ops.split_k_health()
    assert ops.split_k_health() == 0  # the count was reset
    ws = ops._GEMM_WS[torch.device(DEV, torch.cuda.current_device())]
    assert int(ws[:65536 * 4].view(torch.int32).abs().sum().item()) == 0
    for _ in range(2):  # later launches start clean: bitwise the launch before the fault
        again = run()
        torch.cuda.synchronize()
        assert torch.equal(again, ref)
    assert ops.split_k_health() == 0
