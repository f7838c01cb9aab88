"""BSRNet pre-pass on HIP (fdhip/bsrnet.py) against the fp32 oracle (oracle/bsrnet.py, itself pinned to the
reference module's outputs by tests/test_bsrnet_cpu.py), same seeded weights and images, through the C ABI.

Bars: rel-L2 <= 5e-3 on the upscaled image (fp16 activations through nb RRDBs: ~15 * nb + 6 convs in fp32
accumulation, each rounded to fp16 once); the LeakyReLU epilogue and fd_axpby against torch."""
import os

import numpy as np
import pytest
import torch

import parity  # records every measured value (tests/golden/parity.py)
import torch.nn.functional as F

from oracle import bsrnet as ob

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "bsrnet_golden.npz")


def rel(a, b):
    return parity.rel_l2(a.float().cpu(), b.float().cpu())


def test_lrelu_epilogue_and_axpby():
    from fdhip import ops
    x = torch.randn(4096, 192, device="cuda").to(torch.float16)
    w = (torch.randn(32, 9 * 128, device="cuda") * 0.05).to(torch.float16)
    b = torch.randn(32, device="cuda") * 0.1
    out = torch.zeros(4096, 192, device="cuda", dtype=torch.float16)
    ops.conv3x3(x[:, :128], w, b, 1, 64, 64, out=out[:, 64:96], act="lrelu", lda=192)  # strided in / out
    xin = x[:, :128].float().reshape(1, 64, 64, 128).permute(0, 3, 1, 2)
    wt = w.float().reshape(32, 3, 3, 128).permute(0, 3, 1, 2)
    ref = F.leaky_relu(F.conv2d(xin, wt, b, padding=1), 0.2).permute(0, 2, 3, 1).reshape(4096, 32)
    assert rel(out[:, 64:96], ref) < 2e-3
    assert torch.count_nonzero(out[:, :64]) == 0 and torch.count_nonzero(out[:, 96:]) == 0
    y = torch.randn(4096, 192, device="cuda").to(torch.float16)
    z = y.clone()
    ops.axpby(x[:, 8:72], z[:, 8:72], z[:, 8:72], 0.2, 1.0)
    want = 0.2 * x[:, 8:72].float() + y[:, 8:72].float()
    assert rel(z[:, 8:72], want) < 1e-3 and torch.equal(z[:, :8], y[:, :8]) and torch.equal(z[:, 72:], y[:, 72:])


def _hip(sd, nb):
    from fdhip.bsrnet import HipRRDBNet
    return HipRRDBNet(sd, nb, "cuda")


def test_forward_and_deg_remove_match_oracle_on_golden_inputs():
    z = np.load(GOLD)
    nb = int(z["nb"])
    sd = ob.random_weights(int(z["seed"]), nb)
    net = _hip(sd, nb)
    y = net.forward(torch.from_numpy(z["x"]).cuda())
    y2 = net.deg_remove(torch.from_numpy(z["x2"]).cuda(), int(z["tile_size"]), int(z["tile_pad"]))
    torch.cuda.synchronize()
    assert y.shape == (1, 3, 72, 52) and y2.shape == (1, 3, 84, 56)
    assert rel(y, torch.from_numpy(z["y"])) < 5e-3, rel(y, torch.from_numpy(z["y"]))
    assert rel(y2, torch.from_numpy(z["y2"])) < 5e-3, rel(y2, torch.from_numpy(z["y2"]))


def test_product_bsrnet_full_depth_matches_oracle():
    """create_bsrnet('random-init') (nb = 23, the published depth) through the drop-in surface, test.py:98-101."""
    from FaithDiff.create_FaithDiff_model import create_bsrnet
    from utils.image_process import image2tensor, tensor2image
    net = create_bsrnet("random-init")
    net.to("cuda")
    net.eval()
    img = np.random.default_rng(4).integers(0, 256, (26, 20, 3), dtype=np.uint8)
    x = image2tensor(img)
    y = net.deg_remove(x.cuda(), tile_size=16, tile_pad=4)
    with torch.no_grad():
        want = ob.deg_remove(net.state_dict(), x, 23, 16, 4)
    torch.cuda.synchronize()
    assert y.shape == (1, 3, 104, 80)
    assert rel(y, want) < 5e-3, rel(y, want)
    assert tensor2image(y).shape == (104, 80, 3)
