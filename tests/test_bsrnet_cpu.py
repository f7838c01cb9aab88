"""BSRNet pre-pass (FaithDiff/models/bsrnet_arch.py) -- host side: the fp32 oracle against the
golden vectors the reference module itself produced (tests/golden/make_bsrnet_golden.py), the product's key layout,
weight loading and the test.py image helpers."""
import os

import numpy as np
import pytest
import torch

from oracle import bsrnet as ob

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "bsrnet_golden.npz")


def test_oracle_matches_reference_golden():
    z = np.load(GOLD)
    sd = ob.random_weights(int(z["seed"]), int(z["nb"]))
    with torch.no_grad():
        y = ob.forward(sd, torch.from_numpy(z["x"]), int(z["nb"]))
        y2 = ob.deg_remove(sd, torch.from_numpy(z["x2"]), int(z["nb"]), int(z["tile_size"]), int(z["tile_pad"]))
    assert y.shape == (1, 3, 72, 52) and y2.shape == (1, 3, 84, 56)
    assert torch.allclose(y, torch.from_numpy(z["y"]), rtol=0, atol=1e-6)
    assert torch.allclose(y2, torch.from_numpy(z["y2"]), rtol=0, atol=1e-6)


def test_product_keys_match_reference_layout():
    from fdhip import arch
    for nb in (1, 23):
        assert arch.bsrnet_param_shapes(nb) == ob.param_shapes(nb)
    n = sum(int(np.prod(s)) for s in arch.bsrnet_param_shapes(23).values())
    assert n == 16697987  # RRDBNet(3, 3, 64, 23, 32): the published BSRNet / ESRGAN x4 parameter count


def test_create_bsrnet_loads_weights_only_files(tmp_path):
    from FaithDiff.create_FaithDiff_model import create_bsrnet
    from FaithDiff.models.bsrnet_arch import RRDBNet
    net = create_bsrnet("random-init")
    sd = net.state_dict()
    p = tmp_path / "BSRNet.pth"
    torch.save(sd, p)
    net2 = create_bsrnet(str(p))
    assert all(torch.equal(net2.state_dict()[k], v) for k, v in sd.items())
    bad = dict(sd)
    bad.pop("conv_last.bias")
    with pytest.raises(RuntimeError):
        RRDBNet(nb=23).load_state_dict(bad, strict=True)
    with pytest.raises(NotImplementedError):
        RRDBNet(nf=32)
    with pytest.raises(RuntimeError):  # no CPU execution path
        net.forward(torch.zeros(1, 3, 8, 8))


def test_image_tensor_helpers_roundtrip():
    from utils.image_process import image2tensor, tensor2image
    a = np.random.default_rng(0).integers(0, 256, (7, 5, 3), dtype=np.uint8)
    t = image2tensor(a)
    assert t.shape == (1, 3, 7, 5) and t.dtype == torch.float32
    assert np.array_equal(tensor2image(t), a)
