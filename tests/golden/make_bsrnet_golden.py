"""Golden vectors for the BSRNet pre-pass from the reference's own module (FaithDiff/models/bsrnet_arch.py,
plain torch: loaded by file path, no stubs needed).  Run in the build container only (the reference is not on the
GPU box):
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_bsrnet_golden.py

RRDBNet(nb=2) with oracle.bsrnet.random_weights(seed=3, nb=2) loaded strictly; writes inputs and outputs only
(tests/golden/bsrnet_golden.npz):
  * forward on a 1 x 3 x 18 x 13 image (odd sizes: the zero pad to a multiple of 4 and the crop, :92-114);
  * deg_remove on a 1 x 3 x 21 x 14 image with tile_size 8, tile_pad 2 (3 x 2 tiles, clipped padding, :116-175).
"""
import contextlib
import importlib.util
import io
import os
import sys

import numpy as np
import torch

REF = "/root/reference/FaithDiff/models/bsrnet_arch.py"
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
from oracle.bsrnet import random_weights  # noqa: E402

SEED, NB = 3, 2


def main():
    spec = importlib.util.spec_from_file_location("ref_bsrnet_arch", REF)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    with contextlib.redirect_stdout(io.StringIO()):  # the constructor prints its arguments
        net = mod.RRDBNet(in_nc=3, out_nc=3, nf=64, nb=NB, gc=32, sf=4)
    net.load_state_dict(random_weights(SEED, NB), strict=True)
    net.eval()
    g = torch.Generator().manual_seed(11)
    x = torch.rand((1, 3, 18, 13), generator=g)
    x2 = torch.rand((1, 3, 21, 14), generator=g)
    with torch.no_grad():
        y = net(x)
        y2 = net.deg_remove(x2, tile_size=8, tile_pad=2)
    out = os.path.join(HERE, "bsrnet_golden.npz")
    np.savez_compressed(out, seed=SEED, nb=NB, x=x.numpy(), y=y.numpy(), x2=x2.numpy(), y2=y2.numpy(),
                        tile_size=8, tile_pad=2)
    print("wrote", out, y.shape, y2.shape, float(y.abs().mean()), float(y2.abs().mean()))


if __name__ == "__main__":
    main()
