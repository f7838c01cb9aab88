"""BSRNet pre-pass (RRDBNet x4, the ESRGAN generator) restated in fp32 torch on the CPU -- TEST INFRASTRUCTURE ONLY
(the checker for fdhip/bsrnet.py; nothing in the product path imports it).

Follows /root/reference/FaithDiff/models/bsrnet_arch.py:
  * ResidualDenseBlock_5C (:35-58): five 3x3 convs over the growing concat (nf + k*gc channels), LeakyReLU(0.2)
    after the first four, output x5 * 0.2 + x;
  * RRDB (:61-74): three dense blocks, output out * 0.2 + x;
  * RRDBNet.forward (:100-114): zero pad to a multiple of 4 on the right / bottom (check_image_size, :92-98),
    conv_first, trunk of nb RRDBs, trunk_conv, fea + trunk, two (nearest x2 -> conv -> LeakyReLU), HRconv ->
    LeakyReLU -> conv_last, crop to 4H x 4W;
  * deg_remove (:116-175): tiles of tile_size with tile_pad context, each upscaled on its own, the unpadded part
    pasted into a zero image.
Parity of this restatement is pinned by tests/golden/bsrnet_golden.npz, written by running the reference module
itself on the same weights (tests/golden/make_bsrnet_golden.py).  Weights are seeded random (no BSRNet.pth
offline): random_weights() is the one generator the golden script, the CPU tests and the GPU tests share.
"""
import math

import numpy as np
import torch
import torch.nn.functional as F


def param_shapes(nb=23, nf=64, gc=32, in_nc=3, out_nc=3):
    """The reference's state-dict keys and shapes (RRDBNet(in_nc, out_nc, nf, nb, gc, sf=4))."""
    d = {}

    def conv(name, cin, cout):
        d[name + ".weight"] = (cout, cin, 3, 3)
        d[name + ".bias"] = (cout,)
    conv("conv_first", in_nc, nf)
    for i in range(nb):
        for j in (1, 2, 3):
            p = f"RRDB_trunk.{i}.RDB{j}"
            for k in range(1, 5):
                conv(f"{p}.conv{k}", nf + (k - 1) * gc, gc)
            conv(f"{p}.conv5", nf + 4 * gc, nf)
    for n in ("trunk_conv", "upconv1", "upconv2", "HRconv"):
        conv(n, nf, nf)
    conv("conv_last", nf, out_nc)
    return d


def random_weights(seed, nb=23):
    """Seeded fp32 weights in key order: dense-block convs at 0.1 x He-normal (the reference's
    initialize_weights(..., 0.1), :45), the others He-normal / 4; biases N(0, 0.01)."""
    rng = np.random.default_rng(seed)
    sd = {}
    for k, shp in param_shapes(nb).items():
        if k.endswith(".bias"):
            v = rng.standard_normal(shp) * 0.01
        else:
            fan_in = shp[1] * 9
            scale = 0.1 if ".RDB" in k else 0.25
            v = rng.standard_normal(shp) * math.sqrt(2.0 / fan_in) * scale
        sd[k] = torch.from_numpy(v.astype(np.float32))
    return sd


def _conv(x, sd, name):
    return F.conv2d(x, sd[name + ".weight"], sd[name + ".bias"], padding=1)


def _lrelu(x):
    return F.leaky_relu(x, 0.2)


def _rdb(x, sd, p):
    x1 = _lrelu(_conv(x, sd, p + ".conv1"))
    x2 = _lrelu(_conv(torch.cat((x, x1), 1), sd, p + ".conv2"))
    x3 = _lrelu(_conv(torch.cat((x, x1, x2), 1), sd, p + ".conv3"))
    x4 = _lrelu(_conv(torch.cat((x, x1, x2, x3), 1), sd, p + ".conv4"))
    x5 = _conv(torch.cat((x, x1, x2, x3, x4), 1), sd, p + ".conv5")
    return x5 * 0.2 + x


def forward(sd, x, nb):
    """x: NCHW fp32 [B, 3, H, W] -> [B, 3, 4H, 4W]."""
    _, _, H, W = x.shape
    x = F.pad(x, (0, (4 - W % 4) % 4, 0, (4 - H % 4) % 4))
    fea = _conv(x, sd, "conv_first")
    t = fea
    for i in range(nb):
        p = f"RRDB_trunk.{i}"
        o = _rdb(_rdb(_rdb(t, sd, p + ".RDB1"), sd, p + ".RDB2"), sd, p + ".RDB3")
        t = o * 0.2 + t
    fea = fea + _conv(t, sd, "trunk_conv")
    fea = _lrelu(_conv(F.interpolate(fea, scale_factor=2, mode="nearest"), sd, "upconv1"))
    fea = _lrelu(_conv(F.interpolate(fea, scale_factor=2, mode="nearest"), sd, "upconv2"))
    out = _conv(_lrelu(_conv(fea, sd, "HRconv")), sd, "conv_last")
    return out[:, :, :H * 4, :W * 4]


def tiles(height, width, tile_size, tile_pad):
    """deg_remove's tile plan (:129-168): per tile (input box with padding, output box, crop inside the tile)."""
    plan = []
    for ty in range(math.ceil(height / tile_size)):
        for tx in range(math.ceil(width / tile_size)):
            x0, y0 = tx * tile_size, ty * tile_size
            x1, y1 = min(x0 + tile_size, width), min(y0 + tile_size, height)
            px0, px1 = max(x0 - tile_pad, 0), min(x1 + tile_pad, width)
            py0, py1 = max(y0 - tile_pad, 0), min(y1 + tile_pad, height)
            cx0, cy0 = (x0 - px0) * 4, (y0 - py0) * 4
            plan.append(((py0, py1, px0, px1), (y0 * 4, y1 * 4, x0 * 4, x1 * 4),
                         (cy0, cy0 + (y1 - y0) * 4, cx0, cx0 + (x1 - x0) * 4)))
    return plan


def deg_remove(sd, x, nb, tile_size=512, tile_pad=16):
    b, c, h, w = x.shape
    out = x.new_zeros((b, c, h * 4, w * 4))
    for (py0, py1, px0, px1), (oy0, oy1, ox0, ox1), (cy0, cy1, cx0, cx1) in tiles(h, w, tile_size, tile_pad):
        t = forward(sd, x[:, :, py0:py1, px0:px1], nb)
        out[:, :, oy0:oy1, ox0:ox1] = t[:, :, cy0:cy1, cx0:cx1]
    return out
