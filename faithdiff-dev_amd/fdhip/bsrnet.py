"""BSRNet pre-pass (RRDBNet x4, ESRGAN generator) on the HIP kernel library (the degradation-removal
pre-pass test.py:97-101 runs before the LLaVA caption; bsrnet_arch.py:77-175).

Layout: NHWC activations in fp16 (the reference runs fp32; the VAE's storage type here).  Every 3x3 conv with
Cin >= 64 is one implicit-GEMM fd_gemm; conv_first (Cin = 3) is fd_conv2d_direct.

Dense blocks without concatenation copies: each ResidualDenseBlock_5C works in one [H*W, 192] buffer whose column
ranges are x (0:64), x1 (64:96), x2 (96:128), x3 (128:160), x4 (160:192).  conv_k writes its output straight into
its range (a strided output view) and reads the buffer's first Cin_k columns (a strided input: the conv's pixel
stride is 192), so torch.cat((x, x1, ..)) is never formed.  The implicit GEMM needs Cin % 64 == 0, so conv2
(96 inputs) and conv4 (160) read 128 / 192 columns with zero weights on the 32 extra ones -- their own output
range, zeroed before the conv, so a stale value of an earlier block (an fp16 inf would make 0 * inf = NaN) is never
read.  forward() raises FloatingPointError on a non-finite output (fp16 trunk; the reference runs fp32).
LeakyReLU(0.2), the 0.2 residual
scale (alpha = 0.2 with a pre-scaled bias) and the residual add are in the conv epilogue; the RRDB's own
out * 0.2 + x is one fd_axpby.  Nearest x2 upsampling is folded into upconv1 / upconv2's gather.
"""
import math

import torch

from . import lib as L
from . import ops

NF, GC = 64, 32


def _pack(w, cin_pad=None, dtype=torch.float16):
    """[Cout, Cin, 3, 3] -> [Cout, 9 * Cin_pad] tap-major (ops.pack_conv3x3), zero weights for channels >= Cin."""
    co, ci = w.shape[:2]
    wt = w.permute(0, 2, 3, 1)  # [Cout, 3, 3, Cin]
    if cin_pad and cin_pad > ci:
        wt = torch.cat([wt, wt.new_zeros((co, 3, 3, cin_pad - ci))], -1)
    return wt.reshape(co, -1).to(dtype).contiguous()


class HipRRDBNet:
    def __init__(self, sd, nb, device="cuda", dtype=torch.float16):
        L.require_device()
        self.nb, self.device, self.dtype = nb, torch.device(device), dtype
        dev = self.device
        f32 = lambda t: t.to(device=dev, dtype=torch.float32).contiguous()  # noqa: E731
        self.first = (f32(sd["conv_first.weight"].permute(0, 2, 3, 1)), f32(sd["conv_first.bias"]))
        self.rdbs = []
        for i in range(nb):
            blk = []
            for j in (1, 2, 3):
                p = f"RRDB_trunk.{i}.RDB{j}"
                convs = []
                for k in range(1, 6):
                    cin = NF + (k - 1) * GC
                    cp = (cin + 63) // 64 * 64
                    w = sd[f"{p}.conv{k}.weight"].to(dev)
                    b = f32(sd[f"{p}.conv{k}.bias"])
                    if k == 5:
                        b = b * 0.2  # x5 * 0.2 + x: alpha = 0.2 on the accumulator, the bias pre-scaled
                    convs.append((_pack(w, cp, dtype).to(dev), b, cp))
                blk.append(convs)
            self.rdbs.append(blk)
        self.convs = {n: (_pack(sd[n + ".weight"].to(dev), None, dtype), f32(sd[n + ".bias"]))
                      for n in ("trunk_conv", "upconv1", "upconv2", "HRconv", "conv_last")}

    # ------------------------------------------------------------------------------------------------------------
    def _rdb(self, buf, convs, out, H, W):
        """ResidualDenseBlock_5C (bsrnet_arch.py:50-58) on buf[:, 0:64] -> out (a [H*W, 64] view)."""
        ld = buf.stride(0)
        for k, (wp, b, cp) in enumerate(convs[:4]):
            c0 = NF + k * GC
            if cp > c0:  # conv2 / conv4: the padded input columns are this conv's own output range
                buf[:, c0:cp].zero_()
            ops.conv3x3(buf[:, :cp], wp, b, 1, H, W, out=buf[:, c0:c0 + GC], act="lrelu", lda=ld)
        wp, b, cp = convs[4]
        ops.conv3x3(buf[:, :cp], wp, b, 1, H, W, out=out, residual=buf[:, :NF], alpha=0.2, lda=ld)

    @torch.no_grad()
    def forward(self, x):
        """x: NCHW fp32 [1, 3, H, W] on the device (the reference's RRDBNet.forward, :100-114) -> [1, 3, 4H, 4W]."""
        if x.dim() != 4 or x.shape[0] != 1 or x.shape[1] != 3:
            raise ValueError(f"BSRNet expects a [1, 3, H, W] image, got {tuple(x.shape)}")
        _, _, H, W = x.shape
        Hp, Wp = H + (4 - H % 4) % 4, W + (4 - W % 4) % 4  # check_image_size: zero pad right / bottom (:92-98)
        dev, dt = self.device, self.dtype
        xp = torch.zeros((1, 3, Hp, Wp), device=dev, dtype=torch.float32)
        xp[:, :, :H, :W] = x.to(dev, torch.float32)
        HW = Hp * Wp
        xn = torch.empty((HW, 3), device=dev, dtype=dt)
        ops.nchw_to_nhwc(xp, xn, 1, 3, HW)
        fea = ops.conv_direct(xn, *self.first, 1, Hp, Wp, 3, 3, 1, 1, out_dtype=dt)  # [HW, 64]
        # three dense-block buffers rotate: RDB1 a -> b, RDB2 b -> c, RDB3 c -> b[:, :64], RRDB residual into b
        bufs = [torch.zeros((HW, 192), device=dev, dtype=dt) for _ in range(3)]
        a, b, c = bufs
        ops.add_strided(fea, NF, None, 0, a, a.stride(0), HW, NF)
        for blk in self.rdbs:
            self._rdb(a, blk[0], b[:, :NF], Hp, Wp)
            self._rdb(b, blk[1], c[:, :NF], Hp, Wp)
            self._rdb(c, blk[2], b[:, :NF], Hp, Wp)
            ops.axpby(b[:, :NF], a[:, :NF], b[:, :NF], 0.2, 1.0)  # RRDB: out * 0.2 + x (:72-76)
            a, b = b, a
        wp, bb = self.convs["trunk_conv"]
        fea = ops.conv3x3(a[:, :NF], wp, bb, 1, Hp, Wp, residual=fea, lda=a.stride(0))  # fea + trunk
        wp, bb = self.convs["upconv1"]
        h = ops.conv3x3(fea, wp, bb, 1, Hp, Wp, upsample=True, act="lrelu")
        wp, bb = self.convs["upconv2"]
        h = ops.conv3x3(h, wp, bb, 1, 2 * Hp, 2 * Wp, upsample=True, act="lrelu")
        wp, bb = self.convs["HRconv"]
        h = ops.conv3x3(h, wp, bb, 1, 4 * Hp, 4 * Wp, act="lrelu")
        wp, bb = self.convs["conv_last"]
        y = ops.conv3x3(h, wp, bb, 1, 4 * Hp, 4 * Wp)  # [16 HW, 3]
        out = torch.empty((1, 3, 4 * Hp, 4 * Wp), device=dev, dtype=torch.float32)
        ops.nhwc_to_nchw(y, out, 1, 3, 16 * HW)
        if not bool(torch.isfinite(out).all()):
            raise FloatingPointError("BSRNet: non-finite output (fp16 trunk overflow)")
        return out[:, :, :4 * H, :4 * W]

    @torch.no_grad()
    def deg_remove(self, x, tile_size=512, tile_pad=16):
        """bsrnet_arch.py:116-175: tiles of tile_size (tile_pad context each side, clipped at the border) upscaled
        one by one, the unpadded part pasted into a zero image."""
        b, c, h, w = x.shape
        x = x.to(self.device, torch.float32)
        out = torch.zeros((b, c, h * 4, w * 4), device=self.device, dtype=torch.float32)
        for ty in range(math.ceil(h / tile_size)):
            for tx in range(math.ceil(w / tile_size)):
                x0, y0 = tx * tile_size, ty * tile_size
                x1, y1 = min(x0 + tile_size, w), min(y0 + tile_size, h)
                px0, px1 = max(x0 - tile_pad, 0), min(x1 + tile_pad, w)
                py0, py1 = max(y0 - tile_pad, 0), min(y1 + tile_pad, h)
                t = self.forward(x[:, :, py0:py1, px0:px1])
                cx0, cy0 = (x0 - px0) * 4, (y0 - py0) * 4
                out[:, :, y0 * 4:y1 * 4, x0 * 4:x1 * 4] = t[:, :, cy0:cy0 + (y1 - y0) * 4, cx0:cx0 + (x1 - x0) * 4]
        return out
