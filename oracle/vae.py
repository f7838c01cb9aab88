"""fp32 CPU restatement of AutoencoderKL (sdxl-vae-fp16-fix) and the FaithDiff denoise ``Encoder``.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

  * ``Encoder`` (FaithDiff denoise_encoder) ... unet_2d_condition_vae_extension.py:39-196
    - trunk = conv_in + 4 DownEncoderBlock2D + UNetMidBlock2D, NO conv_norm_out/conv_out (ext:122-148)
    - ``tiled_encode`` / ``blend_v`` / ``blend_h`` (ext:150-190); ``forward`` tiles when the
      *pixel* size exceeds ``tile_latent_min_size`` (ext:192-196).
  * ``AutoencoderKL`` per SURVEY App. B.2: encoder (+conv_norm_out, conv_out 512->8), quant_conv,
    post_quant_conv, decoder (up blocks 512,512,256,128 x 3 resnets), GN eps 1e-6,
    mid attention 1 head d=512 with residual.  latent_dist: mean/logvar, logvar clamp [-30, 20].
Key names are diffusers'.
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from .unet import ResnetBlock2D, Downsample2D, Upsample2D, Attention


class VAEAttention(Attention):
    """Mid-block attention: group_norm -> q,k,v (bias) -> SDPA (1 head, d=512) -> to_out -> +residual."""

    def __init__(self, ch=512):
        super().__init__(ch, heads=1, dim_head=ch, bias=True, out_bias=True, group_norm_groups=32, eps=1e-6)

    def forward(self, x):  # x NCHW
        B, C, H, W = x.shape
        res = x
        h = self.group_norm(x).view(B, C, H * W).transpose(1, 2)
        h = super().forward(h)
        return h.transpose(1, 2).reshape(B, C, H, W) + res


class VAEMidBlock(nn.Module):
    def __init__(self, ch=512):
        super().__init__()
        self.resnets = nn.ModuleList([ResnetBlock2D(ch, ch, None, eps=1e-6), ResnetBlock2D(ch, ch, None, eps=1e-6)])
        self.attentions = nn.ModuleList([VAEAttention(ch)])

    def forward(self, x):
        x = self.resnets[0](x)
        x = self.attentions[0](x)
        return self.resnets[1](x)


class DownEncoderBlock2D(nn.Module):
    def __init__(self, cin, cout, add_downsample):
        super().__init__()
        self.resnets = nn.ModuleList([ResnetBlock2D(cin if i == 0 else cout, cout, None, eps=1e-6) for i in range(2)])
        self.downsamplers = nn.ModuleList([Downsample2D(cout, padding=0)]) if add_downsample else None

    def forward(self, x):
        for r in self.resnets:
            x = r(x)
        if self.downsamplers is not None:
            x = self.downsamplers[0](x)
        return x


class UpDecoderBlock2D(nn.Module):
    def __init__(self, cin, cout, add_upsample):
        super().__init__()
        self.resnets = nn.ModuleList([ResnetBlock2D(cin if i == 0 else cout, cout, None, eps=1e-6) for i in range(3)])
        self.upsamplers = nn.ModuleList([Upsample2D(cout)]) if add_upsample else None

    def forward(self, x):
        for r in self.resnets:
            x = r(x)
        if self.upsamplers is not None:
            x = self.upsamplers[0](x)
        return x


VAE_CHANNELS = (128, 256, 512, 512)


class EncoderTrunk(nn.Module):
    def __init__(self, with_out=True):
        super().__init__()
        ch = VAE_CHANNELS
        self.conv_in = nn.Conv2d(3, ch[0], 3, padding=1)
        blocks, prev = [], ch[0]
        for i, c in enumerate(ch):
            blocks.append(DownEncoderBlock2D(prev, c, i < len(ch) - 1))
            prev = c
        self.down_blocks = nn.ModuleList(blocks)
        self.mid_block = VAEMidBlock(ch[-1])
        if with_out:
            self.conv_norm_out = nn.GroupNorm(32, ch[-1], eps=1e-6)
            self.conv_out = nn.Conv2d(ch[-1], 8, 3, padding=1)
        else:
            self.conv_norm_out = None
            self.conv_out = None

    def encode(self, x):
        x = self.conv_in(x)
        for b in self.down_blocks:
            x = b(x)
        x = self.mid_block(x)
        if self.conv_out is not None:
            x = self.conv_out(F.silu(self.conv_norm_out(x)))
        return x


class Decoder(nn.Module):
    def __init__(self):
        super().__init__()
        rch = tuple(reversed(VAE_CHANNELS))
        self.conv_in = nn.Conv2d(4, rch[0], 3, padding=1)
        self.mid_block = VAEMidBlock(rch[0])
        blocks, prev = [], rch[0]
        for i, c in enumerate(rch):
            blocks.append(UpDecoderBlock2D(prev, c, i < len(rch) - 1))
            prev = c
        self.up_blocks = nn.ModuleList(blocks)
        self.conv_norm_out = nn.GroupNorm(32, rch[-1], eps=1e-6)
        self.conv_out = nn.Conv2d(rch[-1], 3, 3, padding=1)

    def forward(self, z):
        x = self.conv_in(z)
        x = self.mid_block(x)
        for b in self.up_blocks:
            x = b(x)
        return self.conv_out(F.silu(self.conv_norm_out(x)))


def _blend_v(a, b, e):
    e = min(a.shape[2], b.shape[2], e)
    for y in range(e):
        b[:, :, y, :] = a[:, :, -e + y, :] * (1 - y / e) + b[:, :, y, :] * (y / e)
    return b


def _blend_h(a, b, e):
    e = min(a.shape[3], b.shape[3], e)
    for x in range(e):
        b[:, :, :, x] = a[:, :, :, -e + x] * (1 - x / e) + b[:, :, :, x] * (x / e)
    return b


def _tiled(x, fn, step, size, blend, limit):
    """diffusers tiled_encode / tiled_decode skeleton (0.28): tiles every `step`, in-place blends in
    row-major order, crop to `limit`."""
    rows = []
    for i in range(0, x.shape[2], step):
        rows.append([fn(x[:, :, i:i + size, j:j + size]) for j in range(0, x.shape[3], step)])
    out_rows = []
    for i, row in enumerate(rows):
        out = []
        for j, tile in enumerate(row):
            if i > 0:
                tile = _blend_v(rows[i - 1][j], tile, blend)
            if j > 0:
                tile = _blend_h(row[j - 1], tile, blend)
            out.append(tile[:, :, :limit, :limit])
        out_rows.append(torch.cat(out, dim=3))
    return torch.cat(out_rows, dim=2)


class AutoencoderKL(nn.Module):
    """diffusers AutoencoderKL (sdxl-vae-fp16-fix config); use_tiling -> tiled_encode / tiled_decode with
    tile_sample_min_size = sample_size (1024), tile_latent_min_size = 128, overlap 0.25."""
    scaling_factor = 0.13025

    def __init__(self):
        super().__init__()
        self.encoder = EncoderTrunk(with_out=True)
        self.decoder = Decoder()
        self.quant_conv = nn.Conv2d(8, 8, 1)
        self.post_quant_conv = nn.Conv2d(4, 4, 1)
        self.use_tiling = False
        self.tile_sample_min_size = 1024
        self.tile_latent_min_size = 128
        self.tile_overlap_factor = 0.25

    def encode_moments(self, x):
        if self.use_tiling and (x.shape[-1] > self.tile_sample_min_size or x.shape[-2] > self.tile_sample_min_size):
            ts, tl, f = self.tile_sample_min_size, self.tile_latent_min_size, self.tile_overlap_factor
            return _tiled(x, lambda t: self.quant_conv(self.encoder.encode(t)), int(ts * (1 - f)), ts, int(tl * f),
                          tl - int(tl * f))
        return self.quant_conv(self.encoder.encode(x))

    def encode_sample(self, x, eps):
        """latent_dist.sample() with the N(0,1) draw ``eps`` passed in explicitly."""
        m = self.encode_moments(x)
        mean, logvar = m.chunk(2, dim=1)
        logvar = logvar.clamp(-30.0, 20.0)
        return mean + torch.exp(0.5 * logvar) * eps

    def decode(self, z):
        if self.use_tiling and (z.shape[-1] > self.tile_latent_min_size or z.shape[-2] > self.tile_latent_min_size):
            ts, tl, f = self.tile_sample_min_size, self.tile_latent_min_size, self.tile_overlap_factor
            return _tiled(z, lambda t: self.decoder(self.post_quant_conv(t)), int(tl * (1 - f)), tl, int(ts * f),
                          ts - int(ts * f))
        return self.decoder(self.post_quant_conv(z))


class DenoiseEncoder(EncoderTrunk):
    """FaithDiff ``Encoder`` (ext:39-196): trunk only, optional tiled encode."""

    def __init__(self):
        super().__init__(with_out=False)
        self.tile_sample_min_size = 1024
        self.tile_latent_min_size = int(self.tile_sample_min_size / 8)
        self.tile_overlap_factor = 0.25
        self.use_tiling = False

    @staticmethod
    def blend_v(a, b, blend_extent):  # ext:150-155
        blend_extent = min(a.shape[2], b.shape[2], blend_extent)
        for y in range(blend_extent):
            b[:, :, y, :] = a[:, :, -blend_extent + y, :] * (1 - y / blend_extent) + b[:, :, y, :] * (y / blend_extent)
        return b

    @staticmethod
    def blend_h(a, b, blend_extent):  # ext:157-162
        blend_extent = min(a.shape[3], b.shape[3], blend_extent)
        for x in range(blend_extent):
            b[:, :, :, x] = a[:, :, :, -blend_extent + x] * (1 - x / blend_extent) + b[:, :, :, x] * (x / blend_extent)
        return b

    def tiled_encode(self, x):  # ext:164-190
        overlap_size = int(self.tile_sample_min_size * (1 - self.tile_overlap_factor))
        blend_extent = int(self.tile_latent_min_size * self.tile_overlap_factor)
        row_limit = self.tile_latent_min_size - blend_extent
        rows = []
        for i in range(0, x.shape[2], overlap_size):
            row = []
            for j in range(0, x.shape[3], overlap_size):
                row.append(self.encode(x[:, :, i:i + self.tile_sample_min_size, j:j + self.tile_sample_min_size]))
            rows.append(row)
        result_rows = []
        for i, row in enumerate(rows):
            out = []
            for j, tile in enumerate(row):
                if i > 0:
                    tile = self.blend_v(rows[i - 1][j], tile, blend_extent)
                if j > 0:
                    tile = self.blend_h(row[j - 1], tile, blend_extent)
                out.append(tile[:, :, :row_limit, :row_limit])
            result_rows.append(torch.cat(out, dim=3))
        return torch.cat(result_rows, dim=2)

    def forward(self, x):  # ext:192-196
        if self.use_tiling and (x.shape[-1] > self.tile_latent_min_size or x.shape[-2] > self.tile_latent_min_size):
            return self.tiled_encode(x)
        return self.encode(x)
