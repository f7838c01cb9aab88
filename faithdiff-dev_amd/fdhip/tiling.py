"""Tiled VAE decode / encode and the FaithDiff tiled denoise encoder on HIP.

Semantics (reproduced, including the in-place blending order):
  * AutoencoderKL.tiled_decode (diffusers 0.28): latent tiles of tile_latent_min_size (128) every
    int(128 * (1 - overlap)) = 96 latents; each tile post_quant_conv + decoder; blend_extent =
    int(1024 * overlap) = 256 px; crop to row_limit = 1024 - 256 = 768 px.
  * AutoencoderKL.tiled_encode: pixel tiles of 1024 every int(1024 * (1 - overlap)) = 768 px; encoder +
    quant_conv; blend_extent = int(128 * overlap) = 32 latents; crop 96.
  * FaithDiff Encoder.tiled_encode (ext:164-190): as tiled_encode but the trunk only (512 ch).
Blending is the reference's recurrence: tile (i, j) is first blended (in place) with the already-final
tile above, then with the already-final tile to its left (blend_v / blend_h), then cropped.  Every
per-element step is a device kernel (fd_blend_edge, strided copies); only the tile bookkeeping is host.
"""
import math

import torch
import torch.distributed as dist

from . import ops
from .comm import all_gather_into


def map_tiles(specs, fn, C, device, dtype, group=None):
    """Run fn(*spec[:-1]) -> [spec[-1] rows, C] for every tile spec, in tile order.  With a process group of G
    ranks (the tiles of a tiled VAE decode / encode are independent), rank r computes the
    contiguous shard [r*ceil(N/G), ...) into row-padded slots and ONE all_gather_into_tensor (RCCL over xGMI on
    the GPUs) hands every rank every tile; the blend that follows is then the same on all ranks, bit for bit."""
    world = dist.get_world_size(group) if group is not None else 1
    if world == 1:
        return [fn(*s[:-1]) for s in specs]
    rank = dist.get_rank(group)
    n = len(specs)
    per = math.ceil(n / world)
    begin = min(rank * per, n)
    count = max(0, min(n, begin + per) - begin)
    maxr = max(s[-1] for s in specs)
    local = torch.zeros((per, maxr, C), dtype=dtype, device=device)
    for k in range(count):
        s = specs[begin + k]
        local[k, :s[-1]].copy_(fn(*s[:-1]))
    buf = torch.empty((world * per, maxr, C), dtype=dtype, device=device)
    all_gather_into(buf, local, group)
    return [buf[t, :specs[t][-1]] for t in range(n)]


def _crop(src, H, W, C, i, j, th, tw):
    out = torch.empty((th * tw, C), dtype=src.dtype, device=src.device)
    base = src[(i * W + j):]  # view starting at row i, column j
    ops.copy_2d(base, W * C, out, tw * C, th, tw * C)
    return out


def _assemble(rows, C, blend, limit, out_h, out_w, device, dtype):
    """rows[i][j] = (tile NHWC tensor, Ht, Wt); blends in place in the reference order and writes the
    cropped tiles into one NHWC [out_h * out_w, C] canvas."""
    out = torch.empty((out_h * out_w, C), dtype=dtype, device=device)
    y0 = 0
    for i, row in enumerate(rows):
        x0 = 0
        rh = 0
        for j, (t, Ht, Wt) in enumerate(row):
            if i > 0:
                a, Ha, Wa = rows[i - 1][j]
                ops.blend_edge(a, t, Ha, Wa, Ht, Wt, C, blend, True)
            if j > 0:
                a, Ha, Wa = row[j - 1]
                ops.blend_edge(a, t, Ha, Wa, Ht, Wt, C, blend, False)
            ch, cw = min(limit, Ht), min(limit, Wt)
            ops.copy_2d(t, Wt * C, out[(y0 * out_w + x0):], out_w * C, ch, cw * C)
            x0 += cw
            rh = ch
        y0 += rh
    return out


def tiled_vae_decode(vae, z, h, w, group=None):
    """z: NHWC [h*w, 4] (already / scaling_factor) -> NHWC [8h * 8w, 3].  group: shard the tiles (map_tiles)."""
    tl, ts, f = vae.tile_latent_min_size, vae.tile_sample_min_size, vae.tile_overlap_factor
    overlap, blend, limit = int(tl * (1 - f)), int(ts * f), ts - int(ts * f)
    dec = vae.decoder_hip()
    grid = [[(i, j, min(tl, h - i), min(tl, w - j)) for j in range(0, w, overlap)] for i in range(0, h, overlap)]
    specs = [(i, j, th, tw, 64 * th * tw) for row in grid for (i, j, th, tw) in row]
    # decode_graphed returns the graph's static buffer: copy each tile out before the next replay
    outs = map_tiles(specs, lambda i, j, th, tw: dec.decode_graphed(_crop(z, h, w, 4, i, j, th, tw), 1, th, tw).clone(),
                     3, z.device, z.dtype, group)
    it = iter(outs)
    rows = [[(next(it), 8 * th, 8 * tw) for (_, _, th, tw) in row] for row in grid]
    return _assemble(rows, 3, blend, limit, 8 * h, 8 * w, z.device, z.dtype)


def _tiled_encode(encode_fn, x, H, W, C_out, ts, tl, f, group=None):
    overlap, blend, limit = int(ts * (1 - f)), int(tl * f), tl - int(tl * f)
    grid = [[(i, j, min(ts, H - i), min(ts, W - j)) for j in range(0, W, overlap)] for i in range(0, H, overlap)]
    specs = [(i, j, th, tw, (th // 8) * (tw // 8)) for row in grid for (i, j, th, tw) in row]
    outs = map_tiles(specs, lambda i, j, th, tw: encode_fn(_crop(x, H, W, 3, i, j, th, tw), th, tw), C_out,
                     x.device, x.dtype, group)
    it = iter(outs)
    rows = [[(next(it), th // 8, tw // 8) for (_, _, th, tw) in row] for row in grid]
    # output extent: the cropped tiles tile the latent exactly when 8 * limit == overlap; otherwise
    # (the reference's quirk at non-default settings) the concatenation defines the size.
    out_h = sum(min(limit, r[0][1]) for r in rows)
    out_w = sum(min(limit, t[2]) for t in rows[0])
    return _assemble(rows, C_out, blend, limit, out_h, out_w, x.device, x.dtype)


def tiled_vae_encode(vae, x, H, W, group=None):
    """x: NHWC [H*W, 3] -> moments NHWC [(H/8)*(W/8), 8] (quant_conv output)."""
    enc = vae.encoder_hip()
    return _tiled_encode(lambda t, th, tw: enc.encode_graphed(t, 1, th, tw).clone(), x, H, W, 8,
                         vae.tile_sample_min_size,
                         vae.tile_latent_min_size, vae.tile_overlap_factor, group)


def tiled_encoder_forward(encoder, x, H, W, group=None):
    """FaithDiff Encoder.tiled_encode (ext:164-190): x NHWC [H*W, 3] -> [(H/8)*(W/8), 512]."""
    enc = encoder.hip()
    return _tiled_encode(lambda t, th, tw: enc.encode_graphed(t, 1, th, tw).clone(), x, H, W, 512,
                         encoder.tile_sample_min_size,
                         encoder.tile_latent_min_size, encoder.tile_overlap_factor, group)
