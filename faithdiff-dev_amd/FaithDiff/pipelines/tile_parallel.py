"""Tile-parallel TLC denoise loop across the GPUs of one node.

The reference runs every latent tile of every step sequentially on one GPU (pipeline:1330-1376) and
blends them (grids_inverse, :1409) before the next step re-grids (:1326): tiles are independent
*within* a step but coupled *across* steps.  Here tile t is owned by rank t // ceil(N / G) (contiguous
shards), each rank runs its tiles (several per UNet forward), then ONE all_gather_into_tensor of the
fp32 tile outputs (N x 4 x 128 x 128 x 4 B: 3.2 MB at 49 tiles) over RCCL/xGMI, and every rank applies
the same in-order fp32 blend, so the canvas is bitwise identical on every rank and for every G.

The loop is written against two callables so that the exchange/blend logic is testable on CPU with
gloo (tests/test_tile_parallel_cpu.py) and runs on HIP kernels + RCCL on the GPU box:
  compute(step, tile_begin, ntiles, out) -- writes fp32 [ntiles, 4, kh, kw] tile outputs of a step
  blend(all_tiles) -> canvas           -- the grids_inverse of the full tile set
"""
import math

import torch
import torch.distributed as dist

from fdhip.comm import all_gather_into, broadcast  # noqa: F401  (re-exported for the pipeline)


class TileShard:
    def __init__(self, ntiles, group=None):
        self.group = group
        self.world = dist.get_world_size(group) if group is not None else 1
        self.rank = dist.get_rank(group) if group is not None else 0
        self.ntiles = ntiles
        self.per = math.ceil(ntiles / self.world)
        self.begin = min(self.rank * self.per, ntiles)
        self.count = max(0, min(ntiles, self.begin + self.per) - self.begin)

    def gather(self, local, buf):
        """local: [per, ...] (first `count` rows valid); buf: [world*per, ...].  Returns the first N rows."""
        if self.world == 1:
            return local[:self.ntiles]
        all_gather_into(buf, local, self.group)
        return buf[:self.ntiles]


def broadcast_state_dict(sd, group=None, src=0, device=None, bucket_bytes=256 << 20):
    """Make every rank's weights rank `src`'s, in place (weights broadcast once over RCCL/xGMI,
    instead of every rank reading the checkpoint; with same-seed random init it is a no-op consistency pass).
    Tensors go through `device` (the rank's GPU under RCCL, CPU under gloo) in flat buckets of one dtype, in
    sorted key order, so every rank issues the same collectives."""
    if group is None and (not dist.is_initialized() or dist.get_world_size() == 1):
        return sd
    src_global = dist.get_global_rank(group, src) if group is not None else src
    keys = sorted(k for k, v in sd.items() if torch.is_tensor(v))
    by_dtype = {}
    for k in keys:
        by_dtype.setdefault(sd[k].dtype, []).append(k)
    for dt in sorted(by_dtype, key=str):
        bucket, nbytes = [], 0
        for k in by_dtype[dt] + [None]:
            if k is not None:
                bucket.append(k)
                nbytes += sd[k].numel() * sd[k].element_size()
            if bucket and (k is None or nbytes >= bucket_bytes):
                flat = torch.cat([sd[b].reshape(-1) for b in bucket]).to(device or sd[bucket[0]].device)
                broadcast(flat, src_global, group)
                off = 0
                for b in bucket:
                    n = sd[b].numel()
                    sd[b].copy_(flat[off:off + n].view_as(sd[b]).to(sd[b].device))
                    off += n
                bucket, nbytes = [], 0
    return sd


def run_tile_loop(nsteps, shard, tile_shape, compute, blend, device, dtype=torch.float32, on_step=None):
    """Returns the final canvas.  tile_shape = (4, kh, kw)."""
    local = torch.zeros((shard.per,) + tuple(tile_shape), dtype=dtype, device=device)
    buf = torch.empty((shard.world * shard.per,) + tuple(tile_shape), dtype=dtype, device=device) \
        if shard.world > 1 else None
    canvas = None
    for i in range(nsteps):
        if shard.count:
            compute(i, shard.begin, shard.count, local)
        tiles = shard.gather(local, buf)
        canvas = blend(tiles)
        if on_step is not None:
            on_step(i, canvas)
    return canvas
