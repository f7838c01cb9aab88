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


def _dtype_of(name):
    return getattr(torch, name.split(".")[-1])


def broadcast_state_dict(sd, group=None, src=0, device=None, bucket_bytes=256 << 20):
    """Make every rank's weights rank `src`'s, in place, and return the bytes broadcast (weights go
    out once over RCCL/xGMI instead of every rank reading the checkpoint; create_FaithDiff_model.py:13-22 loads
    them per process).  Rank `src` first broadcasts a manifest (key, dtype, shape); a receiving rank allocates
    whatever it lacks or holds with another dtype / shape (it may start from an empty dict, having read nothing)
    and drops keys the source does not have.  The tensors then go through `device` (the rank's GPU under RCCL,
    the CPU under gloo) in flat buckets of one dtype, in sorted key order, so every rank issues the same
    collectives."""
    if group is None and (not dist.is_initialized() or dist.get_world_size() == 1):
        return 0
    src_global = dist.get_global_rank(group, src) if group is not None else src
    me = dist.get_rank(group)
    keys = sorted(k for k, v in sd.items() if torch.is_tensor(v))
    man = [[(k, str(sd[k].dtype), tuple(sd[k].shape)) for k in keys] if me == src else None]
    mdev = device if device is not None and torch.device(device).type == "cuda" else None
    dist.broadcast_object_list(man, src=src_global, group=group, device=mdev)
    if me != src:
        where = next((v.device for v in sd.values() if torch.is_tensor(v)), torch.device("cpu"))
        want = {k: (_dtype_of(dt), shp) for k, dt, shp in man[0]}
        for k in [k for k in sd if k not in want]:
            del sd[k]
        for k, (dt, shp) in want.items():
            v = sd.get(k)
            if not torch.is_tensor(v) or v.dtype != dt or tuple(v.shape) != tuple(shp):
                sd[k] = torch.empty(shp, dtype=dt, device=where)
        keys = sorted(want)
    by_dtype, total = {}, 0
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
                total += flat.numel() * flat.element_size()
                off = 0
                for b in bucket:
                    n = sd[b].numel()
                    sd[b].copy_(flat[off:off + n].view_as(sd[b]).to(sd[b].device))
                    off += n
                bucket, nbytes = [], 0
    return total


def staging_device(group=None):
    """Where broadcast_state_dict stages its buckets: the rank's GPU under RCCL ('nccl'), the host under gloo."""
    if dist.get_backend(group) == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def run_tile_loop(nsteps, shard, tile_shape, compute, blend, device, dtype=torch.float32, on_step=None, timer=None):
    """Returns the final canvas.  tile_shape = (4, kh, kw).  timer(label, i) (a measurement hook, e.g. bench.py's
    EventTimer) brackets each step's exchange with "gather_start" / "gather_end" when the tiles are sharded."""
    local = torch.zeros((shard.per,) + tuple(tile_shape), dtype=dtype, device=device)
    buf = torch.empty((shard.world * shard.per,) + tuple(tile_shape), dtype=dtype, device=device) \
        if shard.world > 1 else None
    canvas = None
    for i in range(nsteps):
        if shard.count:
            compute(i, shard.begin, shard.count, local)
        if timer is not None and shard.world > 1:
            timer("gather_start", i)
        tiles = shard.gather(local, buf)
        if timer is not None and shard.world > 1:
            timer("gather_end", i)
        canvas = blend(tiles)
        if on_step is not None:
            on_step(i, canvas)
    return canvas
