"""Multi-rank TLC tile sharding (FaithDiff/pipelines/tile_parallel.py) on CPU with gloo, world size 2 and 3.

The per-tile compute is a cheap deterministic stand-in (a nonlinear function of the tile and the step
index, reading the current canvas like the real step does), and the blend is the oracle's
grids_inverse: the point is the exchange -- shard ownership, the all-gather and the in-order blend --
which must give a canvas bitwise identical to the single-rank run for every world size.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _loop(h, w, steps, group):
    from FaithDiff.pipelines.tile_parallel import TileShard, run_tile_loop
    from FaithDiff.pipelines.tlc import TileGrid
    from oracle.tlc import LocalAttention
    grid = TileGrid(h, w, (64, 64), 0.5)
    la = LocalAttention((64, 64), 0.5)
    g = torch.Generator().manual_seed(0)
    state = {"cv": torch.randn(1, 4, h, w, generator=g)}
    la.grids(state["cv"])  # sets idxes / weights
    shard = TileShard(grid.ntiles, group)

    def compute(i, begin, count, out):
        for t in range(count):
            r, c = grid.origin(begin + t)
            x = state["cv"][0, :, r:r + grid.kh, c:c + grid.kw]
            out[t] = torch.tanh(x * (1.0 + 0.1 * i)) + 0.01 * (begin + t)

    def blend(tiles):
        state["cv"] = la.grids_inverse(tiles)
        return state["cv"]

    return run_tile_loop(steps, shard, (4, grid.kh, grid.kw), compute, blend, "cpu"), shard


def _worker(rank, world, port, h, w, steps, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        out, shard = _loop(h, w, steps, dist.group.WORLD)
        q.put((rank, out.numpy(), shard.begin, shard.count))
    finally:
        dist.destroy_process_group()


def _run(world, h, w, steps):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, h, w, steps, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return sorted(res, key=lambda r: r[0])


@pytest.mark.parametrize("world", [2, 3])
def test_tile_parallel_bitwise_equals_single_rank(world):
    h, w, steps = 160, 224, 3  # 4 x 6 = 24 tiles of 64x64
    ref, shard1 = _loop(h, w, steps, None)
    assert shard1.count == shard1.ntiles
    res = _run(world, h, w, steps)
    covered = sorted((b, c) for _, _, b, c in res)
    assert sum(c for _, c in covered) == shard1.ntiles
    for rank, out, begin, count in res:
        assert (out == ref.numpy()).all(), f"rank {rank} canvas differs"
