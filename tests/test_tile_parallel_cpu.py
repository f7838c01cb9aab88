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


def _vae_tiles_and_weights_worker(rank, world, port, q):
    """map_tiles (the sharded tiled VAE decode / encode exchange) and broadcast_state_dict under gloo."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from FaithDiff.pipelines.tile_parallel import broadcast_state_dict
        from fdhip.tiling import map_tiles
        specs = [(i, j, th, tw, th * tw) for i, th in ((0, 7), (5, 3)) for j, tw in ((0, 8), (6, 5), (9, 2))]

        def fn(i, j, th, tw):  # a tile "decode": deterministic in its coordinates, ragged sizes
            g = torch.Generator().manual_seed(100 * i + j)
            return torch.randn(th * tw, 3, generator=g)

        tiles = map_tiles(specs, fn, 3, "cpu", torch.float32, dist.group.WORLD)
        # ranks start from different weights; after the broadcast all hold rank 0's
        g = torch.Generator().manual_seed(rank)
        sd = {"a.weight": torch.randn(5, 7, generator=g), "b.bias": torch.randn(3, generator=g),
              "c.idx": torch.arange(4) + rank, "d.half": torch.randn(6, generator=g).half()}
        broadcast_state_dict(sd, None, 0, "cpu", bucket_bytes=64)
        # numpy (pickled by value): torch tensors would travel as shared-memory handles that die with the worker
        q.put((rank, [t.numpy().copy() for t in tiles], {k: v.numpy().copy() for k, v in sd.items()}))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_vae_tiles_and_weight_broadcast(world):
    from fdhip.tiling import map_tiles
    specs = [(i, j, th, tw, th * tw) for i, th in ((0, 7), (5, 3)) for j, tw in ((0, 8), (6, 5), (9, 2))]

    def fn(i, j, th, tw):
        g = torch.Generator().manual_seed(100 * i + j)
        return torch.randn(th * tw, 3, generator=g)

    ref = map_tiles(specs, fn, 3, "cpu", torch.float32, None)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_vae_tiles_and_weights_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in procs], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    sd0 = res[0][2]
    for rank, tiles, sd in res:
        assert len(tiles) == len(ref) and all((a == b.numpy()).all() for a, b in zip(tiles, ref)), rank
        assert all((sd[k] == sd0[k]).all() for k in sd0), rank
    g = torch.Generator().manual_seed(0)
    assert (sd0["a.weight"] == torch.randn(5, 7, generator=g).numpy()).all()


@pytest.mark.parametrize("world,h,w", [(2, 160, 224), (3, 160, 224), (4, 64, 128)])
def test_tile_parallel_bitwise_equals_single_rank(world, h, w):
    """160x224: 4 x 6 = 24 tiles of 64x64; 64x128: 3 tiles over 4 ranks -- the last rank's shard is empty (as rank 7
    of the 49-tile C3 image on 8 GPUs): it still joins every all-gather and blends the same canvas."""
    steps = 3
    ref, shard1 = _loop(h, w, steps, None)
    assert shard1.count == shard1.ntiles
    res = _run(world, h, w, steps)
    covered = sorted((b, c) for _, _, b, c in res)
    assert sum(c for _, c in covered) == shard1.ntiles
    for rank, out, begin, count in res:
        assert (out == ref.numpy()).all(), f"rank {rank} canvas differs"


def _seeded_pipeline_worker(rank, world, port, q):
    """FaithDiff_pipeline('random-init', seed=rank): the ranks start from different weights; enable_tile_parallel
    makes them rank 0's before anything is packed."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import zlib
        from CKPT_PTH import FAITHDIFF_PATH, SDXL_PATH, VAE_FP16_PATH
        from FaithDiff.create_FaithDiff_model import FaithDiff_pipeline
        pipe = FaithDiff_pipeline(SDXL_PATH, VAE_FP16_PATH, FAITHDIFF_PATH, seed=rank)
        before = zlib.crc32(pipe.unet._sd["conv_in.weight"].numpy())
        pipe.enable_tile_parallel()
        dig = {}
        for name, m in pipe._weight_owners():
            if m is not None:
                dig[name] = {k: zlib.crc32(v.contiguous().view(torch.uint8).numpy()) for k, v in m._sd.items()}
        q.put((rank, before, dig, pipe.last_broadcast_bytes, pipe.vae.process_group is not None))
    finally:
        dist.destroy_process_group()


def test_enable_tile_parallel_broadcasts_rank0_weights():
    """SURVEY 8(e) "RCCL broadcast of weights" through the product surface, gloo world 2 on CPU: ranks built from
    different seeds hold bitwise rank 0's UNet (+ extras), VAE, denoise encoder and both text encoders after
    pipe.enable_tile_parallel() (the GPU leg, tests/test_tile_parallel_gpu.py, then checks the canvases)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_seeded_pipeline_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=600) for _ in procs], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    (_, b0, d0, n0, t0), (_, b1, d1, n1, t1) = res
    assert b0 != b1, "the ranks were meant to start from different weights"
    assert set(d0) == {"unet", "vae", "denoise_encoder", "text_encoder", "text_encoder_2"}
    assert d0 == d1 and n0 == n1 > 10e9 and t0 and t1


def _release_worker(rank, world, port, q):
    """broadcast_weights on a bare pipeline whose components hold small host state dicts; rank 1 has released
    its UNet weights.  Every rank must raise (a collective agreement first), none may block in the broadcast."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from types import SimpleNamespace

        from FaithDiff.pipelines.pipeline_FaithDiff_tlc import FaithDiffStableDiffusionXLPipeline as P
        pipe = object.__new__(P)
        unet = SimpleNamespace(_sd={} if rank == 1 else {"w": torch.full((4,), float(rank))})
        vae = SimpleNamespace(_sd={"v": torch.full((3,), float(rank))})
        pipe._weight_owners = lambda: [("unet", unet), ("vae", vae)]
        pipe._weights_group = None
        try:
            pipe.broadcast_weights(dist.group.WORLD)
            q.put((rank, "no error"))
        except RuntimeError as e:
            q.put((rank, "raised" if "released" in str(e) else str(e)))
        # sync_weights=False: no transfer (each rank keeps its own, e.g. identical checkpoint loads)
        unet._sd = {"w": torch.full((4,), float(rank))}
        pipe.vae = pipe.denoise_encoder = None
        pipe.enable_tile_parallel(sync_weights=False)
        q.put((rank, float(unet._sd["w"][0])))
    finally:
        dist.destroy_process_group()


def test_broadcast_weights_released_raises_on_every_rank_and_sync_opt_out():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_release_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(4)], key=lambda r: (r[0], isinstance(r[1], float)))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert res == [(0, "raised"), (0, 0.0), (1, "raised"), (1, 1.0)]
