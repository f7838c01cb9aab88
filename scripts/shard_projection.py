#!/usr/bin/env python3
"""Project the 8-GPU tile split of C3 / C4 from ONE GPU.  A projection, not a multi-GPU
measurement: no RCCL collective runs here.

The product's tile-parallel loop (FaithDiff/pipelines/tile_parallel.py TileShard: contiguous ceil(N / G) shards)
gives rank r of G the tiles [r * per, min(N, (r + 1) * per)), and the rank batches its shard into UNet forwards of
at most FD_TILE_BATCH (25) tiles in equal batches (tlc.tile_batches(count, 25, balance=True)).  The step of the
slowest rank (rank 0: the largest shard) bounds the job, then ONE all_gather_into_tensor of G * per fp32 tile
outputs (4 x 128 x 128 x 4 B = 256 KiB per tile) per step.

Here, on one GPU, every forward size that any rank's batching produces is timed through the product path
(HipUNet.run: the same hipGraph replay __call__ uses, cond_embedded, CFG pairs) plus the per-batch CFG + Euler and
the blend of all N tiles, and each rank's step is the sum over its batches.  Reported per (config, G): per-rank
ms/step (max over ranks), the projected job steps/s and tile-steps/s, the efficiency against G x the one-GPU rate,
and the padded all-gather bytes per step (its time is NOT measured: no multi-GPU box).

    python scripts/shard_projection.py [--out gpurun_out/shard_projection.json] [--reps 10]
"""
import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "faithdiff-dev_amd"))

import torch  # noqa: E402

import bench  # noqa: E402

CONFIGS = {"c3": dict(ntiles=49, fp8=False, desc="4096^2 image, 49 TLC tiles of 128^2, bf16 UNet"),
           "c4": dict(ntiles=225, fp8=True, desc="8192^2 output (8K-output reading), 225 tiles, e4m3-MFMA UNet")}
GS = (1, 2, 4, 8)
TILE_BYTES = 4 * 128 * 128 * 4


def shards(n, g):
    per = math.ceil(n / g)
    return per, [max(0, min(n, (r + 1) * per) - r * per) for r in range(g)]


def time_forward(unet, n, k, reps, dev):
    """ms per HipUNet.run of n tiles (2n CFG rows), graph-replayed, cond_embedded (as __call__'s loop)."""
    from fdhip import ops
    B = 2 * n
    g = torch.Generator(device=dev).manual_seed(100 + n)
    x = torch.randn((B * k * k, 4), generator=g, device=dev).to(unet.dtype)
    t = torch.full((B,), 951.0, device=dev)
    tids = torch.tensor([[1024, 1024, 0, 0, 1024, 1024]] * B, dtype=torch.float32, device=dev)
    text = torch.randn((B, 1280), generator=g, device=dev)
    ie = torch.randn((B * k * k, 320), generator=g, device=dev).to(unet.dtype)
    with ops.tile_groups(n):
        for _ in range(3):  # eager, capture, replay
            unet.run(x, t, tids, text, ie, B, k, k, cond_embedded=True)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            unet.run(x, t, tids, text, ie, B, k, k, cond_embedded=True)
        e1.record()
        torch.cuda.synchronize()
    unet.graphs.clear()
    return e0.elapsed_time(e1) / reps


def time_glue(ntiles, n, k, reps, dev):
    """ms of one batch's CFG + Euler (n tiles) and of the blend of all ntiles (per step, every rank)."""
    from fdhip import ops
    from FaithDiff.pipelines.tlc import TileGrid
    side = {49: 512, 225: 1024}[ntiles]
    grid = TileGrid(side, side, (k, k), 0.5)
    assert grid.ntiles == ntiles
    rows = torch.tensor(grid.rows, dtype=torch.int32, device=dev)
    cols = torch.tensor(grid.cols, dtype=torch.int32, device=dev)
    w = torch.tensor(grid.weights(), dtype=torch.float64, device=dev)
    canvas = torch.randn((4, side, side), device=dev)
    nxt = torch.empty_like(canvas)
    eps = torch.randn((2 * n * k * k, 4), device=dev).to(torch.bfloat16)
    tiles = torch.randn((ntiles, 4, k, k), device=dev)

    def cfg_euler():
        ops.tlc_cfg_euler_step(eps, canvas, rows, cols, side, side, k, k, 0, n, 2, 5.0, 0.0, 11.0, 10.0, tiles[:n])

    def blend():
        ops.tlc_blend(tiles, w, rows, cols, 4, side, side, k, k, nxt)
    out = []
    for fn in (cfg_euler, blend):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        out.append(e0.elapsed_time(e1) / reps)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "shard_projection.json"))
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--configs", default="c3,c4")
    args = ap.parse_args()
    from fdhip import knobs
    from fdhip import lib as L
    from FaithDiff.pipelines.tlc import tile_batches
    L.require_device()
    dev = torch.device("cuda", 0)
    tb = knobs.default("FD_TILE_BATCH")
    res = {"what": "one-GPU projection of the contiguous-shard tile split (tile_parallel.TileShard) at G = 1, 2, 4, 8; "
                   "per-rank step = sum of the product's graph-replayed UNet forwards over the rank's balanced tile "
                   "batches + their CFG/Euler launches + the all-tile blend; the all-gather is NOT timed",
           "tile_batch": tb, "configs": {}}
    for name in args.configs.split(","):
        cfg = CONFIGS[name]
        N = cfg["ntiles"]
        t0 = time.perf_counter()
        pipe = bench.build_pipe(dev, fp8=cfg["fp8"])
        unet = pipe.unet.hip()
        g = torch.Generator(device=dev).manual_seed(7)
        unet.set_context(torch.randn((2, 77, 2048), generator=g, device=dev))
        plan = {G: shards(N, G) for G in GS}
        sizes = sorted({n for G in GS for c in plan[G][1] for _, n in tile_batches(c, tb, True) if c})
        fwd = {}
        for n in sizes:
            fwd[n] = time_forward(unet, n, 128, args.reps, dev)
            print(f"{name}: forward of {n} tiles {fwd[n]:.2f} ms ({fwd[n] / n:.3f} ms/tile)", flush=True)
        glue = {n: time_glue(N, n, 128, args.reps, dev) for n in sizes}
        rows = []
        base = None
        for G in GS:
            per, counts = plan[G]
            rank_ms = []
            for c in counts:
                bs = tile_batches(c, tb, True) if c else []
                ms = sum(fwd[n] + glue[n][0] for _, n in bs) + glue[sizes[0]][1]
                rank_ms.append(ms)
            step = max(rank_ms)
            sps = 1e3 / step
            if G == 1:
                base = sps
            rows.append({"G": G, "tiles_per_rank": counts, "per": per,
                         "batches_rank0": [n for _, n in tile_batches(counts[0], tb, True)],
                         "rank_ms_per_step": [round(v, 2) for v in rank_ms], "ms_per_step": round(step, 2),
                         "steps_per_s": round(sps, 3), "tile_steps_per_s": round(sps * N, 1),
                         "efficiency_vs_G_x_1gpu": round(sps / (G * base), 3),
                         "all_gather_bytes_per_step": G * per * TILE_BYTES if G > 1 else 0})
            print(json.dumps(rows[-1]), flush=True)
        res["configs"][name] = {"desc": cfg["desc"], "ntiles": N,
                                "forward_ms": {str(n): round(v, 3) for n, v in fwd.items()},
                                "cfg_euler_ms": {str(n): round(v[0], 4) for n, v in glue.items()},
                                "blend_ms": round(glue[sizes[0]][1], 4), "projection": rows,
                                "wall_s": round(time.perf_counter() - t0, 1)}
        del unet, pipe
        torch.cuda.empty_cache()
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
