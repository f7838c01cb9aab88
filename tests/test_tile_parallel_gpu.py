"""The product pipeline's tile-parallel path (``pipe.enable_tile_parallel()``) with real process
groups on the GPU: the TLC tiles of one image sharded over ranks, one all-gather per step, the sharded tiled VAE
decode -- against the same pipeline without a process group.  The output must be bitwise identical (the blend is
in tile order on every rank, and a tile's UNet rows do not depend on which other tiles share its forward).

  * world 1 on RCCL ('nccl'), in this process;
  * world 2 on one GPU: two spawned ranks on cuda:0 under gloo (RCCL refuses two ranks on one device; the
    collectives are host-staged, fdhip/comm.py), each computing half of the tiles.
Reference loop: pipeline_FaithDiff_tlc.py:1324-1409 (tiles), :1436-1442 (decode).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

H, W, TARGET, STEPS = 768, 512, (512, 512), 2  # 96 x 64 latent: 6 TLC tiles of 64 x 64


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _pipe(seed=1):
    from CKPT_PTH import FAITHDIFF_PATH, SDXL_PATH, VAE_FP16_PATH
    from FaithDiff.create_FaithDiff_model import FaithDiff_pipeline
    pipe = FaithDiff_pipeline(SDXL_PATH, VAE_FP16_PATH, FAITHDIFF_PATH, seed=seed, init_device="cuda").to("cuda:0")
    # small VAE tiles so the decode is tiled (and sharded) at this size: 4 x 3 latent tiles of 32
    vae = pipe.vae
    vae.tile_sample_min_size, vae.tile_latent_min_size = 256, 32
    pipe.enable_vae_tiling()
    pipe.tile_batch = 4
    return pipe


def _inputs():
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
    from _det import det_tensor, synthetic_degraded
    img = synthetic_degraded(H, W, 8)
    return img, det_tensor((1, 4, H // 8, W // 8), 31), det_tensor((1, 4, H // 8, W // 8), 32)


def _call(pipe, output_type):
    img, noise, post = _inputs()
    captured = {}

    def cb(p, i, t, kw):
        captured["lat"] = kw["latents"].detach().float().cpu().clone()
        return {}

    out = pipe(lr_img=img, prompt="A sharp photo of a tiled floor", negative_prompt="", num_inference_steps=STEPS,
               guidance_scale=5.0, start_point="lr", height=H, width=W, overlap=0.5, target_size=TARGET,
               latents=noise, posterior_noise=post, callback_on_step_end=cb, output_type=output_type).images
    img_out = np.asarray(out[0]) if output_type == "pil" else None
    return captured["lat"].numpy(), img_out


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # the ranks start from DIFFERENT random weights (seed 1 and 8): enable_tile_parallel broadcasts rank 0's
        # (broadcast_weights) before anything is packed, so both must reproduce the seed-1 single-process run
        pipe = _pipe(seed=1 + 7 * rank)
        pipe.enable_tile_parallel()
        nbytes = pipe.last_broadcast_bytes
        lat, img = _call(pipe, "pil")
        q.put((rank, lat, img, nbytes))
    finally:
        dist.destroy_process_group()


_REF = {}


def _reference():
    if "r" not in _REF:
        pipe = _pipe()
        _REF["pipe"] = pipe
        _REF["r"] = _call(pipe, "pil")
    return _REF["pipe"], _REF["r"]


def test_call_tile_parallel_rccl_world1_bitwise():
    pipe, (lat_ref, img_ref) = _reference()
    store = dist.TCPStore("127.0.0.1", _free_port(), 1, True)
    dist.init_process_group("nccl", store=store, rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        pipe.enable_tile_parallel()
        lat, img = _call(pipe, "pil")
    finally:
        pipe.process_group = None
        pipe.vae.process_group = pipe.denoise_encoder.process_group = None
        dist.destroy_process_group()
    assert (lat == lat_ref).all()
    assert (img == img_ref).all()


def test_call_tile_parallel_two_ranks_one_gpu_bitwise():
    pipe, (lat_ref, img_ref) = _reference()
    # graph replay vs eager forwards inside the same call must agree bitwise too (HipUNet.run)
    unet = pipe.unet.hip()
    unet.graphs.enabled = False
    try:
        lat_eager, _ = _call(pipe, "latent")
    finally:
        unet.graphs.enabled = True
    assert (lat_eager == lat_ref).all()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in procs], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    for rank, lat, img, nbytes in res:
        assert nbytes > 10e9, f"rank {rank}: only {nbytes} bytes broadcast"
        assert (lat == lat_ref).all(), f"rank {rank}: latents differ from the single-process run"
        assert (img == img_ref).all(), f"rank {rank}: image differs from the single-process run"


def test_c3_49_tiles_tile_batch_bitwise():
    """BASELINE configs[2] shape on the GPU: a 4096^2 input restored at target 1024 (latent 512^2 -> 49 TLC tiles,
    tiled VAE encode / decode and tiled denoise encoder at their default 1024-px tiles), one Euler step, through
    the product __call__.  The tiles are batched 25 (the default: 25 + 24) and 4 per UNet forward: every latent and pixel must be equal
    (a tile's rows never depend on which tiles share its forward; m_ref keeps the kernel choices per tile)."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
    from _det import det_tensor, synthetic_degraded
    pipe, _ = _reference()
    vae = pipe.vae
    saved = (vae.tile_sample_min_size, vae.tile_latent_min_size, pipe.tile_batch)
    vae.tile_sample_min_size, vae.tile_latent_min_size = 1024, 128
    S = 4096
    img = synthetic_degraded(S, S, 9)
    noise, post = det_tensor((1, 4, S // 8, S // 8), 41), det_tensor((1, 4, S // 8, S // 8), 42)
    res = []
    try:
        for tb in (25, 4):
            pipe.tile_batch = tb
            cap = {}

            def cb(p, i, t, kw):
                cap["lat"] = kw["latents"].detach().float().cpu().clone()
                return {}
            out = pipe(lr_img=img, prompt="a tiled floor", negative_prompt="", num_inference_steps=1,
                       guidance_scale=5.0, start_point="lr", height=S, width=S, overlap=0.5,
                       target_size=(1024, 1024), latents=noise, posterior_noise=post, callback_on_step_end=cb,
                       output_type="pil").images
            res.append((cap["lat"], np.asarray(out[0])))
    finally:
        vae.tile_sample_min_size, vae.tile_latent_min_size, pipe.tile_batch = saved
    assert res[0][0].shape == (1, 4, 512, 512) and res[0][1].shape == (S, S, 3)
    assert torch.equal(res[0][0], res[1][0])
    assert (res[0][1] == res[1][1]).all()
    assert res[0][1].std() > 1.0
