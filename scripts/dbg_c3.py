#!/usr/bin/env python3
"""Debug: C3-shape one-step pipeline calls with different tile batches; reports NaN / equality."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "faithdiff-dev_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from _det import det_tensor, synthetic_degraded  # noqa: E402
from CKPT_PTH import FAITHDIFF_PATH, SDXL_PATH, VAE_FP16_PATH  # noqa: E402
from FaithDiff.create_FaithDiff_model import FaithDiff_pipeline  # noqa: E402

S = int(os.environ.get("DBG_S", "4096"))
pipe = FaithDiff_pipeline(SDXL_PATH, VAE_FP16_PATH, FAITHDIFF_PATH, seed=1, init_device="cuda").to("cuda:0")
pipe.enable_vae_tiling()
img = synthetic_degraded(S, S, 9)
noise, post = det_tensor((1, 4, S // 8, S // 8), 41), det_tensor((1, 4, S // 8, S // 8), 42)
res = []
for tb in [int(x) for x in os.environ.get("DBG_TB", "13,4").split(",")]:
    pipe.tile_batch = tb
    if os.environ.get("DBG_CLEAR") == "1":
        pipe.unet.hip().graphs.clear()
    if os.environ.get("DBG_CLEAR") == "vae":
        pipe.vae.decoder_hip().graphs.clear()
    cap = {}

    def cb(p, i, t, kw):
        cap["lat"] = kw["latents"].detach().float().cpu().clone()
        return {}
    pipe(lr_img=img, prompt="a tiled floor", negative_prompt="", num_inference_steps=1, guidance_scale=5.0,
         start_point="lr", height=S, width=S, overlap=0.5, target_size=(1024, 1024), latents=noise,
         posterior_noise=post, callback_on_step_end=cb, output_type="latent")
    lat = cap["lat"]
    nanm = torch.isnan(lat[0, 0])
    rows = torch.nonzero(nanm.any(1)).flatten()
    cols = torch.nonzero(nanm.any(0)).flatten()
    print(f"tb={tb} nan={int(nanm.sum())} rows={rows.min().item() if len(rows) else None}..{rows.max().item() if len(rows) else None} "
          f"cols={cols.min().item() if len(cols) else None}..{cols.max().item() if len(cols) else None}", flush=True)
    res.append(lat)
for i in range(1, len(res)):
    print("equal to first:", torch.equal(res[0], res[i]), flush=True)
