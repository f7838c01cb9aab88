#!/usr/bin/env python3
"""The reference's examples/band.png through test_wo_llava.py's whole flow at its default upscale 4 (:18-97): convert
('RGB'), x4 LANCZOS (4316x3112), check_image_size (4320x3112: a 540x389 latent, 48 TLC tiles), the product
``pipe(...)`` with the script's defaults (20 Euler steps, CFG 5, target 1024, overlap 0.5, start 'lr'), crop and adain
colour fix.  The caption (LLaVA, out of scope) is replaced by seeded prompt embeddings (tests/golden/_det.py
band_inputs).  Prints one JSON line: wall time of the pipe() call, its loop / decode split, finiteness and pixel
statistics; writes the colour-fixed PNG to gpurun_out/band_x4.png.  (The reference's script itself cannot run on the
GPU box: /root/reference is not there; scripts/run_dropin.py runs it where it is.)"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "faithdiff-dev_amd"), os.path.join(ROOT, "tests", "golden"), ROOT):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    from _det import band_inputs
    from CKPT_PTH import FAITHDIFF_PATH, SDXL_PATH, VAE_FP16_PATH
    from FaithDiff.create_FaithDiff_model import FaithDiff_pipeline
    from utils.color_fix import adain_color_fix
    sys.path.insert(0, ROOT)
    from bench import EventTimer
    c = band_inputs(4, steps=20)
    pipe = FaithDiff_pipeline(SDXL_PATH, VAE_FP16_PATH, FAITHDIFF_PATH, seed=0, init_device="cuda").to("cuda:0")
    kw = dict(prompt_embeds=c["pe"], negative_prompt_embeds=c["npe"], pooled_prompt_embeds=c["ppe"],
              negative_pooled_prompt_embeds=c["nppe"], guidance_scale=5.0, start_point="lr", height=c["H"],
              width=c["W"], overlap=0.5, target_size=(1024, 1024), latents=c["noise"], posterior_noise=c["post"])
    pipe(lr_img=c["img"], num_inference_steps=2, **kw)  # warm: graphs captured
    last = {}
    tm = EventTimer()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tm("call_start", 0)
    out = pipe(lr_img=c["img"], num_inference_steps=20, timer=tm,
               callback_on_step_end=lambda p, i, t, k: last.update(lat=k["latents"]) or {}, **kw).images[0]
    tm("call_end", 0)
    torch.cuda.synchronize()
    s = time.perf_counter() - t0
    fixed = adain_color_fix(out.crop((0, 0, c["w0"], c["h0"])), c["image"])
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    fixed.save(os.path.join(ROOT, "gpurun_out", "band_x4.png"))
    st = tm.step_ms()
    a = np.asarray(out)
    print(json.dumps({"workload": "band.png x4 (test_wo_llava.py defaults): 4320x3112, 540x389 latent, 48 TLC tiles, "
                                  "20 Euler steps, CFG 5, start 'lr', untiled VAE",
                      "s_per_image": round(s, 3), "loop_s": round(sum(st) / 1e3, 3),
                      "tile_steps_per_s": round(48 * 20 / (sum(st) / 1e3), 2),
                      "pre_loop_ms": round(tm.span_ms("call_start", "loop_start"), 1),
                      "decode_ms": round(tm.span_ms("decode_start", "decode"), 1),
                      "latents_finite": bool(torch.isfinite(last["lat"]).all().item()),
                      "image": list(a.shape), "pixel_std": round(float(a.std()), 3),
                      "colour_fixed": list(fixed.size)}))


if __name__ == "__main__":
    main()
