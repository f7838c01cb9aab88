#!/usr/bin/env python3
"""BASELINE configs[3] in its literal reading: a 7680x4320 input upscaled x4 (LANCZOS, as
test_wo_llava.py:78-82 does) to 30720x17280, restored with the use_fp8 UNet on the e4m3 MFMA, tiled VAE encode /
decode and the tiled denoise encoder -- 1947 TLC tiles of the 3840x2160 latent.  One denoise step (the loop's
per-step cost is what the 225-tile 8K-output bench measures at 20 steps); reports the tile count, per-stage times,
finiteness of the final latents and the output image's size and pixel std.  Prints a heartbeat every 30 s.

    python scripts/c4_literal.py [--steps 1] [--lr 7680x4320]
"""
import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "faithdiff-dev_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402  (the product factory, synthetic input and event timer the bench uses)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--lr", default="7680x4320")
    args = ap.parse_args()
    w0, h0 = (int(v) for v in args.lr.split("x"))
    t_start = time.perf_counter()
    stop = threading.Event()

    def beat():
        while not stop.wait(30):
            print(f"... {time.perf_counter() - t_start:.0f} s", flush=True)
    threading.Thread(target=beat, daemon=True).start()

    from fdhip import knobs
    from fdhip import lib as L
    from FaithDiff.pipelines.tlc import TileGrid
    applied = knobs.apply_env()  # A/B runs (FD_TILE_BATCH ...); reported in the result line
    from PIL import Image
    L.require_device()
    dev = torch.device("cuda", 0)
    pipe = bench.build_pipe(dev, fp8=True)
    lr = bench.synthetic_image(h0, w0, 9)
    W, H = 4 * w0, 4 * h0
    img = lr.resize((W, H), Image.LANCZOS)
    ntiles = TileGrid(H // 8, W // 8, (128, 128), 0.5).ntiles
    print(f"input {w0}x{h0} -> x4 {W}x{H}, latent {W // 8}x{H // 8}, {ntiles} TLC tiles; setup "
          f"{time.perf_counter() - t_start:.0f} s", flush=True)
    pipe.enable_vae_tiling()
    tm = bench.EventTimer()
    gen = torch.Generator(device=dev).manual_seed(42)
    last = {}

    def keep(p, i, t, kw):
        last["lat"] = kw["latents"]
        return {}
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tm("call_start", 0)
    out = pipe(lr_img=img, prompt="A high quality photo restored from a degraded capture.", negative_prompt="",
               num_inference_steps=args.steps, guidance_scale=5.0, generator=gen, start_point="lr", height=H,
               width=W, overlap=0.5, target_size=(1024, 1024), timer=tm, callback_on_step_end=keep)
    tm("call_end", 0)
    torch.cuda.synchronize()
    s = time.perf_counter() - t0
    stop.set()
    im = out.images[0] if hasattr(out, "images") else out[0][0]
    arr = np.asarray(im)
    st = tm.step_ms()
    res = {"workload": f"C4 literal: {w0}x{h0} x4 -> {W}x{H}, {ntiles} TLC tiles x {args.steps} Euler step(s), "
                       "use_fp8 (e4m3 MFMA Linears), tiled VAE encode/decode + tiled denoise encoder",
           "ntiles": ntiles, "steps": args.steps, "s_total": round(s, 2),
           "pre_loop_s": round(tm.span_ms("call_start", "loop_start") / 1e3, 2),
           "step_s": [round(v / 1e3, 2) for v in st],
           "tile_steps_per_s": round(ntiles * len(st) / (sum(st) / 1e3), 2) if st else None,
           "decode_s": round(tm.span_ms("decode_start", "decode") / 1e3, 2),
           "latents_finite": bool(torch.isfinite(last["lat"]).all().item()) if "lat" in last else None,
           "image_size": list(arr.shape), "image_std": round(float(arr.std()), 2),
           "peak_gpu_gb": round(torch.cuda.max_memory_allocated(dev) / 2 ** 30, 1), "knobs": applied}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
