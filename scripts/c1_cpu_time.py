#!/usr/bin/env python3
"""C1 CPU timing (BASELINE.json configs[0]: test_wo_llava.py's single 512x512 tile, 4-step Euler, random-init SDXL in
fp32 on the CPU): the fp32 oracle pipeline (oracle/pipeline.py:run_pipeline, test infrastructure -- the reference
itself cannot run here, diffusers is absent) on the C2 recipe's seeded weights and inputs at 512x512, one tile,
4 steps, CFG 5, start_point 'lr'.  Prints one JSON line: s/image, per-step seconds, threads.

    python scripts/c1_cpu_time.py            (THREADS=<n> to pin the thread count)"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "faithdiff-dev_amd"), os.path.join(ROOT, "tests", "golden")):
    sys.path.insert(0, p)

from _det import det_tensor, synthetic_degraded  # noqa: E402
from make_c2_golden import oracle_models  # noqa: E402


def main():
    from oracle.pipeline import run_pipeline
    threads = int(os.environ.get("THREADS", os.cpu_count() or 8))
    torch.set_num_threads(threads)
    H = W = 512
    img = np.asarray(synthetic_degraded(H, W, 2), dtype=np.uint8)
    x = torch.from_numpy(img.astype(np.float32) / 255.0 * 2 - 1).permute(2, 0, 1)[None].contiguous()
    pe, npe = det_tensor((1, 77, 2048), 9101), det_tensor((1, 77, 2048), 9102)
    ppe, nppe = det_tensor((1, 1280), 9103), det_tensor((1, 1280), 9104)
    noise, post = det_tensor((1, 4, H // 8, W // 8), 9105), det_tensor((1, 4, H // 8, W // 8), 9106)
    t_load = time.time()
    ru, rv, re_ = oracle_models(0)
    t_load = time.time() - t_load
    steps = []

    def cb(i, lat):
        steps.append(time.time())

    t0 = time.time()
    with torch.no_grad():
        ref = run_pipeline(ru, rv, re_, x, pe, npe, ppe, nppe, noise, post, num_inference_steps=4, guidance_scale=5.0,
                           overlap=0.5, target_size=(1024, 1024), original_size=(H, W), start_point="lr",
                           step_callback=cb)
    total = time.time() - t0
    st = [b - a for a, b in zip(steps, steps[1:])]
    print(json.dumps({"config": "C1 512x512, one tile, 4 Euler steps, CFG 5, fp32 oracle on CPU", "threads": threads,
                      "cpu": open("/proc/cpuinfo").read().split("model name")[1].split("\n")[0].strip(" :\t"),
                      "s_per_image": round(total, 2), "step_s_median": round(float(np.median(st)), 2) if st else None,
                      "weights_load_s": round(t_load, 1), "latents_finite": bool(torch.isfinite(ref["latents"]).all())}))


if __name__ == "__main__":
    main()
