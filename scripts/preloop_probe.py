#!/usr/bin/env python3
"""Where the pre-loop part of a C2 pipe(...) call goes: each stage of __call__ before the denoise loop run on its
own (second call, graphs warm), host wall time with a device synchronize after each stage.  JSON line out."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "faithdiff-dev_amd"))
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    pipe = bench.build_pipe(dev, False)
    img = bench.synthetic_image(1024, 1024, 5)
    bench.run_pipeline_image(pipe, img, 1024, 1024, 2, (1024, 1024))
    unet = pipe.unet.hip()
    res = {}

    def stage(name, fn, reps=3):
        best = 1e30
        out = None
        for _ in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            out = fn()
            torch.cuda.synchronize()
            best = min(best, (time.perf_counter() - t0) * 1e3)
        res[name] = round(best, 3)
        return out

    stage("encode_prompt", lambda: pipe.encode_prompt("A high quality photo restored from a degraded capture.",
                                                      do_classifier_free_guidance=True, negative_prompt=""))
    x = stage("preprocess", lambda: pipe._preprocess(img, 1024, 1024))
    stage("denoise_encoder", lambda: pipe.denoise_encoder.encode_nhwc(x, 1024, 1024))
    stage("vae_encode_moments", lambda: pipe.vae.encode_moments_nhwc(x, 1024, 1024))
    ctx = torch.randn((2, 77, 2048), device=dev)
    stage("set_context", lambda: unet.set_context(ctx))
    cond = torch.randn((2 * 128 * 128, 512), device=dev).to(unet.dtype)
    stage("cond_embed", lambda: unet.cond_embed(cond, 2, 128, 128))
    s, tm = bench.run_pipeline_image(pipe, img, 1024, 1024, 20, (1024, 1024))
    res["pipe_s"] = round(s, 4)
    res["pre_loop_ms_events"] = round(tm.span_ms("call_start", "loop_start"), 2)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
