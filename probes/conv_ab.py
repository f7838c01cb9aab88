"""A/B of the 3x3 convs of the UNet (C2, B = 2) and the 1024^2 VAE decode: the halo-staged kernel (with and without
the folded GroupNorm) against the implicit GEMM (gemm8 / gemm256, FD_CONV_HALO = 0) plus its separate GroupNorm
pass.  Graph-timed (20 replays of 10 launches each); one JSON line per shape."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "faithdiff-dev_amd"))
from fdhip import knobs, ops  # noqa: E402
from fdhip import lib as L  # noqa: E402

knobs.apply_env()
DEV = "cuda"
# (tag, nimg, H, W, Cin, Cout, dtype, upsample, m_ref images)
SHAPES = [("unet128_320", 2, 128, 128, 320, 320, torch.bfloat16, False),
          ("unet128_640to320", 2, 128, 128, 640, 320, torch.bfloat16, False),
          ("unet64_640", 2, 64, 64, 640, 640, torch.bfloat16, False),
          ("unet64_1280to640", 2, 64, 64, 1280, 640, torch.bfloat16, False),
          ("unet32_1280", 2, 32, 32, 1280, 1280, torch.bfloat16, False),
          ("unet32_2560to1280", 2, 32, 32, 2560, 1280, torch.bfloat16, False),
          ("unet32_1920to1280", 2, 32, 32, 1920, 1280, torch.bfloat16, False),
          ("unet32_640to1280", 2, 32, 32, 640, 1280, torch.bfloat16, False),
          ("unet64_1920to640", 2, 64, 64, 1920, 640, torch.bfloat16, False),
          ("unet64_960to640", 2, 64, 64, 960, 640, torch.bfloat16, False),
          ("unet64_320to640", 2, 64, 64, 320, 640, torch.bfloat16, False),
          ("unet128_960to320", 2, 128, 128, 960, 320, torch.bfloat16, False),
          ("unet_up64_1280", 2, 32, 32, 1280, 1280, torch.bfloat16, True),
          ("unet_up128_640", 2, 64, 64, 640, 640, torch.bfloat16, True),
          ("vae128_512", 1, 128, 128, 512, 512, torch.float16, False),
          ("vae256_512", 1, 256, 256, 512, 512, torch.float16, False),
          ("vae512_256", 1, 512, 512, 256, 256, torch.float16, False),
          ("vae1024_128", 1, 1024, 1024, 128, 128, torch.float16, False),
          ("vae_up512_512", 1, 256, 256, 512, 512, torch.float16, True),
          ("vae_up1024_256", 1, 1024, 1024, 256, 256, torch.float16, True),
          ("vae1024_256to128", 1, 1024, 1024, 256, 128, torch.float16, False)]


def graph_us(fn, reps=20, inner=10):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        fn()
    torch.cuda.synchronize()
    with torch.cuda.graph(g, stream=s):
        for _ in range(inner):
            fn()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(reps):
        e0.record()
        g.replay()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3 / inner)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    L.require_device()
    only = sys.argv[1:]
    for tag, n, H, W, Cin, Cout, dt, up in SHAPES:
        if only and tag not in only:
            continue
        g = torch.Generator(device=DEV).manual_seed(0)
        Hi, Wi = (H // 2, W // 2) if up else (H, W)
        x = torch.randn(n * Hi * Wi, Cin, device=DEV, generator=g).to(dt)
        wp = (torch.randn(Cout, 9 * Cin, device=DEV, generator=g) / (9 * Cin) ** 0.5).to(dt)
        b = torch.randn(Cout, device=DEV, generator=g) * 0.1
        gamma = torch.ones(Cin, device=DEV)
        beta = torch.zeros(Cin, device=DEV)
        out = torch.empty(n * H * W, Cout, device=DEV, dtype=dt)
        hn = torch.empty_like(x)
        flops = 2.0 * n * H * W * Cout * 9 * Cin
        rec = {"shape": tag, "M": n * H * W, "N": Cout, "K": 9 * Cin}
        kw = dict(upsample=up) if up else {}
        rec["halo_rows"] = ops.halo_conv_rows(x, wp, n, Hi, Wi, **kw)
        rec["halo_us"] = graph_us(lambda: ops.conv3x3(x, wp, b, n, Hi, Wi, out=out, **kw))
        if not up:
            aff = ops.group_norm_affine(x, gamma, beta, n, Hi * Wi, Cin, 32, 1e-5)
            if rec["halo_rows"]:
                rec["halo_gn_us"] = graph_us(lambda: ops.conv3x3(x, wp, b, n, Hi, Wi, out=out, gn_in=(aff, True)))
            rec["gn_pass_us"] = graph_us(lambda: ops.group_norm(x, gamma, beta, n, Hi * Wi, Cin, 32, 1e-5, silu=True,
                                                                out=hn))
            rec["affine_us"] = graph_us(lambda: ops.group_norm_affine(x, gamma, beta, n, Hi * Wi, Cin, 32, 1e-5))
        with knobs.override(FD_CONV_HALO=0):
            rec["igemm_us"] = graph_us(lambda: ops.conv3x3(x, wp, b, n, Hi, Wi, out=out, **kw))
        rec["halo_tflops"] = round(flops / rec["halo_us"] / 1e6, 1)
        rec["igemm_tflops"] = round(flops / rec["igemm_us"] / 1e6, 1)
        print(json.dumps({k: (round(v, 2) if isinstance(v, float) else v) for k, v in rec.items()}), flush=True)


if __name__ == "__main__":
    main()
