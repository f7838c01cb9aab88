#!/usr/bin/env python3
"""Per-shape launch table of one C2 UNet forward (B=2, 128x128 latent): every GEMM / conv / flash launch
timed with HIP events (ops.set_probe), grouped by shape.  Prints and writes gpurun_out/shape_table.json."""
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "faithdiff-dev_amd"))
import torch  # noqa: E402


def main():
    from fdhip import arch, ops
    from fdhip import lib as L
    from fdhip.unet import HipUNet
    L.require_device()
    dev = torch.device("cuda", 0)
    k, B = int(os.environ.get("LAT", "128")), 2
    sd = arch.random_init(arch.unet_param_shapes(True), seed=0, device=dev)
    unet = HipUNet(sd, dev, torch.bfloat16)
    del sd
    g = torch.Generator(device=dev).manual_seed(0)
    unet.set_context(torch.randn((2, 77, 2048), generator=g, device=dev))
    x = torch.randn((B * k * k, 4), generator=g, device=dev).to(torch.bfloat16)
    cond = torch.randn((B * k * k, 512), generator=g, device=dev).to(torch.bfloat16)
    t = torch.full((B,), 951.0, device=dev)
    tids = torch.tensor([[1024.0, 1024.0, 0, 0, 1024.0, 1024.0]] * B, device=dev)
    text = torch.randn((B, 1280), generator=g, device=dev)
    ops.reserve_gn_workspace(1 << 24, dev)
    for _ in range(2):
        unet.forward(x, t, tids, text, cond, B, k, k)
    torch.cuda.synchronize()
    reps = 3
    rec = []
    ops.set_probe(rec)
    for _ in range(reps):
        unet.forward(x, t, tids, text, cond, B, k, k)
    ops.set_probe(None)
    torch.cuda.synchronize()
    agg = defaultdict(lambda: [0, 0.0, 0.0])
    for r in rec:
        kind, fl, nb, e0, e1 = r[:5]
        lab = r[5] if len(r) > 5 else kind
        a = agg[lab]
        a[0] += 1
        a[1] += fl
        a[2] += e0.elapsed_time(e1)
    rows = []
    for lab, (n, fl, ms) in agg.items():
        rows.append({"shape": lab, "per_forward": n // reps, "ms_per_forward": ms / reps,
                     "us_per_launch": ms / n * 1e3, "tflops": fl / (ms / 1e3) / 1e12 if ms else 0.0})
    rows.sort(key=lambda r: -r["ms_per_forward"])
    tot = sum(r["ms_per_forward"] for r in rows)
    for r in rows:
        print(f"{r['shape']:60s} x{r['per_forward']:3d} {r['us_per_launch']:8.1f} us {r['ms_per_forward']:7.3f} ms "
              f"{r['tflops']:7.1f} TF/s")
    print(f"total probed ms/forward {tot:.3f}")
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    json.dump(rows, open(os.path.join(ROOT, "gpurun_out", "shape_table.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
