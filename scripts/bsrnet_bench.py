#!/usr/bin/env python3
"""BSRNet pre-pass throughput (test.py:97-101, the published RRDBNet nb = 23 with seeded weights): deg_remove of one
SIZE x SIZE image (default 512: one 512-pixel tile, the reference's tile_size, -> a 2048^2 output), HIP events
around the call after one warm-up.  Algorithmic FLOPs are the reference's convs (2 * Cin * 9 * Cout per output
pixel, unpadded channel counts); the HIP path also multiplies the 32 zero-weight channels of conv2 / conv4.
JSON line out."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "faithdiff-dev_amd"))
import torch  # noqa: E402


def flops(h, w, nb=23):
    per_px = 0
    for k in range(1, 6):
        cin = 64 + (k - 1) * 32
        per_px += 2 * 9 * cin * (32 if k < 5 else 64)
    trunk = (3 * nb * per_px + 2 * 9 * 64 * 64) * h * w + 2 * 9 * 3 * 64 * h * w
    up = 2 * 9 * 64 * 64 * (4 * h * w + 16 * h * w + 16 * h * w) + 2 * 9 * 64 * 3 * 16 * h * w
    return trunk + up


def main():
    from FaithDiff.create_FaithDiff_model import create_bsrnet
    size = int(os.environ.get("SIZE", "512"))
    net = create_bsrnet("random-init").to("cuda")
    x = torch.rand((1, 3, size, size), generator=torch.Generator().manual_seed(0)).cuda()
    net.deg_remove(x)
    torch.cuda.synchronize()
    ts = []
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        y = net.deg_remove(x)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ms = min(ts)
    fl = flops(size, size)
    print(json.dumps({"workload": f"BSRNet deg_remove {size}x{size} -> {4 * size}x{4 * size} (nb 23, fp16)",
                      "ms": round(ms, 2), "algorithmic_tflop": round(fl / 1e12, 3),
                      "achieved_tflops": round(fl / (ms / 1e3) / 1e12, 1), "frac_of_2p5PF": round(fl / (ms / 1e3) / 2.5e15, 4),
                      "finite": bool(torch.isfinite(y).all().item()), "out_shape": list(y.shape)}), flush=True)


if __name__ == "__main__":
    main()
