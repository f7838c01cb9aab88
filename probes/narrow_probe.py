"""Graph-timed conv_out (128 -> 3 at 1024^2, fp16): the implicit GEMM, the narrow strip kernel, and the narrow
kernel with GroupNorm + SiLU folded (one JSON line each)."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "faithdiff-dev_amd"))
sys.path.insert(0, os.path.join(ROOT, "probes"))
from conv_ab import graph_us  # noqa: E402
from fdhip import knobs, ops  # noqa: E402
from fdhip import lib as L  # noqa: E402

knobs.apply_env()


def main():
    L.require_device()
    H = W = int(os.environ.get("NP_HW", "1024"))
    dev, dt = "cuda", torch.float16
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(H * W, 128, device=dev, generator=g).to(dt)
    w = torch.randn(3, 128, 3, 3, device=dev, generator=g) / 34.0
    b = torch.randn(3, device=dev, generator=g) * 0.1
    w32 = ops.pack_conv3x3(w).float()
    wp = ops.pack_conv3x3(w).to(dt)
    gamma, beta = torch.ones(128, device=dev), torch.zeros(128, device=dev)
    aff = ops.group_norm_affine(x, gamma, beta, 1, H * W, 128, 32, 1e-6)
    out = torch.empty(H * W, 3, device=dev, dtype=dt)
    r = {"HW": H, "gemm_us": graph_us(lambda: ops.conv3x3(x, wp, b, 1, H, W)),
         "narrow_us": graph_us(lambda: ops.conv3x3_narrow(x, w32, b, 1, H, W, out=out)),
         "narrow_gn_us": graph_us(lambda: ops.conv3x3_narrow(x, w32, b, 1, H, W, out=out, gn_in=(aff, True))),
         "gn_pass_us": graph_us(lambda: ops.group_norm(x, gamma, beta, 1, H * W, 128, 32, 1e-6, silu=True))}
    print(json.dumps({k: round(v, 2) if isinstance(v, float) else v for k, v in r.items()}), flush=True)


if __name__ == "__main__":
    main()
