#!/usr/bin/env python3
"""Time a few GEMM shapes under the current FD_GEMM_* env (one process per setting); JSON lines out."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "faithdiff-dev_amd"))
import torch  # noqa: E402

from fdhip import ops  # noqa: E402
from fdhip import lib as L  # noqa: E402

L.require_device()
bf = torch.bfloat16
SHAPES = [(2048, 1280, 1280), (2048, 1280, 5120), (2048, 1280, 12800), (2048, 3840, 1280), (8192, 640, 640)]
if len(sys.argv) > 1:
    SHAPES = [tuple(int(x) for x in s.split(":")[0].split("x")) + ((s.split(":")[1],) if ":" in s else ())
              for s in sys.argv[1:]]
tag = {k: v for k, v in os.environ.items() if k.startswith("FD_GEMM")}
for shp in SHAPES:
    M, N, K = shp[:3]
    act = shp[3] if len(shp) > 3 else "none"
    a = torch.randn(M, K, device="cuda").to(bf)
    w = (torch.randn(N, K, device="cuda") / K ** 0.5).to(bf)
    out = torch.empty(M, N // 2 if act == "geglu" else N, device="cuda", dtype=bf)
    for _ in range(5):
        ops.gemm(a, w, out=out, act=act)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    it = 30
    e0.record()
    for _ in range(it):
        ops.gemm(a, w, out=out, act=act)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / it * 1e3
    print(json.dumps({**tag, "shape": f"{M}x{N}x{K}:{act}", "us": round(us, 2), "tflops": round(2 * M * N * K / us / 1e6, 1)}))
