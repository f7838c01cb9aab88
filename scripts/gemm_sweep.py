#!/usr/bin/env python3
"""Time the UNet's dominant GEMM / conv shapes under the FD_GEMM_* env knobs (one process per setting)."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "faithdiff-dev_amd"))
import torch  # noqa: E402

from fdhip import ops  # noqa: E402
from fdhip import lib as L  # noqa: E402
from fdhip import knobs  # noqa: E402

knobs.apply_env()  # measurement script: FD_* knob overrides from the environment

L.require_device()
dev = "cuda"
torch.manual_seed(0)
bf = torch.bfloat16
SHAPES = [("G1 2048x1280x1280", "gemm", 2048, 1280, 1280), ("G2 2048x1280x5120", "gemm", 2048, 1280, 5120),
          ("G3 2048x3840x1280", "gemm", 2048, 3840, 1280), ("G4 geglu 2048x10240x1280", "geglu", 2048, 10240, 1280),
          ("G5 8192x640x640", "gemm", 8192, 640, 640), ("G6 geglu 8192x5120x640", "geglu", 8192, 5120, 640),
          ("C1 conv32 1280", "conv", 2, 32, 1280), ("C2 conv128 320", "conv", 2, 128, 320),
          ("C3 conv64 640", "conv", 2, 64, 640)]


def timeit(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it * 1e3  # us


tag = {k: os.environ.get(k) for k in ("FD_GEMM_CFG", "FD_GEMM_NS", "FD_GEMM_SWZ")}
for name, kind, a, b, c in SHAPES:
    if kind in ("gemm", "geglu"):
        M, N, K = a, b, c
        x = torch.randn(M, K, device=dev).to(bf)
        w = (torch.randn(N, K, device=dev) / K ** 0.5).to(bf)
        bias = torch.zeros(N, device=dev)
        out = torch.empty(M, N // 2 if kind == "geglu" else N, dtype=bf, device=dev)
        us = timeit(lambda: ops.gemm(x, w, out=out, bias=bias, act="geglu" if kind == "geglu" else "none"))
        flops = 2.0 * M * N * K
    else:
        n, H, C = a, b, c
        x = torch.randn(n * H * H, C, device=dev).to(bf)
        w = (torch.randn(C, 9 * C, device=dev) / (9 * C) ** 0.5).to(bf)
        bias = torch.zeros(C, device=dev)
        out = torch.empty(n * H * H, C, dtype=bf, device=dev)
        us = timeit(lambda: ops.conv3x3(x, w, bias, n, H, H, out=out))
        flops = 2.0 * n * H * H * C * 9 * C
    print(json.dumps({**tag, "shape": name, "us": round(us, 1), "tflops": round(flops / us / 1e6, 1)}), flush=True)
