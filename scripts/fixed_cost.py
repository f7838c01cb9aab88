#!/usr/bin/env python3
"""Fixed per-launch cost under graph replay: tiny / short-K GEMMs, LayerNorm, an elementwise copy."""
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
bf = torch.bfloat16
REP = 50


def timeit(fn):
    st = torch.cuda.Stream()
    with torch.cuda.stream(st):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=st):
            for _ in range(REP):
                fn()
        graph.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        best = 1e30
        for _ in range(5):
            e0.record(st)
            graph.replay()
            e1.record(st)
            torch.cuda.synchronize()
            best = min(best, e0.elapsed_time(e1) / REP * 1e3)
    return round(best, 2)


for M, N, K in [(64, 64, 64), (2048, 1280, 64), (2048, 1280, 128), (2048, 1280, 320), (2048, 1280, 640),
                (2048, 1280, 1280), (2048, 1280, 2560)]:
    a = torch.randn(M, K, device="cuda").to(bf)
    w = (torch.randn(N, K, device="cuda") / K ** 0.5).to(bf)
    out = torch.empty(M, N, device="cuda", dtype=bf)
    print(json.dumps({"gemm": f"{M}x{N}x{K}", "env": {k: v for k, v in os.environ.items() if k.startswith("FD_")},
                      "us": timeit(lambda: ops.gemm(a, w, out=out))}), flush=True)
x = torch.randn(2048, 1280, device="cuda").to(bf)
g = torch.ones(1280, device="cuda")
b = torch.zeros(1280, device="cuda")
y = torch.empty_like(x)
print(json.dumps({"layer_norm": "2048x1280", "us": timeit(lambda: ops.layer_norm(x, g, b, out=y))}), flush=True)
x2 = torch.randn(8192, 640, device="cuda").to(bf)
g2 = torch.ones(640, device="cuda")
b2 = torch.zeros(640, device="cuda")
y2 = torch.empty_like(x2)
print(json.dumps({"layer_norm": "8192x640", "us": timeit(lambda: ops.layer_norm(x2, g2, b2, out=y2))}), flush=True)
print(json.dumps({"copy_5MB": timeit(lambda: y.copy_(x))}), flush=True)
z = torch.empty(1, device="cuda")
print(json.dumps({"fill_1elem": timeit(lambda: z.fill_(1.0))}), flush=True)
for (n, hw, c) in [(2, 16384, 320), (2, 4096, 640), (2, 1024, 1280), (2, 1024, 2560)]:
    xg = torch.randn(n * hw, c, device="cuda").to(bf)
    gg = torch.ones(c, device="cuda")
    bg = torch.zeros(c, device="cuda")
    yg = torch.empty_like(xg)
    print(json.dumps({"group_norm": f"{n}x{hw}x{c}",
                      "us": timeit(lambda: ops.group_norm(xg, gg, bg, n, hw, c, 32, 1e-5, True, out=yg))}), flush=True)
