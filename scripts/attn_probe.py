#!/usr/bin/env python3
"""Graph-timed flash attention (d = 64) at the UNet's shapes; JSON lines (env FD_FLASH_* tag the run)."""
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
SHAPES = [(2, 20, 1024, 1024), (2, 10, 4096, 4096), (2, 20, 1024, 77), (2, 10, 4096, 77)]
if len(sys.argv) > 1:  # extra shapes as BxHxLqxLk
    SHAPES = [tuple(int(v) for v in a.split("x")) for a in sys.argv[1:]]
tag = {k: v for k, v in os.environ.items() if k.startswith("FD_FLASH")}
REP = 20
for B, H, Lq, Lk in SHAPES:
    C = H * 64
    g = torch.Generator(device="cuda").manual_seed(0)
    qkv = torch.randn(B * Lq, 3 * C, device="cuda", generator=g).to(torch.bfloat16)
    kv = torch.randn(B * Lk, 2 * C, device="cuda", generator=g).to(torch.bfloat16)
    o = torch.empty(B * Lq, C, device="cuda", dtype=torch.bfloat16)
    if Lq == Lk:
        fn = lambda: ops.flash_attn(qkv, qkv[:, C:], qkv[:, 2 * C:], o, B, H, Lq, Lk, 3 * C, 3 * C, 3 * C, C,  # noqa
                                    Lq * 3 * C, Lq * 3 * C, Lq * 3 * C, Lq * C, kv_mod=0, scale=0.125)
    else:
        fn = lambda: ops.flash_attn(qkv, kv, kv[:, C:], o, B, H, Lq, Lk, 3 * C, 2 * C, 2 * C, C,  # noqa
                                    Lq * 3 * C, Lk * 2 * C, Lk * 2 * C, Lq * C, kv_mod=0, scale=0.125)
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
    fl = 4.0 * B * H * Lq * Lk * 64
    print(json.dumps({**tag, "shape": f"b{B}h{H}q{Lq}k{Lk}", "us": round(best, 2), "tflops": round(fl / best / 1e6, 1)}),
          flush=True)
