#!/usr/bin/env python3
"""fp8 (e4m3) GEMM vs the bf16 GEMM on the UNet's plain-linear shapes; one JSON line per shape.

Each variant's REP back-to-back launches are captured in one hipGraph and replayed (no Python enqueue cost in
the per-launch time).  Variants: bf16 fd_gemm; fd_gemm_e4m3 alone (operands already e4m3); quant + gemm_e4m3
(activations quantized per row each time, as a UNet layer would).  Usage: fp8_probe.py [MxNxK ...]"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "faithdiff-dev_amd"))
import torch  # noqa: E402

from fdhip import lib as L  # noqa: E402
from fdhip import ops  # noqa: E402

L.require_device()
SHAPES = sys.argv[1:] or ["2048x1280x1280", "2048x1280x5120", "2048x3840x1280", "8192x640x640", "8192x1920x640",
                          "8192x640x2560", "4096x4096x4096", "8192x8192x8192"]
REP = int(os.environ.get("PROBE_REP", "20"))


def graph_us(fn):
    fn()
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr, stream=s):
            for _ in range(REP):
                fn()
    gr.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e30
    for _ in range(5):
        e0.record()
        gr.replay()
        e1.record()
        e1.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1e3 / REP)
    return best


for s in SHAPES:
    M, N, K = (int(v) for v in s.split("x"))
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    w = torch.randn(N, K, device="cuda") * K ** -0.5
    wb, w8 = w.to(torch.bfloat16), ops.pack_e4m3(w)
    b = torch.zeros(N, device="cuda")
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    q, sc = ops.quant_rows_e4m3(x)
    t_bf16 = graph_us(lambda: ops.gemm(x, wb, out=out, bias=b))
    t_f8 = graph_us(lambda: ops.gemm_e4m3(q, sc, w8, out=out, bias=b))
    t_q = graph_us(lambda: ops.quant_rows_e4m3(x, q=q, scale=sc))
    fl = 2.0 * M * N * K
    print(json.dumps({"shape": s, "bf16_us": round(t_bf16, 2), "e4m3_us": round(t_f8, 2), "quant_us": round(t_q, 2),
                      "bf16_tflops": round(fl / t_bf16 / 1e6, 1), "e4m3_tflops": round(fl / t_f8 / 1e6, 1),
                      "e4m3_plus_quant_tflops": round(fl / (t_f8 + t_q) / 1e6, 1)}), flush=True)
