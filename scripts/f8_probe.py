#!/usr/bin/env python3
"""Calibration only: time ops.gemm_e4m3 (fp8 leg) on the UNet's fp8 Linear shapes, back-to-back launches, HIP
events.  Args: MxNxK[:geglu] ...  Env: FD_LIB_PATH (diagnostic builds), PROBE_TAG."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "faithdiff-dev_amd"))
import torch  # noqa: E402

from fdhip import lib as L  # noqa: E402
from fdhip import ops  # noqa: E402
from fdhip import knobs  # noqa: E402

knobs.apply_env()  # measurement script: FD_* knob overrides from the environment

L.require_device()
dev = "cuda"
for arg in sys.argv[1:]:
    shape, _, act = arg.partition(":")
    M, N, K = map(int, shape.split("x"))
    act = act or "none"
    a = torch.randn(M, K, device=dev).to(torch.bfloat16)
    w8 = ops.pack_e4m3(torch.randn(N, K, device=dev) * K ** -0.5)
    q, sc = ops.quant_rows_e4m3(a)
    out = torch.empty(M, N // 2 if act == "geglu" else N, device=dev, dtype=torch.bfloat16)
    fn = lambda: ops.gemm_e4m3(q, sc, w8, out=out, act=act)  # noqa: E731
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    it = 50
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / it * 1e3
    print(json.dumps({"tag": os.environ.get("PROBE_TAG", ""), 
                      "shape": arg, "us": round(us, 2), "tflops": round(2.0 * M * N * K / us / 1e6, 1)}), flush=True)
