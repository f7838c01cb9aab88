#!/usr/bin/env python3
"""Diagnostic (not product): for A nonzero in one 32-element block only, which scale byte got applied?"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "faithdiff-dev_amd"))
import torch  # noqa: E402

from fdhip import lib as L  # noqa: E402
from fdhip import ops  # noqa: E402

L.require_device()
DEV = "cuda"
os.environ["FD_F8_TILE"] = "64160"
M, N, K = 64, 160, 128
# distinct scale per (row, block): s = 100 + 4 * (m % 16) + b  (blocks 0..3), so the applied one identifies both
s = torch.tensor([[100 + 4 * (m % 16) + b for b in range(4)] for m in range(M)], dtype=torch.uint8)
w = torch.ones(N, K)
for b0 in range(4):
    a = torch.zeros(M, K)
    a[:, 32 * b0:32 * b0 + 32] = 1.0
    mx = ops.MX(M, K, DEV)
    mx.q.copy_(a.to(torch.float8_e4m3fn).view(torch.uint8).to(DEV))
    mx.s.zero_()
    mx.s[:, :4].copy_(s.to(DEV))
    got = ops.gemm_mx(mx, w.to(torch.float8_e4m3fn).view(torch.uint8).to(DEV), out_dtype=torch.float32).cpu()
    applied = torch.log2(got[:, 0] / 32.0) + 127
    rows = []
    for m in range(16):
        v = int(round(float(applied[m])))
        k = v - 100
        rows.append(f"r{m}:({k // 4},{k % 4})")
    print("A block", b0, "applied scale (row%16, block):", " ".join(rows), flush=True)
