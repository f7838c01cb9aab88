#!/usr/bin/env python3
"""Eager flash-attention launches at the UNet's self-attention shapes (for rocprofv3 --pmc passes)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "faithdiff-dev_amd"))
import torch  # noqa: E402

from fdhip import ops  # noqa: E402
from fdhip import lib as L  # noqa: E402

L.require_device()
for B, H, Lq in [(2, 20, 1024), (2, 10, 4096)]:
    C = H * 64
    qkv = torch.randn(B * Lq, 3 * C, device="cuda").to(torch.bfloat16)
    o = torch.empty(B * Lq, C, device="cuda", dtype=torch.bfloat16)
    for _ in range(3):
        ops.flash_attn(qkv, qkv[:, C:], qkv[:, 2 * C:], o, B, H, Lq, Lq, 3 * C, 3 * C, 3 * C, C,
                       Lq * 3 * C, Lq * 3 * C, Lq * 3 * C, Lq * C, kv_mod=0, scale=0.125)
    torch.cuda.synchronize()
print("done")
