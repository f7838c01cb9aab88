#!/usr/bin/env python3
"""Diagnostic (not product): where does fd_layer_norm_mx differ from fd_layer_norm + fd_quant_rows_mx (f16)?"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "faithdiff-dev_amd"))
import torch  # noqa: E402

from fdhip import lib as L  # noqa: E402
from fdhip import ops  # noqa: E402

L.require_device()
DEV = "cuda"
torch.manual_seed(0)
for dtype in (torch.float16, torch.bfloat16):
    M, C = 4096, 640
    x = (torch.randn(M, C, device=DEV) * 3 + 1).to(dtype)
    g = torch.randn(C, device=DEV)
    b = torch.randn(C, device=DEV)
    got = ops.layer_norm_mx(x, g, b, 1e-5)
    y = ops.layer_norm(x, g, b, 1e-5)
    ref = ops.quant_rows_mx(y)
    bad = (got.q != ref.q).nonzero()
    print(dtype, "mismatches:", bad.shape[0], flush=True)
    for m, k in bad[:6].tolist():
        E = int(ref.s[m, k // 32]) - 127
        v = float(y[m, k])
        print(f"  ({m},{k}) y={v!r} y*2^-E={v * 2.0 ** -E!r} got={int(got.q[m, k])} ref={int(ref.q[m, k])} "
              f"got_val={float(got.q[m, k:k + 1].view(torch.float8_e4m3fn).float())} "
              f"ref_val={float(ref.q[m, k:k + 1].view(torch.float8_e4m3fn).float())}", flush=True)
