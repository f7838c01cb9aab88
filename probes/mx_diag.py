#!/usr/bin/env python3
"""Diagnostic (not product): which A block scale does fd_gemm_mxe4m3 apply to each (row, K block)?"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "faithdiff-dev_amd"))
import torch  # noqa: E402

from fdhip import lib as L  # noqa: E402
from fdhip import ops  # noqa: E402

L.require_device()
DEV = "cuda"
for tile in ("64160", "256128"):
    os.environ["FD_F8_TILE"] = tile
    for M, K in ((64, 128), (256, 256)):
        N = 160
        a = torch.ones(M, K)
        w = torch.ones(N, K)
        for name, pat in (("block", lambda m, b: 127 + (b % 4)), ("row", lambda m, b: 127 + (m % 4)),
                          ("kstep", lambda m, b: 127 + (b // 4) % 3)):
            mx = ops.MX(M, K, DEV)
            mx.q.copy_(a.to(torch.float8_e4m3fn).view(torch.uint8))
            s = torch.tensor([[pat(m, b) for b in range(K // 32)] for m in range(M)], dtype=torch.uint8)
            mx.s.zero_()
            mx.s[:, :K // 32].copy_(s)
            got = ops.gemm_mx(mx, w.to(torch.float8_e4m3fn).view(torch.uint8).to(DEV), out_dtype=torch.float32).cpu()
            want = (32.0 * torch.exp2(s.double() - 127)).sum(1)
            bad = (got[:, 0].double() != want)
            print(tile, M, K, name, "rows wrong:", int(bad.sum()), "col-uniform:", bool((got == got[:, :1]).all()),
                  "got rows 0..7:", got[:8, 0].tolist(), "want:", want[:8].tolist(), flush=True)

# the exact-integer test's data: where do the results differ?
for tile, (M, N, K) in (("64160", (300, 200, 640)), ("64160", (64, 160, 640)), ("64160", (64, 160, 128)),
                        ("256128", (256, 128, 256))):
    os.environ["FD_F8_TILE"] = tile
    g = torch.Generator().manual_seed(M + N + K)
    a = torch.randint(-6, 7, (M, K), generator=g).float()
    sb = torch.randint(124, 131, (M, K // 32), generator=g).to(torch.uint8)
    w = torch.randint(-4, 5, (N, K), generator=g).float() * 0.5
    for sname, sbb in (("rand", sb), ("unit", torch.full_like(sb, 127))):
        mx = ops.MX(M, K, DEV)
        mx.q.copy_(a.to(torch.float8_e4m3fn).view(torch.uint8).to(DEV))
        mx.s.zero_()
        mx.s[:, :K // 32].copy_(sbb.to(DEV))
        got = ops.gemm_mx(mx, w.to(torch.float8_e4m3fn).view(torch.uint8).to(DEV), out_dtype=torch.float32).cpu()
        want = (a.double() * torch.exp2(sbb.double() - 127).repeat_interleave(32, 1)) @ w.double().T
        bad = got.double() != want
        idx = bad.nonzero()[:4].tolist()
        print(tile, M, N, K, sname, "wrong:", int(bad.sum()), "of", bad.numel(),
              [(m, n, float(got[m, n]), float(want[m, n])) for m, n in idx], flush=True)
