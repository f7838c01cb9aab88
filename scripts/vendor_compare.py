#!/usr/bin/env python3
"""Calibration only (not a product path): time torch.matmul (hipBLASLt) and torch SDPA on the UNet's
dominant shapes next to this repo's kernels, back-to-back launches, HIP events."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "faithdiff-dev_amd"))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from fdhip import ops  # noqa: E402
from fdhip import lib as L  # noqa: E402

L.require_device()
dev, bf = "cuda", torch.bfloat16


def timeit(fn, it=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it * 1e3


for M, N, K in [(2048, 1280, 1280), (2048, 1280, 5120), (2048, 3840, 1280), (2048, 10240, 1280), (8192, 640, 640),
                (8192, 5120, 640), (8192, 640, 2560), (2048, 1280, 11520), (32768, 320, 2880), (8192, 1920, 640)]:
    a = torch.randn(M, K, device=dev).to(bf)
    w = torch.randn(N, K, device=dev).to(bf) / K ** 0.5
    out = torch.empty(M, N, device=dev, dtype=bf)
    t_ours = timeit(lambda: ops.gemm(a, w, out=out))
    wt = w.t()
    t_blas = timeit(lambda: torch.matmul(a, wt, out=out))
    fl = 2.0 * M * N * K
    print(f"gemm {M}x{N}x{K}: ours {t_ours:7.1f} us ({fl / t_ours / 1e6:6.1f} TF/s)  hipBLASLt {t_blas:7.1f} us "
          f"({fl / t_blas / 1e6:6.1f} TF/s)")

# fp8: this repo's e4m3 kernel (per-row activation scale) vs hipBLASLt's e4m3 x e4m3 (torch._scaled_mm, tensor
# scales) on the transformer Linear shapes of the fp8 leg
for M, N, K in [(2048, 1280, 1280), (2048, 1280, 5120), (2048, 3840, 1280), (2048, 10240, 1280), (8192, 640, 640),
                (8192, 5120, 640), (8192, 640, 2560)]:
    a = torch.randn(M, K, device=dev).to(bf)
    w = torch.randn(N, K, device=dev).to(bf) / K ** 0.5
    a8, sa = ops.quant_rows_e4m3(a)
    w8 = w.to(torch.float8_e4m3fn).view(torch.uint8)
    out = torch.empty(M, N, device=dev, dtype=bf)
    t_ours = timeit(lambda: ops.gemm_e4m3(a8, sa, w8, out=out))
    fl = 2.0 * M * N * K
    try:
        af, wf = a8.view(torch.float8_e4m3fn), w8.view(torch.float8_e4m3fn)
        one = torch.ones((), device=dev)
        t_blas = timeit(lambda: torch._scaled_mm(af, wf.t(), scale_a=one, scale_b=one, out_dtype=bf))
        vend = f"hipBLASLt {t_blas:7.1f} us ({fl / t_blas / 1e6:6.1f} TF/s)"
    except Exception as e:  # noqa: BLE001
        vend = f"hipBLASLt fp8 unavailable: {type(e).__name__}: {str(e)[:80]}"
    print(f"fp8 {M}x{N}x{K}: ours {t_ours:7.1f} us ({fl / t_ours / 1e6:6.1f} TF/s)  {vend}")

for b, h, Lq in [(2, 20, 1024), (2, 10, 4096)]:
    q = torch.randn(b, Lq, h * 64, device=dev).to(bf)
    k = torch.randn(b, Lq, h * 64, device=dev).to(bf)
    v = torch.randn(b, Lq, h * 64, device=dev).to(bf)
    o = torch.empty_like(q)
    E = h * 64
    t_ours = timeit(lambda: ops.flash_attn(q, k, v, o, b, h, Lq, Lq, E, E, E, E, Lq * E, Lq * E, Lq * E, Lq * E))
    qh, kh, vh = (x.view(b, Lq, h, 64).transpose(1, 2) for x in (q, k, v))
    t_sdpa = timeit(lambda: F.scaled_dot_product_attention(qh, kh, vh))
    fl = 4.0 * b * h * Lq * Lq * 64
    print(f"attn b{b} h{h} L{Lq}: ours {t_ours:7.1f} us ({fl / t_ours / 1e6:6.1f} TF/s)  torch sdpa {t_sdpa:7.1f} us "
          f"({fl / t_sdpa / 1e6:6.1f} TF/s)")
