#!/usr/bin/env python3
"""Does a copy-engine read of a GEMM's weights (hipMemcpyAsync, hipMemcpyDeviceToDeviceNoCU = SDMA, no compute
units) leave them in the Infinity Cache for the GEMM that follows?  The UNet streams 5 GB of weights per forward, so
every GEMM at the 32^2 level starts on HBM-cold weights (r04f: the 2048x1280x1280 projection 14.1 -> 16.4 us with 120
weight copies).  Per launch (HIP events, median of the launches): warm (the same W every time), cold (a rotating set
of 120 copies, 393 MB > the 256 MB Infinity Cache), cold + an SDMA copy of this launch's W into a scratch buffer first
(waited for), and cold + a blit-kernel copy (torch copy_, for comparison).  One JSON line per shape."""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "faithdiff-dev_amd"))
import torch  # noqa: E402

from fdhip import lib as L  # noqa: E402
from fdhip import ops  # noqa: E402

L.require_device()
hip = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
hip.hipMemcpyAsync.restype = ctypes.c_int
NOCU = 1024  # hipMemcpyDeviceToDeviceNoCU

SHAPES = [(2048, 1280, 1280), (2048, 10240, 1280), (2048, 3840, 1280)]
NCOPY = 120
dev = "cuda"
for M, N, K in SHAPES:
    nc = max(8, min(NCOPY, (400 << 20) // (N * K * 2)))
    A = torch.randn(M, K, device=dev).to(torch.bfloat16)
    Ws = [torch.randn(N, K, device=dev).to(torch.bfloat16) for _ in range(nc)]
    act = "geglu" if N == 10240 else "none"
    scratch = torch.empty(N * K, device=dev, dtype=torch.bfloat16)
    side = torch.cuda.Stream()
    main = torch.cuda.current_stream()

    def run(mode, reps):
        ts = []
        for r in range(reps):
            w = Ws[0] if mode == "warm" else Ws[r % nc]
            if mode == "sdma":
                ev = torch.cuda.Event()
                rc = hip.hipMemcpyAsync(scratch.data_ptr(), w.data_ptr(), N * K * 2, NOCU, side.cuda_stream)
                assert rc == 0, rc
                ev.record(side)
                main.wait_event(ev)
            elif mode == "blit":
                scratch.copy_(w.view(-1))
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            ops.gemm(A, w, act=act)
            e1.record()
            ts.append((e0, e1))
        torch.cuda.synchronize()
        v = sorted(a.elapsed_time(b) * 1e3 for a, b in ts[nc if reps > nc else 0:])  # skip the first pass
        return round(v[len(v) // 2], 2), round(v[0], 2)

    run("warm", 10)
    out = {"shape": f"{M}x{N}x{K}{':geglu' if act == 'geglu' else ''}", "copies": nc}
    for mode in ("warm", "cold", "sdma", "blit", "cold"):
        out[mode] = run(mode, 3 * nc)
    print(json.dumps(out), flush=True)
    del Ws
    torch.cuda.empty_cache()
