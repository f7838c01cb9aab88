#!/usr/bin/env python3
"""Graph-timed cost of the LayerNorm fold on its GEMMs: producer with / without ln_out, consumer with / without
ln_in, at the UNet's 32^2-level shapes (M = 2048, C = 1280)."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "faithdiff-dev_amd"))
import torch  # noqa: E402

from fdhip import ops  # noqa: E402
from fdhip import lib as L  # noqa: E402

L.require_device()
bf = torch.bfloat16
REP = 20


def timeit(fn):
    st = torch.cuda.Stream()
    with torch.cuda.stream(st):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=st):
            for _ in range(REP):
                fn()
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        best = 1e30
        for _ in range(5):
            e0.record(st)
            g.replay()
            e1.record(st)
            torch.cuda.synchronize()
            best = min(best, e0.elapsed_time(e1) / REP * 1e3)
    return round(best, 2)


M, C = int(os.environ.get("M", 2048)), int(os.environ.get("C", 1280))
att = torch.randn(M, C, device="cuda").to(bf)
wo = (torch.randn(C, C, device="cuda") / C ** 0.5).to(bf)
bo = torch.zeros(C, device="cuda")
h = torch.randn(M, C, device="cuda").to(bf)
st = torch.zeros(M, C // 160, 2, device="cuda")
ops.gemm(att, wo, bias=bo, residual=h, out=h, ln_out=st)
res = {}
res["producer"] = timeit(lambda: ops.gemm(att, wo, bias=bo, residual=h, out=h))
res["producer+ln_out"] = timeit(lambda: ops.gemm(att, wo, bias=bo, residual=h, out=h, ln_out=st))
gamma, beta = torch.ones(C, device="cuda"), torch.zeros(C, device="cuda")
for kind, n in (("q", C), ("qkv", 3 * C), ("geglu", 8 * C)):
    w = (torch.randn(n, C, device="cuda") / C ** 0.5).to(bf)
    b = torch.zeros(n, device="cuda")
    wp, c, d = ops.fold_layer_norm(w, gamma, beta, b)
    act = "geglu" if kind == "geglu" else "none"
    out = torch.empty(M, n // 2 if act == "geglu" else n, device="cuda", dtype=bf)
    res[kind] = timeit(lambda: ops.gemm(h, w, bias=b, act=act, out=out))
    res[kind + "+ln_in"] = timeit(lambda: ops.gemm(h, wp, bias=d, act=act, out=out, ln_in=st, ln_c=c))
nrm = torch.empty_like(h)
res["layer_norm"] = timeit(lambda: ops.layer_norm(h, gamma, beta, 1e-5, out=nrm))
print(json.dumps({"M": M, "C": C, **res}), flush=True)
