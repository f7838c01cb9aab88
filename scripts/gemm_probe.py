#!/usr/bin/env python3
"""Time GEMM shapes under the current FD_GEMM_* env; JSON lines out.

Each shape's launches are captured in one hipGraph (REP back-to-back launches) and the graph replayed, so the
per-launch time excludes the ~10 us ctypes/Python enqueue cost that dominates small shapes when launched eagerly.
Usage: gemm_probe.py [MxNxK[:act] ...]; conv shapes as convHxWxCinxCout (nimg 2)."""
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
bf = torch.bfloat16
SHAPES = ["2048x1280x1280", "2048x1280x5120", "2048x3840x1280", "2048x10240x1280:geglu", "8192x640x640"]
if len(sys.argv) > 1:
    SHAPES = sys.argv[1:]
tag = {k: v for k, v in os.environ.items() if k.startswith(("FD_GEMM", "PROBE_"))}
REP = int(os.environ.get("PROBE_REP", "20"))
# PROBE_COPIES=n: n distinct weight copies cycled through the graph (n x |W| past the 256 MB Infinity Cache
# gives cold weights, as inside a UNet forward where every weight is read once)
COPIES = int(os.environ.get("PROBE_COPIES", "1"))
if COPIES > 1:
    REP = max(REP, COPIES)
g = torch.Generator(device="cuda").manual_seed(0)
for s in SHAPES:
    if s.startswith("conv"):
        H, W, Cin, Cout = (int(x) for x in s[4:].split("x"))
        NI = int(os.environ.get("PROBE_NIMG", "2"))  # images in the launch (C3 batches 13 tiles x 2 CFG rows)
        x = torch.rand(NI * H * W, Cin, device="cuda", generator=g).to(bf) * 2 - 1
        wp = ((torch.rand(Cout, 9 * Cin, device="cuda", generator=g) * 2 - 1) / (9 * Cin) ** 0.5).to(bf)
        b = torch.zeros(Cout, device="cuda")
        out = torch.empty(NI * H * W, Cout, device="cuda", dtype=bf)
        fn = lambda: ops.conv3x3(x, wp, b, NI, H, W, out=out)  # noqa: E731
        flops = 2 * NI * H * W * Cout * 9 * Cin
    else:
        dims, act = (s.split(":") + ["none"])[:2]
        M, N, K = (int(v) for v in dims.split("x"))
        a = (torch.rand(M, K, device="cuda", generator=g) * 2 - 1).to(bf)
        w = ((torch.rand(N, K, device="cuda", generator=g) * 2 - 1) / K ** 0.5).to(bf)
        ws_ = [w] + [w.clone() for _ in range(COPIES - 1)]
        out = torch.empty(M, N // 2 if act == "geglu" else N, device="cuda", dtype=bf)
        ctr = [0]

        # PROBE_RES=1: residual add (in place, as the UNet's residual-stream GEMMs); PROBE_LNO=1: also write the
        # LayerNorm-fold partials (ln_out)
        res = out if os.environ.get("PROBE_RES") == "1" else None
        lno = (torch.empty((M, N // 160, 2), device="cuda") if os.environ.get("PROBE_LNO") == "1" and N % 160 == 0
               else None)

        def fn(a=a, ws_=ws_, out=out, act=act, res=res, lno=lno):
            ctr[0] += 1
            return ops.gemm(a, ws_[ctr[0] % len(ws_)], out=out, act=act, residual=res, ln_out=lno)
        flops = 2 * M * N * K
    st = torch.cuda.Stream()
    # PROBE_GROUPS=n: the launch batches n TLC tiles (ops.tile_groups), so the planner sees m_ref = M / n as in
    # a batched UNet forward
    with torch.cuda.stream(st), ops.tile_groups(int(os.environ.get("PROBE_GROUPS", "1"))):
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
    print(json.dumps({**tag, "shape": s, "us": round(best, 2), "tflops": round(flops / best / 1e6, 1)}), flush=True)
