#!/usr/bin/env python3
"""e4m3 GEMM kernel A/B on the use_fp8 UNet's Linear shapes: the eight-wave
family with its own tile choice, each forced tile shape (FD_F8_TILE), the bf16 fd_gemm of the same shape, and the MX
(block-scaled A) form, GEGLU also with the MX output (PROBE_MX_TILES=1: every MX tile shape).
REP launches per variant are captured into one hipGraph and replayed between HIP events (no Python enqueue in
the per-launch time).  One JSON line per shape.  Usage: f8_tiles.py [MxNxK[:geglu] ...]"""
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
SHAPES = sys.argv[1:] or ["2048x1280x1280", "2048x1280x5120", "2048x3840x1280", "2048x10240x1280:geglu",
                          "8192x640x640", "8192x1920x640", "8192x640x2560", "8192x5120x640:geglu",
                          "26624x1280x1280", "26624x10240x1280:geglu"]
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
        s.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        best = 1e30
        for _ in range(5):
            e0.record(s)
            gr.replay()
            e1.record(s)
            s.synchronize()
            best = min(best, e0.elapsed_time(e1) * 1e3 / REP)
    return best


def with_env(env, fn):
    """Graph-time fn with the given planner knobs (None = default)."""
    kw = {k: knobs.default(k) if v is None else v for k, v in env.items()}
    with knobs.override(**kw):
        return graph_us(fn)


dev = "cuda"
for arg in SHAPES:
    shape, _, act = arg.partition(":")
    M, N, K = map(int, shape.split("x"))
    act = act or "none"
    a = torch.randn(M, K, device=dev).to(torch.bfloat16)
    w = torch.randn(N, K, device=dev) * K ** -0.5
    w8 = ops.pack_e4m3(w)
    wb = w.to(torch.bfloat16)
    q, sc = ops.quant_rows_e4m3(a)
    out = torch.empty(M, N // 2 if act == "geglu" else N, device=dev, dtype=torch.bfloat16)
    f8 = lambda: ops.gemm_e4m3(q, sc, w8, out=out, act=act)  # noqa: E731
    bf = lambda: ops.gemm(a, wb, out=out, act=act)  # noqa: E731
    flop = 2.0 * M * N * K
    rec = {"shape": arg}
    rec["f8_8wave_us"] = with_env({"FD_F8_TILE": None}, f8)
    for t in ("256160", "256128", "128160", "64160"):
        if act == "geglu" and t in ("128160", "64160"):
            continue
        rec[f"f8_tile{t}_us"] = with_env({"FD_F8_TILE": t}, f8)
    rec["bf16_us"] = graph_us(bf)
    amx = ops.quant_rows_mx(a)
    rec["mx_us"] = with_env({"FD_F8_TILE": None},
                            lambda: ops.gemm_mx(amx, w8, out=out, act=act))
    if act == "geglu":
        omx = ops.MX(M, N // 2, dev)
        rec["mx_out_us"] = with_env({"FD_F8_TILE": None},
                                    lambda: ops.gemm_mx(amx, w8, out=omx, act=act))
    if os.environ.get("PROBE_MX_TILES"):
        for t in ("256160", "256128", "128160", "64160"):
            if act == "geglu" and t in ("128160", "64160"):
                continue
            rec[f"mx_tile{t}_us"] = with_env({"FD_F8_TILE": t},
                                             lambda: ops.gemm_mx(amx, w8, out=out, act=act))
    rec = {k: (round(v, 2) if isinstance(v, float) else v) for k, v in rec.items()}
    rec["f8_8wave_tflops"] = round(flop / rec["f8_8wave_us"] / 1e6, 1)
    rec["f8_4wave_tflops"] = round(flop / rec["f8_4wave_us"] / 1e6, 1)
    print(json.dumps(rec), flush=True)
