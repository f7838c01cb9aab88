"""Probe: does running the two CFG halves of a C2 UNet forward as two B = 1 graphs on two streams beat one B = 2
graph?  (After the FaithDiff extras every row of the UNet is independent; two concurrent launch chains let one
half's kernel prologue / epilogue / launch ramp overlap the other half's main loop.)  Timing only: the extras run
per half here (MHA over one row), so the numbers are not a parity result.  The two concurrent forwards also share
one HipUNet's persistent two-GEMM cross-attention P buffer (ops._pbuf, keyed by (M, KP)) and the GEMM split-K
workspace, so they RACE: the outputs of this probe are meaningless and only its timings stand.  Concurrent forwards
in the product would need a P buffer and workspace per stream; the product has no such mode (the FD_CFG_STREAMS
knob was removed)."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "faithdiff-dev_amd"))
from fdhip import arch, ops  # noqa: E402
from fdhip.unet import HipUNet  # noqa: E402

# per-stream split-K / GroupNorm workspaces (the product keys them by device only)
_ws = {}


def _key(device):
    return (torch.device(device), torch.cuda.current_stream().cuda_stream)


def gemm_ws(nbytes, device):
    k = _key(device)
    ws = _ws.get(("g",) + k)
    if ws is None or ws.numel() < nbytes:
        ws = torch.zeros(max(nbytes, 1 << 24), dtype=torch.uint8, device=device)
        _ws[("g",) + k] = ws
    return ws


def gn_ws(nbytes, device):
    k = _key(device)
    ws = _ws.get(("n",) + k)
    if ws is None or ws.numel() < nbytes:
        ws = torch.empty(max(nbytes, 1 << 24), dtype=torch.uint8, device=device)
        _ws[("n",) + k] = ws
    return ws


def attach_ws(p, device):
    groups = ops._TILE_GROUPS[-1]
    p.m_ref = p.M // groups if groups > 1 and p.M % groups == 0 else p.M
    need = ops.L.load().fd_gemm_ws_bytes(ops.ctypes.byref(p))
    if need <= 0:
        return
    ws = gemm_ws(need, device)
    p.ws, p.ws_bytes = ws.data_ptr(), ws.numel()


ops._attach_ws = attach_ws
ops._gn_ws = gn_ws


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    sd = arch.random_init(arch.unet_param_shapes(), seed=1, device="cuda")
    hip = HipUNet(sd, dev, torch.bfloat16)
    del sd
    h = w = 128
    g = torch.Generator(device="cuda").manual_seed(0)
    ctx = torch.randn(2, 77, 2048, device=dev, generator=g)
    x = torch.randn(2 * h * w, 4, device=dev, generator=g).to(torch.bfloat16)
    cond = torch.randn(2 * h * w, 512, device=dev, generator=g).to(torch.bfloat16)
    tids = torch.tensor([[1024.0, 1024.0, 0, 0, 1024.0, 1024.0]] * 2, device=dev)
    text = torch.randn(2, 1280, device=dev, generator=g)
    t = torch.full((2,), 951.0, device=dev)

    def capture(fn, stream):
        fn()  # eager: sizes workspaces
        torch.cuda.synchronize()
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr, stream=stream):
            fn()
        torch.cuda.synchronize()
        return gr

    s0, s1, s2 = torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.Stream()
    hip.set_context(ctx)
    g2 = capture(lambda: hip.forward(x, t, tids, text, cond, 2, h, w), s0)
    hip1 = hip
    keep = (hip._kv, hip.ctx)  # g2 reads these buffers on replay
    hip1.set_context(ctx[:1])
    half = h * w
    ga = capture(lambda: hip1.forward(x[:half], t[:1], tids[:1], text[:1], cond[:half], 1, h, w), s1)
    gb = capture(lambda: hip1.forward(x[half:], t[1:], tids[1:], text[1:], cond[half:], 1, h, w), s2)

    # one graph with a fork / join inside (does ROCm's graph launch run the two branches concurrently?)
    sf = torch.cuda.Stream()

    def forked():
        main = torch.cuda.current_stream()
        sf.wait_stream(main)
        hip1.forward(x[:half], t[:1], tids[:1], text[:1], cond[:half], 1, h, w)
        with torch.cuda.stream(sf):
            hip1.forward(x[half:], t[1:], tids[1:], text[1:], cond[half:], 1, h, w)
        main.wait_stream(sf)
    forked()  # eager: sizes the side stream's workspaces
    torch.cuda.synchronize()
    gf = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gf, stream=s0):
        forked()
    torch.cuda.synchronize()

    def timeit(fn, n=30):
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / n * 1e3

    cur = torch.cuda.current_stream()

    def both():
        s1.wait_stream(cur)
        s2.wait_stream(cur)
        with torch.cuda.stream(s1):
            ga.replay()
        with torch.cuda.stream(s2):
            gb.replay()
        cur.wait_stream(s1)
        cur.wait_stream(s2)

    def seq():
        with torch.cuda.stream(s1):
            ga.replay()
            gb.replay()

    for rep in range(2):
        print(f"B=2 one graph: {timeit(lambda: g2.replay()):.3f} ms   B=1 x2 sequential: {timeit(seq):.3f} ms   "
              f"B=1 x2 concurrent streams: {timeit(both):.3f} ms   one forked graph: {timeit(lambda: gf.replay()):.3f} ms   "
              f"one B=1: {timeit(lambda: ga.replay()):.3f} ms",
              flush=True)


if __name__ == "__main__":
    main()
