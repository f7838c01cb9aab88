#!/usr/bin/env python3
"""Why are kernels slower inside the C2 UNet forward than replayed as their own family?

Phases, each a run of hipGraph replays on the capture stream, separated by marker launches (fd_postprocess_u8, never
part of the forward) so a rocprofv3 kernel trace of this script splits into them (scripts/incontext_report.py):

  idle     -- nothing but the clock sampler (the idle / boost clock)
  forward  -- the whole C2 UNet forward graph (bench.py's step, cond_embedded), in context
  proj     -- only the forward's M = 2048, N = 1280, K = 1280 projections (the 4-wave 64 x 160 tiles), one graph
  flash    -- only its flash-attention launches, one graph
  gemm     -- only its GEMM-family launches, one graph (bench.py's roofline graph)

During every phase a one-wave sampler on a side stream (probes/clk_probe.so) records (s_memrealtime, s_memtime) every
20 us: the shader clock = d(cycles) / d(100 MHz ticks).  Prints per phase the replay time (HIP events) and the clock's
median / p10 / p90, and writes gpurun_out/<tag>_clock.json with the samples' clock series per phase.

    python scripts/incontext_probe.py [--tag r06d] [--no-clock]
"""
import argparse
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "faithdiff-dev_amd"))
import torch  # noqa: E402

import bench  # noqa: E402

INTERVAL = 2000  # 100 MHz ticks per sample: 20 us


class Clock:
    def __init__(self, dev, nmax=60000):
        self.lib = ctypes.CDLL(os.path.join(ROOT, "probes", "clk_probe.so"))
        self.lib.clk_launch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_ulonglong,
                                        ctypes.c_void_p, ctypes.c_void_p]
        self.buf = torch.zeros((nmax, 2), dtype=torch.int64, device=dev)
        self.cnt = torch.zeros(1, dtype=torch.int32, device=dev)
        self.stop = torch.zeros(1, dtype=torch.int32, device=dev)
        self.side = torch.cuda.Stream(dev)
        self.nmax = nmax

    def start(self):
        self.stop.zero_()
        self.cnt.zero_()
        torch.cuda.synchronize()
        rc = self.lib.clk_launch(self.buf.data_ptr(), self.cnt.data_ptr(), self.nmax, INTERVAL, self.stop.data_ptr(),
                                 ctypes.c_void_p(self.side.cuda_stream))
        if rc != 0:
            raise RuntimeError(f"clk_launch rc={rc}")

    def finish(self):
        self.stop.fill_(1)  # on the capture stream, behind the phase's replays
        torch.cuda.synchronize()
        n = int(self.cnt.item())
        s = self.buf[:n].cpu().tolist()
        self.raw = s
        mhz = [(c1 - c0) / (r1 - r0) * 100.0 for (r0, c0), (r1, c1) in zip(s[:-1], s[1:]) if r1 > r0]
        k = len(mhz) // 20  # drop the ramp-in / ramp-out edges
        return mhz[k:len(mhz) - k] if len(mhz) > 40 else mhz


def stats(v):
    if not v:
        return None
    q = sorted(v)
    return {"median": round(statistics.median(q), 1), "p10": round(q[len(q) // 10], 1),
            "p90": round(q[(9 * len(q)) // 10], 1), "n": len(q)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", default="incontext")
    ap.add_argument("--no-clock", action="store_true")
    ap.add_argument("--reps", type=int, default=40)
    a = ap.parse_args()
    from fdhip import knobs, ops
    from fdhip import lib as L
    knobs.apply_env()
    L.require_device()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    pipe = bench.build_pipe(dev, fp8=False)
    loop = bench.C2Loop(pipe, 1024, 0)
    for i in range(3):  # eager, capture, replay (graph_inputs after the capture)
        loop.step(i)
    torch.cuda.synchronize()
    unet = loop.unet
    rec = []
    g_all = torch.cuda.CUDAGraph()
    ops.set_recorder(rec)
    try:
        with torch.cuda.graph(g_all):
            unet.forward(*loop.args(), cond_embedded=True)
    finally:
        ops.set_recorder(None)

    def graph_of(sel):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for r in sel:
                r[3]()
        return g
    proj = [r for r in rec if r[0] == "gemm" and (r[4] or "").startswith("gemm M=2048 N=1280 K=1280 ")]
    phases = {"forward": (g_all, len(rec)),
              "proj": (graph_of(proj), len(proj)),
              "flash": (graph_of([r for r in rec if r[0] == "flash_attn"]), None),
              "gemm": (graph_of([r for r in rec if r[0] == "gemm"]), None)}
    clk = None if a.no_clock else Clock(dev)
    mk_in = torch.zeros(64, dtype=torch.float32, device=dev)
    mk_out = torch.empty(64, dtype=torch.uint8, device=dev)
    raw = {}
    res = {"what": "C2 UNet forward in context vs kernel-family graphs: replay ms and the shader clock (MHz) sampled "
                   "every 20 us by a one-wave side-stream sampler (s_memtime / s_memrealtime)",
           "proj_launches_per_forward": len(proj), "phases": {}}
    if clk is not None:  # idle clock: the sampler alone for ~20 ms
        clk.start()
        torch.cuda._sleep(int(2e7))
        res["phases"]["idle"] = {"clock_mhz": stats(clk.finish())}
        raw["idle"] = clk.raw
        print("idle", res["phases"]["idle"], flush=True)
    for name, (g, n) in phases.items():
        g.replay()
        torch.cuda.synchronize()
        reps = a.reps * (4 if name in ("proj", "flash") else 1)
        ops.postprocess_u8(mk_in, mk_out)  # phase marker (kernel trace)
        if clk is not None:
            clk.start()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            g.replay()
        e1.record()
        mhz = clk.finish() if clk is not None else []
        if clk is not None:
            raw[name] = clk.raw
        torch.cuda.synchronize()
        ops.postprocess_u8(mk_in, mk_out)
        res["phases"][name] = {"replays": reps, "ms_per_replay": round(e0.elapsed_time(e1) / reps, 4),
                               "clock_mhz": stats(mhz)}
        if n:
            res["phases"][name]["launches"] = n
        print(name, res["phases"][name], flush=True)
    torch.cuda.synchronize()
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", f"{a.tag}_clock.json"), "w") as f:
        json.dump(res, f, indent=1)
    if raw:  # (s_memrealtime, s_memtime) samples per phase, for aligning with a kernel trace (incontext_report.py)
        import numpy as np
        np.savez_compressed(os.path.join(ROOT, "gpurun_out", f"{a.tag}_samples.npz"),
                            **{k: np.asarray(v, dtype=np.int64) for k, v in raw.items()})
    print(json.dumps(res))


if __name__ == "__main__":
    main()
