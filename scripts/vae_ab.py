#!/usr/bin/env python3
"""VAE decode at 1024^2 (128^2 latent), graph-timed, plus a per-launch breakdown by kind / label (eager, HIP events
around every launch).  One JSON line; FD_LIB_PATH / FD_GN_* / FD_GEMM* env vars tag the run (A/B of library
builds on one box)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "faithdiff-dev_amd"))
import torch  # noqa: E402

import bench  # noqa: E402
from fdhip import ops  # noqa: E402
from fdhip import knobs  # noqa: E402

knobs.apply_env()  # measurement script: FD_* knob overrides from the environment


def main():
    dev = torch.device("cuda:0")
    pipe = bench.build_pipe(dev, False)
    dec = pipe.vae.decoder_hip()
    h = w = 128
    g = torch.Generator(device="cuda").manual_seed(0)
    z = torch.randn((h * w, 4), generator=g, device=dev).to(torch.float16)
    for _ in range(3):
        dec.decode_graphed(z, 1, h, w)
    torch.cuda.synchronize()
    times = []
    for _ in range(9):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        dec.decode_graphed(z, 1, h, w)
        e1.record()
        torch.cuda.synchronize()
        times.append(e0.elapsed_time(e1))
    rec = []
    for it in range(2):
        rec.clear()
        ops.set_probe(rec)
        try:
            dec.decode(z, 1, h, w)
        finally:
            ops.set_probe(None)
        torch.cuda.synchronize()
    by = {}
    for r in rec:
        key = r[0] + (" " + r[5] if len(r) > 5 else "")
        ms = r[3].elapsed_time(r[4])
        n, t = by.get(key, (0, 0.0))
        by[key] = (n + 1, t + ms)
    kinds = {}
    for k, (n, t) in by.items():
        kk = k.split()[0]
        kinds[kk] = round(kinds.get(kk, 0.0) + t, 3)
    tag = {k: v for k, v in os.environ.items() if k.startswith(("FD_LIB", "FD_GN", "FD_GEMM", "FD_D512", "AB_TAG"))}
    top = sorted(by.items(), key=lambda kv: -kv[1][1])[:12]
    print(json.dumps({**tag, "decode_ms_median": round(sorted(times)[4], 3), "decode_ms_min": round(min(times), 3),
                      "eager_kind_ms": kinds,
                      "top": [[k, n, round(t, 3)] for k, (n, t) in top]}), flush=True)


if __name__ == "__main__":
    main()
