#!/usr/bin/env python3
"""Workload for the rocprofv3 PMC passes (scripts/pmc.sh): one C2 UNet forward (B=2, 128x128 latent, bf16)
preceded by a calibration copy of known size.  Writes gpurun_out/pmc/meta.json with the number of GEMM /
flash launches per forward so the parser (scripts/pmc_parse.py) can pick the last forward's dispatches.
Run only under rocprofv3 --pmc <counter> (one counter group per pass, no trace domains)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "faithdiff-dev_amd"))
import torch  # noqa: E402


def main():
    from fdhip import arch, ops
    from fdhip import lib as L
    from fdhip.unet import HipUNet
    L.require_device()
    dev = torch.device("cuda", 0)
    k, B = 128, 2
    sd = arch.random_init(arch.unet_param_shapes(True), seed=0, device=dev)
    unet = HipUNet(sd, dev, torch.bfloat16)
    del sd
    g = torch.Generator(device=dev).manual_seed(0)
    unet.set_context(torch.randn((2, 77, 2048), generator=g, device=dev))
    x = torch.randn((B * k * k, 4), generator=g, device=dev).to(torch.bfloat16)
    cond = torch.randn((B * k * k, 512), generator=g, device=dev).to(torch.bfloat16)
    t = torch.full((B,), 951.0, device=dev)
    tids = torch.tensor([[1024.0, 1024.0, 0, 0, 1024.0, 1024.0]] * B, device=dev)
    text = torch.randn((B, 1280), generator=g, device=dev)
    ops.reserve_gn_workspace(1 << 24, dev)
    rec = []
    ops.set_probe(rec)
    unet.forward(x, t, tids, text, cond, B, k, k)
    ops.set_probe(None)
    torch.cuda.synchronize()
    counts = {}
    for kind, fl, nb, _, _, *_ in rec:
        c = counts.setdefault(kind, [0, 0.0])
        c[0] += 1
        c[1] += fl
    # calibration: a 1 GiB -> 1 GiB copy (torch's vectorized copy, 16-B lanes), larger than the 256 MiB
    # Infinity Cache.  fd_postprocess_u8 (never launched by the UNet) brackets the windows as a marker.
    rows, cols = 16384, 32768
    src = torch.empty((rows, cols), dtype=torch.bfloat16, device=dev).normal_()
    dst = torch.empty_like(src)
    mk_in = torch.zeros(64, dtype=torch.float32, device=dev)
    mk_out = torch.empty(64, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    ops.postprocess_u8(mk_in, mk_out)
    dst.copy_(src)
    ops.postprocess_u8(mk_in, mk_out)
    unet.forward(x, t, tids, text, cond, B, k, k)  # the measured forward
    ops.postprocess_u8(mk_in, mk_out)
    torch.cuda.synchronize()
    out = os.path.join(ROOT, "gpurun_out", "pmc")
    os.makedirs(out, exist_ok=True)
    with open(os.path.join(out, "meta.json"), "w") as f:
        json.dump({"workload": "C2 1024", "launches_per_forward": {k: v[0] for k, v in counts.items()},
                   "flops_per_forward": {k: v[1] for k, v in counts.items()},
                   "calib_bytes_read": rows * cols * 2, "calib_bytes_written": rows * cols * 2}, f)
    print("ok", counts)


if __name__ == "__main__":
    main()
