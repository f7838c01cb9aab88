#!/usr/bin/env python3
"""Workloads for rocprofv3 passes (kernel trace, PMC counters): ``--what unet`` = one C2 UNet forward (B=2,
128x128 latent, bf16; the prompt K/V and the condition embedding precomputed, as in the denoise loop); ``--what unet_fp8`` = the same with quantize_8bit weights and the
e4m3-MFMA Linears; ``--what vae`` = one 1024^2 fp16 VAE decode; ``--what attn`` = the 140 flash-attention
launches of one C2 forward.  Each is preceded by a calibration copy of known size (1 GiB -> 1 GiB, larger than
the Infinity Cache); fd_postprocess_u8 launches (never part of the workloads) mark the windows: [m1, m2) = the
copy, [m2, m3) = the measured workload.  The workload runs once eagerly first (warm caches and workspaces, same
kernels as the graph replays).  Writes /tmp/fdprof/pmc_<what>/meta.json (launch / FLOP / algorithmic-byte counts
per kernel family).  Run under rocprofv3 with ONE counter group per pass and no trace domains besides
--kernel-trace (scripts/prof.sh)."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "faithdiff-dev_amd"))
import torch  # noqa: E402


def unet_work(dev, fp8=False):
    from fdhip import arch, ops
    from fdhip.unet import HipUNet
    k, B = 128, 2
    sd = arch.random_init(arch.unet_param_shapes(True), seed=0, device=dev)
    if fp8:  # quantize_8bit weights, transformer Linears on the e4m3 MFMA (bench.py --fp8)
        sd = arch.quantize_e4m3(sd)
    unet = HipUNet(sd, dev, torch.bfloat16, fp8_mfma=fp8)
    del sd
    g = torch.Generator(device=dev).manual_seed(0)
    unet.set_context(torch.randn((2, 77, 2048), generator=g, device=dev))
    x = torch.randn((B * k * k, 4), generator=g, device=dev).to(torch.bfloat16)
    cond = torch.randn((B * k * k, 512), generator=g, device=dev).to(torch.bfloat16)
    t = torch.full((B,), 951.0, device=dev)
    tids = torch.tensor([[1024.0, 1024.0, 0, 0, 1024.0, 1024.0]] * B, device=dev)
    text = torch.randn((B, 1280), generator=g, device=dev)
    ops.reserve_gn_workspace(1 << 24, dev)
    name = "C2 1024 UNet forward" + (" (use_fp8, e4m3 MFMA Linears)" if fp8 else "")
    ie = unet.cond_embed(cond, B, k, k)  # once per tile in __call__ and in bench.py's step (not in the window)
    return name, lambda: unet.forward(x, t, tids, text, ie, B, k, k, cond_embedded=True)


def vae_work(dev):
    from fdhip import arch
    from fdhip.vae import HipDecoder
    sd = arch.random_init(arch.vae_param_shapes(), seed=3, device=dev)
    dec = HipDecoder(sd, dev, torch.float16)
    del sd
    h = w = 128
    z = (torch.randn((h * w, 4), generator=torch.Generator(device=dev).manual_seed(1), device=dev) * 8).half()
    return "VAE decode 1024", lambda: dec.decode(z, 1, h, w)


def attn_work(dev):
    from fdhip import ops
    launches = []
    for B, H, L, Lk, n in [(2, 10, 4096, 4096, 10), (2, 10, 4096, 77, 10), (2, 20, 1024, 1024, 60),
                           (2, 20, 1024, 77, 60)]:
        C = H * 64
        q = torch.randn(B * L, 3 * C, device=dev).to(torch.bfloat16)
        kv = torch.randn(B * Lk, 2 * C, device=dev).to(torch.bfloat16)
        o = torch.empty(B * L, C, device=dev, dtype=torch.bfloat16)
        launches.append((n, B, H, L, Lk, C, q, kv, o))

    def run():
        for n, B, H, L, Lk, C, q, kv, o in launches:
            for _ in range(n):
                ops.flash_attn(q, kv, kv[:, C:], o, B, H, L, Lk, 3 * C, 2 * C, 2 * C, C, L * 3 * C, Lk * 2 * C,
                               Lk * 2 * C, L * C, kv_mod=0, scale=0.125)
    return "C2 flash attention (one forward's 140 launches)", run


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--what", choices=("unet", "unet_fp8", "vae", "attn"), required=True)
    a = ap.parse_args()
    from fdhip import knobs
    from fdhip import lib as L
    from fdhip import ops
    knobs.apply_env()  # measurement script: FD_* knob overrides from the environment
    L.require_device()
    dev = torch.device("cuda", 0)
    work = {"unet": unet_work, "unet_fp8": lambda d: unet_work(d, fp8=True), "vae": vae_work, "attn": attn_work}
    name, fn = work[a.what](dev)
    fn()
    torch.cuda.synchronize()
    rec = []
    ops.set_recorder(rec)
    fn()  # the recorded (eager) pass also warms every workspace
    ops.set_recorder(None)
    torch.cuda.synchronize()
    fam = {}
    labels = [(kind, lab, fl) for kind, fl, nb, _, lab in rec]
    for kind, fl, nb, *_ in rec:
        c = fam.setdefault(kind, [0, 0.0, 0.0])
        c[0] += 1
        c[1] += fl
        c[2] += nb
    rows, cols = 16384, 32768
    src = torch.empty((rows, cols), dtype=torch.bfloat16, device=dev).normal_()
    dst = torch.empty_like(src)
    mk_in = torch.zeros(64, dtype=torch.float32, device=dev)
    mk_out = torch.empty(64, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    ops.postprocess_u8(mk_in, mk_out)
    dst.copy_(src)
    ops.postprocess_u8(mk_in, mk_out)
    fn()  # the measured pass
    ops.postprocess_u8(mk_in, mk_out)
    torch.cuda.synchronize()
    out = os.environ.get("FD_PMC_DIR") or os.path.join("/tmp/fdprof", f"pmc_{a.what}")
    os.makedirs(out, exist_ok=True)
    with open(os.path.join(out, "meta.json"), "w") as f:
        json.dump({"workload": name, "families": {k: {"launches": v[0], "flops": v[1], "algorithmic_bytes": v[2]}
                                                  for k, v in fam.items()},
                   "calib_bytes_read": rows * cols * 2, "calib_bytes_written": rows * cols * 2,
                   "labels": labels}, f, indent=1)
    print("ok", name, {k: v[0] for k, v in fam.items()})


if __name__ == "__main__":
    main()
