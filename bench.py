#!/usr/bin/env python3
"""FaithDiff denoising hot path on MI355X -- headline benchmark (BASELINE.json metric).

metric: denoise steps/s at 1024x1024 (C2: one 128x128 latent tile, CFG batch 2, 20-step Euler), plus the
fp16 VAE decode time at 1024^2.  A "step" = one pass of the hot path over one tile batch: TLC split +
scale_model_input -> UNet (SDXL + FaithDiff extras, bf16) -> CFG combine + Euler step -> gaussian blend,
exactly the per-step work of pipeline_FaithDiff_tlc.py:1324-1409.  Weights are seeded random-init of the
real architecture (2.58 B params), inputs synthetic; everything is resident in HBM before timing.

Multi-GPU (torchrun, one rank per GPU): every rank restores its own 1024^2 image (C5-style independent
images, no data-path collective), so `scaling` is "weak" and value = total steps/s of all ranks (timed
with a barrier + synchronize on both sides, max over ranks).  The tile-sharded path for one large image
(C3/C4, one all-gather per step) is FaithDiff/pipelines/tile_parallel.py, exercised by the tests.

roofline: the dominant kernel is the MFMA GEMM (gemm_kernel: every projection, FF and implicit-GEMM 3x3
conv of the UNet, ~76% of a step).  achieved = its algorithmic FLOPs (2*M*N*K per launch, summed over the
launches of one UNet forward) / the summed launch durations, each launch bracketed by HIP events on its
launch stream in an instrumented (eager) forward after the timed region; peak = 2500 TFLOP/s dense bf16
MFMA (MI355X_MICROARCH.md).  traffic = HBM bytes of the same launches from the committed rocprofv3 PMC
pass (profiles/r01_gemm_traffic.json: 2*FETCH_SIZE + WRITE_SIZE, gfx950 correction), else null.
"step_roofline" is the same ratio for the whole graph-replayed step (14.217 TFLOP analytic);
"attention" and "vae_norm" report flash-attention MFMA TFLOP/s and VAE GroupNorm HBM GB/s the same way.
cpu_baseline: the fp32 CPU oracle (the repo's restatement of the reference path) timed on this host for
a bounded sample (1 denoise step of the same C2 tile).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "faithdiff-dev_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

PEAK_BF16_TFLOPS = 2500.0
PEAK_FP8_TFLOPS = 5000.0  # dense e4m3 (block-scaled MFMA), MI355X_MICROARCH.md
PEAK_HBM_GBS = 8000.0


def event_pair_overhead_ms(n=64):
    """Median elapsed time of an event pair with nothing between them, on a busy-then-idle stream: the
    per-launch bias the probe subtracts (rocprofv3 --kernel-trace of the same run cross-checks it)."""
    x = torch.empty(1 << 20, device="cuda")
    ts = []
    for _ in range(n):
        x.mul_(1.0)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        e1.record()
        ts.append((e0, e1))
    torch.cuda.synchronize()
    v = sorted(a.elapsed_time(b) for a, b in ts)
    return v[len(v) // 2]


def probe(fn, reps=3):
    """Run fn() `reps` times with the per-launch event probe on; per kind: (launches, FLOPs, bytes, ms),
    averaged per call of fn, each launch's event time less the empty event-pair time."""
    from fdhip import ops
    bias = event_pair_overhead_ms()
    rec = []
    ops.set_probe(rec)
    try:
        for _ in range(reps):
            fn()
    finally:
        ops.set_probe(None)
    torch.cuda.synchronize()
    agg = {}
    for kind, fl, nb, e0, e1, *_ in rec:
        a = agg.setdefault(kind, [0, 0.0, 0.0, 0.0])
        a[0] += 1
        a[1] += fl
        a[2] += nb
        a[3] += max(e0.elapsed_time(e1) - bias, 1e-4)
    return {k: (v[0] // reps, v[1] / reps, v[2] / reps, v[3] / reps) for k, v in agg.items()}


def load_traffic():
    path = os.path.join(ROOT, "profiles", "r01_gemm_traffic.json")
    try:
        with open(path) as f:
            return json.load(f)
    except (OSError, ValueError):
        return None


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--size", type=int, default=1024, help="image side (latent = size/8)")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--fp8", action="store_true", help="use_fp8 model (quantize_8bit weights; transformer Linears "
                                                       "on the e4m3 MFMA): the C4 arithmetic on the C2 tile")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-vae", action="store_true")
    ap.add_argument("--profile-steps", type=int, default=0, help="extra untimed steps (for rocprof windows)")
    return ap.parse_args()


def setup_dist(n):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    return world, rank, local


def build(size, seed, fp8=False):
    from fdhip import arch
    from fdhip.unet import HipUNet
    dev = torch.device("cuda", torch.cuda.current_device())
    sd = arch.random_init(arch.unet_param_shapes(True), seed=seed, device=dev)
    if fp8:
        sd = arch.quantize_e4m3(sd)
    unet = HipUNet(sd, dev, torch.bfloat16, fp8_mfma=fp8)
    del sd
    return unet


def cpu_baseline(size):
    """One denoise step of the same C2 tile with the fp32 CPU oracle (test infrastructure, not shipped)."""
    sys.path.insert(0, ROOT)
    from oracle import schedulers as S
    from oracle.unet import UNet2DConditionModel
    threads = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    threads = max(1, min(threads, 64))
    torch.set_num_threads(threads)
    with torch.no_grad():
        ref = UNet2DConditionModel()
        for p in ref.parameters():  # values do not affect CPU time; keep init cheap
            p.uniform_(-0.02, 0.02)
        ref.eval()
        h = size // 8
        g = torch.Generator().manual_seed(0)
        x = torch.randn(1, 4, h, h, generator=g)
        cond = torch.randn(1, 512, h, h, generator=g)
        ctx = torch.randn(2, 77, 2048, generator=g)
        text = torch.randn(2, 1280, generator=g)
        tids = torch.tensor([[size, size, 0, 0, size, size]] * 2, dtype=torch.float32)
        ts, sig, _ = S.euler_schedule(20)
        t0 = time.perf_counter()
        xin = S.euler_scale(torch.cat([x] * 2), float(sig[0]))
        eps = ref(xin, ts[0], ctx, {"text_embeds": text, "time_ids": tids}, input_embedding=torch.cat([cond] * 2))
        u, c = eps.chunk(2)
        S.euler_step(u + 5.0 * (c - u), x, float(sig[0]), float(sig[1]))
        dt = time.perf_counter() - t0
    return {"value": 1.0 / dt, "unit": "steps/s", "cores": threads, "kind": "port",
            "sample": f"1 denoise step (UNet fwd B=2 @ {h}x{h} latent + CFG/Euler) of C2, fp32 oracle, "
                      f"{threads} host threads, {dt:.1f} s"}


def main():
    args = parse()
    world, rank, local = setup_dist(args.gpus)
    from fdhip import arch, ops
    from fdhip import lib as L
    L.require_device()
    dev = torch.device("cuda", torch.cuda.current_device())
    h = w = args.size // 8
    k = min(128, h)
    cfg, B = 2, 2
    unet = build(args.size, seed=0, fp8=args.fp8)

    g = torch.Generator(device=dev).manual_seed(1234 + rank)
    canvas = torch.randn((4, h, w), generator=g, device=dev) * 11.0
    canvas_next = torch.empty_like(canvas)
    cond = (torch.randn((B * k * k, 512), generator=g, device=dev)).to(torch.bfloat16)
    ctx = torch.randn((2, 77, 2048), generator=g, device=dev)
    text = torch.randn((B, 1280), generator=g, device=dev)
    tids = torch.tensor([[args.size, args.size, 0, 0, args.size, args.size]] * B, dtype=torch.float32, device=dev)
    rows = torch.tensor([0], dtype=torch.int32, device=dev)
    cols = torch.tensor([0], dtype=torch.int32, device=dev)
    from FaithDiff.pipelines.tlc import TileGrid
    from FaithDiff.schedulers import EulerDiscreteScheduler
    grid = TileGrid(h, w, (128, 128), 0.5)
    rows = torch.tensor(grid.rows, dtype=torch.int32, device=dev)
    cols = torch.tensor(grid.cols, dtype=torch.int32, device=dev)
    weights = torch.tensor(grid.weights(), dtype=torch.float64, device=dev)
    sch = EulerDiscreteScheduler()
    sch.set_timesteps(20)
    sig = sch.sigmas
    unet.set_context(ctx)
    xin = torch.empty((B * k * k, 4), dtype=torch.bfloat16, device=dev)
    t_buf = torch.full((B,), float(sch.timesteps[0]), device=dev)
    out_tiles = torch.empty((grid.ntiles, 4, k, k), device=dev)
    ops.reserve_gn_workspace(1 << 24, dev)

    def unet_fwd():
        return unet.forward(xin, t_buf, tids, text, cond, B, k, k)

    graph = None
    eps_static = None
    if not args.no_graph:
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(2):
                unet_fwd()
        torch.cuda.current_stream().wait_stream(s)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            eps_static = unet_fwd()

    state = {"cv": canvas, "nx": canvas_next}

    def step(i):
        s_, sn = float(sig[i % 20]), float(sig[i % 20 + 1])
        ops.tlc_scale_input(state["cv"], rows, cols, h, w, k, k, 0, grid.ntiles, cfg, s_, xin)
        t_buf.fill_(float(sch.timesteps[i % 20]))
        if graph is not None:
            graph.replay()
            eps = eps_static
        else:
            eps = unet_fwd()
        ops.tlc_cfg_euler_step(eps, state["cv"], rows, cols, h, w, k, k, 0, grid.ntiles, cfg, 5.0, 0.0, s_, sn,
                               out_tiles)
        ops.tlc_blend(out_tiles, weights, rows, cols, 4, h, w, k, k, state["nx"])
        state["cv"], state["nx"] = state["nx"], state["cv"]

    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record()
    for i in range(args.steps):
        step(i)
    ev1.record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    wall = time.perf_counter() - t0
    ev_ms = ev0.elapsed_time(ev1)
    t_local = torch.tensor([wall], device=dev)
    if world > 1:
        dist.all_reduce(t_local, op=dist.ReduceOp.MAX)
    t_max = float(t_local.item())
    for i in range(args.profile_steps):
        step(i)
    torch.cuda.synchronize()
    # instrumented eager forwards (outside the timed region): per-kernel-family durations
    kstats = probe(unet_fwd)

    # ---- VAE decode at the same size (ms), separately timed
    vae_ms, vstats = None, {}
    if not args.no_vae:
        from fdhip.vae import HipDecoder
        vsd = arch.random_init(arch.vae_param_shapes(), seed=3, device=dev)
        dec = HipDecoder(vsd, dev, torch.float16)
        del vsd
        z = torch.empty((h * w, 4), dtype=torch.float16, device=dev)
        ops.nchw_to_nhwc(state["cv"], z, 1, 4, h * w, 1.0 / 0.13025)
        for _ in range(2):
            dec.decode(z, 1, h, w)
        torch.cuda.synchronize()
        times = []
        for _ in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            dec.decode(z, 1, h, w)
            e1.record()
            torch.cuda.synchronize()
            times.append(e0.elapsed_time(e1))
        vae_ms = sorted(times)[1]
        vstats = probe(lambda: dec.decode(z, 1, h, w), reps=2)

    steps_total = args.steps * world
    value = steps_total / t_max
    ms_step = t_max / args.steps * 1e3
    flops = arch.unet_flops(k, k, B)
    step_s = ev_ms / 1e3 / args.steps
    achieved = flops / step_s / 1e12
    n_g, fl_g, _, ms_g = kstats["gemm"]
    gemm_tf = fl_g / (ms_g / 1e3) / 1e12
    tr = load_traffic()
    traffic = None
    if tr and tr.get("workload") == f"C2 {args.size}" and not args.fp8:
        traffic = tr["hbm_bytes_per_forward"]
    n_a, fl_a, _, ms_a = kstats["flash_attn"]
    attn_tf = fl_a / (ms_a / 1e3) / 1e12
    vae_norm = None
    if "group_norm" in vstats:
        n_n, _, nb_n, ms_n = vstats["group_norm"]
        vae_norm = {"bound": "hbm", "achieved": round(nb_n / (ms_n / 1e3) / 1e9, 1), "peak": PEAK_HBM_GBS,
                    "unit": "GB/s", "frac": round(nb_n / (ms_n / 1e3) / 1e9 / PEAK_HBM_GBS, 4),
                    "launches": n_n, "ms": round(ms_n, 3), "algorithmic_bytes": nb_n}
    result = {
        "metric": "denoise steps/sec @1024px 20-step + VAE decode ms",
        "value": round(value, 4), "unit": "steps/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(ms_step, 3), "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "fp8-e4m3+bf16" if args.fp8 else "bf16", "data": "synthetic (seeded random-init SDXL+FaithDiff weights, random latents/conditions)",
        "config": {"workload": f"C2: {args.size}x{args.size} single TLC tile, CFG batch 2, Euler step + blend, "
                               f"UNet {'use_fp8: transformer Linears e4m3 MFMA, convs bf16' if args.fp8 else 'bf16'} "
                               f"(hipGraph={graph is not None}), VAE fp16",
                   "model": "SDXL UNet + FaithDiff extras (2.58B params)", "global_batch": 2 * world,
                   "latent": [h, w], "parallelism": f"replicas x{world}"},
        "vae_decode_ms": None if vae_ms is None else round(vae_ms, 2),
        "vae_decode_tflops": None if vae_ms is None else round(arch.vae_decode_flops(h, w) / (vae_ms / 1e3) / 1e12, 1),
        "roofline": {"bound": "mfma", "achieved": round(gemm_tf, 1), "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
                     "frac": round(gemm_tf / PEAK_BF16_TFLOPS, 4), "traffic": traffic,
                     "kernel": "gemm8_kernel + gemm_kernel (all MFMA GEMM + implicit-GEMM conv launches of one UNet forward)",
                     "launches": n_g, "algorithmic_flops": fl_g, "kernel_ms_per_forward": round(ms_g, 3),
                     "avg_launch_us": round(ms_g / n_g * 1e3, 2),
                     "traffic_note": "HBM bytes per forward of these launches (PMC pass)" if traffic else
                                     "no PMC pass committed for this workload"},
        "step_roofline": {"bound": "mfma", "achieved": round(achieved, 1), "peak": PEAK_BF16_TFLOPS,
                          "unit": "TFLOP/s", "frac": round(achieved / PEAK_BF16_TFLOPS, 4),
                          "algorithmic_flops_per_step": flops, "event_ms_per_step": round(step_s * 1e3, 3)},
        "attention": {"bound": "mfma", "achieved": round(attn_tf, 1), "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
                      "frac": round(attn_tf / PEAK_BF16_TFLOPS, 4), "launches": n_a, "ms": round(ms_a, 3)},
        "vae_norm": vae_norm,
        "kernel_ms_per_forward": {k: round(v[3], 3) for k, v in kstats.items()},
    }
    if "gemm_e4m3" in kstats:  # use_fp8: the e4m3 Linears against the fp8 peak (the bf16 roofline above = convs)
        n_f, fl_f, _, ms_f = kstats["gemm_e4m3"]
        f8_tf = fl_f / (ms_f / 1e3) / 1e12
        result["roofline_fp8"] = {"bound": "mfma", "achieved": round(f8_tf, 1), "peak": PEAK_FP8_TFLOPS,
                                  "unit": "TFLOP/s", "frac": round(f8_tf / PEAK_FP8_TFLOPS, 4),
                                  "kernel": "gemm_e4m3_dma_kernel (transformer Linears, e4m3 x e4m3)",
                                  "launches": n_f, "algorithmic_flops": fl_f, "kernel_ms_per_forward": round(ms_f, 3)}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            result["cpu_baseline"] = cpu_baseline(args.size)
        except Exception as e:  # the baseline must not sink the GPU measurement
            result["cpu_baseline"] = {"value": None, "error": repr(e)}
    if rank == 0:
        print(json.dumps(result))
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
