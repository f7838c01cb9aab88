#!/usr/bin/env python3
"""FaithDiff denoising hot path on MI355X -- headline benchmark (BASELINE.json metric).

metric: denoise steps/s at 1024x1024 (C2 = BASELINE configs[1]: one 128x128 latent tile, CFG batch 2, 20-step
Euler), plus the fp16 VAE decode time at 1024^2.  A "step" = one pass of the hot path over one tile batch: TLC
split + scale_model_input -> UNet (SDXL + FaithDiff extras, bf16; one hipGraph replay through HipUNet.run, the
same call the pipeline's denoise loop makes) -> CFG combine + Euler step -> gaussian blend, i.e. the per-step
work of pipeline_FaithDiff_tlc.py:1324-1409.  Weights are seeded random-init of the real architecture (2.58 B
params, built by the product factory FaithDiff_pipeline('random-init', ...)), inputs synthetic; everything is
resident in HBM before timing.

Launch: ``python bench.py --gpus N`` starts N rank processes itself (torch.distributed.run, before any GPU call)
unless it already runs under torchrun (WORLD_SIZE set, which must equal N).

Workloads (``--workload``; all ranks time exactly --steps steps between barrier + synchronize, max over ranks):
  c2 (default)  every rank restores its own 1024^2 image (replicas, no data-path collective): value = total
                steps/s, scaling "weak".  The same line also carries
                  * "pipeline": the product ``pipe(...)`` call end to end at C2 (encode_prompt, denoise encoder,
                    VAE encode, 20 steps, VAE decode, postprocess) -- s/image and its per-step time;
                  * "c3": BASELINE configs[2] -- one 4096^2 image (49 TLC tiles, tiled VAE) restored by ALL
                    ranks together through the product pipeline with ``enable_tile_parallel`` (tiles sharded,
                    one all_gather_into_tensor per step over RCCL, sharded tiled decode): s/image, tile-steps/s;
  c3            the C3 image is the timed unit: value = tile-steps/s of the whole job (strong scaling);
  c4            BASELINE configs[3], 8K-output reading: one 8192^2 image (2048^2 input after the 4x upscale,
                225 TLC tiles) through the same tile-sharded path on the use_fp8 model (e4m3 MFMA Linears):
                value = tile-steps/s of the whole job (strong scaling);
  c5            BASELINE configs[4]: 8 images of 1024^2 x 50 steps split over the ranks: value = images/s.

roofline: the dominant kernel family is the MFMA GEMM (gemm8_kernel + gemm_kernel: every projection, FF and
implicit-GEMM conv of the UNet, ~80 % of a step).  While the UNet forward is captured, every launch is also
recorded (ops.set_recorder); the GEMM launches of one forward are then captured on their own into a second
hipGraph and that graph is timed with HIP events on its stream: achieved = sum 2*M*N*K of those launches / the
measured time per forward.  The same is done for flash attention ("attention") and for the VAE decoder's
GroupNorms ("vae_norm", HBM bytes).  profiles/<round>_roofline_check.json recomputes each figure from the
rocprofv3 kernel trace of the same command.  peak: 2500 TFLOP/s dense bf16 MFMA (MI355X_MICROARCH.md).
traffic: HBM bytes of the same launches from the committed rocprofv3 PMC pass (profiles/*_gemm_traffic.json).
cpu_baseline: the fp32 CPU oracle (the repo's restatement of the reference path; the reference itself cannot run
here: diffusers is absent) timed on this host for a bounded sample (1 denoise step of the same C2 tile).
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "faithdiff-dev_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

PEAK_BF16_TFLOPS = 2500.0
PEAK_FP8_TFLOPS = 5000.0  # dense e4m3 (block-scaled MFMA), MI355X_MICROARCH.md
PEAK_HBM_GBS = 8000.0
# committed rocprofv3 PMC traffic passes (scripts/prof.sh + scripts/traffic_from_pmc.py), newest round first: the
# file names start with the round tag (r04 > r03c > r03 > r02f), so a reverse name sort is newest first
TRAFFIC_FILES = sorted((os.path.join(ROOT, "profiles", f) for f in os.listdir(os.path.join(ROOT, "profiles"))
                        if "_gemm_traffic" in f and f.endswith(".json")), reverse=True)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", choices=("c2", "c3", "c4", "c5"), default="c2")
    ap.add_argument("--size", type=int, default=1024, help="C2 image side (latent = size/8)")
    ap.add_argument("--fp8", action="store_true", help="use_fp8 model (quantize_8bit weights; transformer Linears "
                                                       "on the e4m3 MFMA): the C4 arithmetic")
    ap.add_argument("--unet-fp16", action="store_true", help="UNet computing in fp16 (the reference's own UNet dtype, "
                                                             "create_FaithDiff_model.py:21-22) instead of bf16 "
                                                             "(BASELINE configs[1], the default)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-vae", action="store_true")
    ap.add_argument("--no-pipeline", action="store_true", help="skip the C2 pipe(...) s/image leg")
    ap.add_argument("--no-c3", action="store_true", help="skip the C3 leg of the c2 workload")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--c3-size", type=int, default=4096)
    ap.add_argument("--c3-steps", type=int, default=20)
    ap.add_argument("--c4-size", type=int, default=8192, help="C4 output side (8K output reading of configs[3])")
    ap.add_argument("--c5-images", type=int, default=8)
    ap.add_argument("--c5-steps", type=int, default=50)
    ap.add_argument("--profile-steps", type=int, default=0, help="extra untimed steps (for rocprof windows)")
    return ap.parse_args(argv)


# ------------------------------------------------------------------------------------------------ launch
def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launcher_cmd(argv, n, port):
    """The torchrun command that runs this script as n ranks (the driver's own form of the N-GPU run)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)


def maybe_launch(args, argv):
    """--gpus N without WORLD_SIZE: start N rank processes (before anything touches the GPU) and return their
    exit code; under torchrun, WORLD_SIZE must equal --gpus.  Returns None when this process is a rank."""
    world = os.environ.get("WORLD_SIZE")
    if world is None:
        if args.gpus > 1:
            env = dict(os.environ, MASTER_ADDR="127.0.0.1")
            return subprocess.call(launcher_cmd(argv, args.gpus, _free_port()), env=env)
        return None
    if int(world) != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; refusing to report a mislabelled run",
              file=sys.stderr)
        return 2
    return None


def setup_dist():
    """One rank per GPU over RCCL ('nccl').  FD_BENCH_REHEARSAL=1 (tests on a one-GPU box only) puts every rank
    on cuda:0 with gloo, to exercise the N-rank code path where N GPUs are not available."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    rehearsal = os.environ.get("FD_BENCH_REHEARSAL") == "1"
    if rehearsal:
        local = 0
    torch.cuda.set_device(local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if rehearsal:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    return world, rank, local


def barrier(world):
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()


def max_over_ranks(x, world, dev):
    if world > 1 and dist.get_backend() == "gloo":
        dev = torch.device("cpu")
    t = torch.tensor([float(x)], device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


# ------------------------------------------------------------------------------------------------ model
def build_pipe(dev, fp8, world=1, unet_dtype=torch.bfloat16):
    """The product factory; with N ranks it is built collectively (process_group=WORLD): rank 0 alone reads / draws
    the weights and broadcasts them over RCCL before anything is packed (pipe.last_broadcast_bytes)."""
    from CKPT_PTH import FAITHDIFF_PATH, SDXL_PATH, VAE_FP16_PATH  # 'random-init' sentinels offline
    from FaithDiff.create_FaithDiff_model import FaithDiff_pipeline
    t0 = time.perf_counter()
    pipe = FaithDiff_pipeline(SDXL_PATH, VAE_FP16_PATH, FAITHDIFF_PATH, use_fp8=fp8, fp8_mfma=fp8 or None, seed=0,
                              init_device=dev, process_group=dist.group.WORLD if world > 1 else None,
                              unet_dtype=unet_dtype)
    pipe.build_s = time.perf_counter() - t0
    pipe = pipe.to(dev)
    pipe.unet.release_host_weights()
    return pipe


def synthetic_image(H, W, seed):
    """A smooth seeded RGB test card (content does not change the work; parity uses tests/golden inputs)."""
    from PIL import Image
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:H, 0:W].astype(np.float32)
    img = np.zeros((H, W, 3), np.float32)
    for c in range(3):
        fx, fy = rng.uniform(1, 8, 2)
        img[..., c] = np.sin(xx / W * fx * 6.28) * np.cos(yy / H * fy * 6.28)
    img += rng.normal(0, 0.1, (H, W, 3)).astype(np.float32)
    img = (img - img.min()) / (img.max() - img.min())
    return Image.fromarray((img * 255).astype(np.uint8))


class EventTimer:
    """The pipeline's ``timer`` hook: an event per (label, step) on the current stream."""

    def __init__(self):
        self.ev = []

    def __call__(self, label, i):
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        self.ev.append((label, i, e))

    def step_ms(self):
        st = [e for (lab, _, e) in self.ev if lab in ("loop_start", "step")]
        d = [a.elapsed_time(b) for a, b in zip(st[:-1], st[1:])]
        return d

    def gather_ms(self):
        """Per-step durations of the tile exchange (run_tile_loop's "gather_start" / "gather_end" events)."""
        a = [e for (lab, _, e) in self.ev if lab == "gather_start"]
        b = [e for (lab, _, e) in self.ev if lab == "gather_end"]
        return [x.elapsed_time(y) for x, y in zip(a, b)]

    def span_ms(self, a, b):
        ea = next(e for (lab, _, e) in self.ev if lab == a)
        eb = next(e for (lab, _, e) in reversed(self.ev) if lab == b)
        return ea.elapsed_time(eb)


# ------------------------------------------------------------------------------------------------ C2 hot loop
class C2Loop:
    """The per-step work of pipeline_FaithDiff_tlc.py:1324-1409 for one 128^2 tile (C2), on the pipeline's own
    HipUNet.  Each step: fd_tlc_scale_input -> HipUNet.run (hipGraph replay) -> fd_tlc_cfg_euler_step ->
    fd_tlc_blend."""

    def __init__(self, pipe, size, rank):
        from FaithDiff.pipelines.tlc import TileGrid
        from FaithDiff.schedulers import EulerDiscreteScheduler
        from fdhip import ops
        self.ops = ops
        self.unet = unet = pipe.unet.hip()
        dev = unet.device
        self.h = self.w = h = size // 8
        self.k = k = min(128, h)
        self.cfg, self.B = 2, 2
        g = torch.Generator(device=dev).manual_seed(1234 + rank)
        self.canvas = torch.randn((4, h, h), generator=g, device=dev) * 11.0
        self.nxt = torch.empty_like(self.canvas)
        self.cond = torch.randn((self.B * k * k, 512), generator=g, device=dev).to(unet.dtype)
        self.ctx = ctx = torch.randn((2, 77, 2048), generator=g, device=dev)
        self.text = torch.randn((self.B, 1280), generator=g, device=dev)
        self.tids = torch.tensor([[size, size, 0, 0, size, size]] * self.B, dtype=torch.float32, device=dev)
        self.grid = TileGrid(h, h, (128, 128), 0.5)
        self.rows = torch.tensor(self.grid.rows, dtype=torch.int32, device=dev)
        self.cols = torch.tensor(self.grid.cols, dtype=torch.int32, device=dev)
        self.weights = torch.tensor(self.grid.weights(), dtype=torch.float64, device=dev)
        sch = EulerDiscreteScheduler()
        sch.set_timesteps(20)
        self.sig, self.ts = [float(s) for s in sch.sigmas], [float(t) for t in sch.timesteps]
        unet.set_context(ctx)
        self.xin = torch.empty((self.B * k * k, 4), dtype=unet.dtype, device=dev)
        self.ie = torch.empty((self.B * k * k, 320), dtype=unet.dtype, device=dev)
        self.t_buf = torch.full((self.B,), self.ts[0], device=dev)
        self.static = None
        self.static_tried = False  # graph_inputs() asked once after the capture step (None for good with FD_GRAPHS=0)
        self.per_image()
        self.out_tiles = torch.empty((self.grid.ntiles, 4, k, k), device=dev)
        ops.reserve_gn_workspace(1 << 24, dev)

    def args(self):
        return (self.xin, self.t_buf, self.tids, self.text, self.ie, self.B, self.k, self.k)

    def per_image(self):
        """What __call__ does once per image: the prompt's attn2 K/V projection (set_context) and the condition
        embedding of the tile's image latents (cond_embed).  Once run()'s graph is captured, the per-image inputs
        (condition embedding, time ids, pooled text) are written into its static buffers here, and every step writes
        its latent tile and timestep there too (fd_tlc_scale_input_t): a step is HIP kernels only, no input copies."""
        self.unet.set_context(self.ctx)
        if self.static is None:
            st = self.unet.graph_inputs(self.B, self.k, self.k, cond_embedded=True)
            if st is not None:
                self.static = st
                self.xin, self.t_buf = st[0], st[1]
                st[2].copy_(self.tids)
                st[3].copy_(self.text)
                self.tids, self.text, self.ie = st[2], st[3], st[4]
        self.ie = self.unet.cond_embed(self.cond, self.B, self.k, self.k, out=self.ie)

    def step(self, i):
        ops, k, h = self.ops, self.k, self.h
        # once per 20-step image, as __call__ does; and once at step 2, when run()'s graph has been captured, to move
        # the per-image inputs into its static buffers (never again when graphs are off: FD_GRAPHS=0 A/B arms)
        if i % 20 == 0 or (i >= 2 and not self.static_tried):
            self.static_tried = i >= 2
            self.per_image()
        s_, sn = self.sig[i % 20], self.sig[i % 20 + 1]
        ops.tlc_scale_input(self.canvas, self.rows, self.cols, h, h, k, k, 0, self.grid.ntiles, self.cfg, s_,
                            self.xin, t_out=self.t_buf, timestep=self.ts[i % 20])
        eps = self.unet.run(*self.args(), cond_embedded=True)
        ops.tlc_cfg_euler_step(eps, self.canvas, self.rows, self.cols, h, h, k, k, 0, self.grid.ntiles, self.cfg,
                               5.0, 0.0, s_, sn, self.out_tiles)
        ops.tlc_blend(self.out_tiles, self.weights, self.rows, self.cols, 4, h, h, k, k, self.nxt)
        self.canvas, self.nxt = self.nxt, self.canvas


# ------------------------------------------------------------------------------------------------ kernel families
def family_times(fn, kinds, reps=20):
    """Capture fn() into a hipGraph with the launch recorder on, then capture the launches of each kind on their
    own into a second graph and time its replays with HIP events.  Returns {kind: (launches, flops, bytes,
    ms per call of fn)} plus the full graph's ms per call under key '_all'."""
    from fdhip import ops
    rec = []
    torch.cuda.synchronize()
    g_all = torch.cuda.CUDAGraph()
    ops.set_recorder(rec)
    try:
        with torch.cuda.graph(g_all):
            fn()
    finally:
        ops.set_recorder(None)
    out = {}

    def timed(g):
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps

    g_all.replay()
    out["_all"] = (len(rec), sum(r[1] for r in rec), sum(r[2] for r in rec), timed(g_all))
    for kind in kinds:
        sel = [r for r in rec if r[0] == kind]
        if not sel:
            continue
        gk = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gk):
            for r in sel:
                r[3]()
        out[kind] = (len(sel), sum(r[1] for r in sel), sum(r[2] for r in sel), timed(gk))
        del gk
    del g_all
    return out


def load_traffic_floor():
    """The newest committed 8-XCD traffic floor of the bf16 C2 forward (scripts/gemm_traffic_floor.py), or None."""
    for path in sorted((os.path.join(ROOT, "profiles", f) for f in os.listdir(os.path.join(ROOT, "profiles"))
                        if f.endswith("_gemm_traffic_floor.json")), reverse=True):
        try:
            with open(path) as f:
                fl = json.load(f)
            return (fl["read_floor_8xcd_gb"] + fl["write_gb"]) * 1e9, os.path.basename(path)
        except (OSError, ValueError, KeyError):
            continue
    return None


def load_traffic(workload):
    """The newest committed traffic file measured on this workload (its key), or None."""
    for path in TRAFFIC_FILES:
        try:
            with open(path) as f:
                tr = json.load(f)
        except (OSError, ValueError):
            continue
        if tr.get("workload") == workload:
            tr["file"] = os.path.basename(path)
            return tr
    return None


# ------------------------------------------------------------------------------------------------ legs
def cpu_baseline(size):
    """One denoise step of the same C2 tile with the fp32 CPU oracle (test infrastructure, not shipped)."""
    sys.path.insert(0, ROOT)
    from oracle import schedulers as S
    from oracle.unet import UNet2DConditionModel
    threads = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    threads = max(1, min(threads, int(os.environ.get("OMP_NUM_THREADS", threads))))
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
                      f"{threads} host threads (OMP_NUM_THREADS / affinity), {dt:.1f} s"}


def run_pipeline_image(pipe, img, H, W, steps, target, seed=42):
    """One product ``pipe(...)`` call as test_wo_llava.py:86 makes it; returns (s, EventTimer).  The final latents
    are checked for non-finite values after the timed call (tm.finite)."""
    tm = EventTimer()
    gen = torch.Generator(device=pipe.device).manual_seed(seed)
    last = {}

    def keep(p, i, t, kw):  # keeps a reference only; inspected after the clock stops
        last["lat"] = kw["latents"]
        return {}
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tm("call_start", 0)
    pipe(lr_img=img, prompt="A high quality photo restored from a degraded capture.", negative_prompt="",
         num_inference_steps=steps, guidance_scale=5.0, generator=gen, start_point="lr", height=H, width=W,
         overlap=0.5, target_size=target, timer=tm, callback_on_step_end=keep)
    tm("call_end", 0)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    tm.finite = bool(torch.isfinite(last["lat"]).all().item()) if "lat" in last else None
    return el, tm


def run_batch(pipe, imgs, prompts, size, steps, seed=42):
    """One product pipe(lr_img=[...], prompt=[...]) call over several images (C5); returns its EventTimer, the
    images and the final latents (a reference to the device tensor, kept by the step-end callback: no copy, no
    sync inside the timed call).  check_batch() validates them outside the timed region."""
    tm = EventTimer()
    gen = torch.Generator(device=pipe.device).manual_seed(seed)
    last = {}

    def keep(p, i, t, k):
        last["latents"] = k["latents"]
        return {}
    tm("call_start", 0)
    out = pipe(lr_img=imgs, prompt=prompts, negative_prompt="", num_inference_steps=steps, guidance_scale=5.0,
               generator=gen, start_point="lr", height=size, width=size, overlap=0.5, target_size=(1024, 1024),
               timer=tm, callback_on_step_end=keep).images
    tm("call_end", 0)
    torch.cuda.synchronize()
    return tm, out, last.get("latents")


def check_batch(out, latents, n):
    """C5 output check: one image per input, final latents finite, no flat image (a NaN or a dropped image would
    otherwise go unnoticed in the timed leg)."""
    if len(out) != n or latents is None or latents.shape[0] != n:
        raise RuntimeError(f"C5 batch: {len(out)} images / latents {None if latents is None else tuple(latents.shape)}"
                           f" for {n} inputs")
    if not bool(torch.isfinite(latents).all()):
        raise RuntimeError("C5 batch: non-finite latents")
    stds = [float(np.asarray(im, dtype=np.float32).std()) for im in out]
    if min(stds) <= 1.0:
        raise RuntimeError(f"C5 batch: flat output image (pixel std {min(stds):.3f})")
    return stds


def pipeline_leg(pipe, size, steps=20):
    img = synthetic_image(size, size, 5)
    run_pipeline_image(pipe, img, size, size, 2, (1024, 1024))  # warm: captures the UNet / VAE graphs
    s, tm = run_pipeline_image(pipe, img, size, size, steps, (1024, 1024))
    st = tm.step_ms()
    return {"workload": f"C2 pipe(...) {size}x{size}, {steps} Euler steps, start_point 'lr', CFG 5, test_wo_llava.py "
                        "call (encode_prompt + denoise encoder + VAE encode + denoise loop + VAE decode + postprocess)",
            "s_per_image": round(s, 4), "loop_ms": round(sum(st), 2),
            "step_ms_median": round(float(np.median(st)), 3), "step_ms_min": round(min(st), 3),
            "decode_ms": round(tm.span_ms("decode_start", "decode"), 2),
            "pre_loop_ms": round(tm.span_ms("call_start", "loop_start"), 2), "latents_finite": tm.finite}


def c3_run(pipe, world, rank, dev, size, steps, warm=True, tag="C3"):
    """BASELINE configs[2]: one size^2 image (49 TLC tiles at 4096^2) restored by all ranks together (configs[3]
    at 8192^2, 225 tiles, with the use_fp8 model)."""
    from FaithDiff.pipelines.tlc import TileGrid
    if world > 1 and pipe.process_group is None:
        pipe.enable_tile_parallel()
    pipe.enable_vae_tiling()
    img = synthetic_image(size, size, 6)
    ntiles = TileGrid(size // 8, size // 8, (128, 128), 0.5).ntiles
    try:
        if warm:
            run_pipeline_image(pipe, img, size, size, 1, (1024, 1024))
        barrier(world)
        s, tm = run_pipeline_image(pipe, img, size, size, steps, (1024, 1024))
        barrier(world)
    finally:
        pipe.disable_vae_tiling()
    s = max_over_ranks(s, world, dev)
    st = tm.step_ms()
    loop_s = max_over_ranks(sum(st) / 1e3, world, dev)
    gm = tm.gather_ms()
    per = -(-ntiles // world)
    counts = [max(0, min(ntiles, r * per + per) - r * per) for r in range(world)]
    return {"workload": f"{tag}: {size}x{size} tiled restoration, {ntiles} TLC tiles x {steps} Euler steps, tiled VAE "
                        f"encode/decode, tiles sharded over {world} rank(s), one all_gather_into_tensor per step",
            "ntiles": ntiles, "steps": steps, "n_ranks": world, "s_per_image": round(s, 3),
            "loop_s": round(loop_s, 3), "tile_steps_per_s": round(ntiles * steps / loop_s, 3),
            "step_ms_median": round(float(np.median(st)), 2),
            "pre_loop_ms": round(tm.span_ms("call_start", "loop_start"), 1),
            "decode_ms": round(tm.span_ms("decode_start", "decode"), 1),
            "all_gather_bytes_per_step": per * world * 4 * 128 * 128 * 4 if world > 1 else 0,
            # the per-step exchange, HIP events around TileShard.gather on the loop's stream (max over ranks): with
            # tiles_per_rank it tells whether the exchange or the largest shard bounds a multi-GPU step
            "all_gather_ms_per_step": round(max_over_ranks(float(np.mean(gm)), world, dev), 3) if gm else 0.0,
            "all_gather_ms_max": round(max_over_ranks(max(gm), world, dev), 3) if gm else 0.0,
            "tiles_per_rank": counts, "latents_finite": tm.finite}


def roofline_leg(loop, fp8):
    from fdhip import arch
    fam = family_times(lambda: loop.unet.forward(*loop.args(), cond_embedded=True), ["gemm", "flash_attn", "gemm_e4m3"])
    n_g, fl_g, nb_g, ms_g = fam["gemm"]
    gemm_tf = fl_g / (ms_g / 1e3) / 1e12
    res = {}
    tr = load_traffic(f"C2 {loop.h * 8}" + (" (use_fp8, e4m3 MFMA Linears)" if fp8 else ""))
    tr16 = None if fp8 else tr  # the fp8 file's bytes are the e4m3 family's (roofline_fp8), not this one's
    res["roofline"] = {
        "bound": "mfma", "achieved": round(gemm_tf, 1), "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
        "frac": round(gemm_tf / PEAK_BF16_TFLOPS, 4),
        "traffic": None if tr16 is None else tr16["hbm_bytes_per_forward"],
        "kernel": "gemm8_kernel + gemm256_kernel + gemm_kernel (all MFMA GEMM + implicit-GEMM conv launches of one UNet forward)",
        "launches": n_g, "algorithmic_flops": fl_g, "kernel_ms_per_forward": round(ms_g, 3),
        # every operand once per launch (ops._gemm_bytes: A or the conv source image, weights, output, residual);
        # traffic / algorithmic_bytes is the re-read factor (per-XCD L2 replication)
        "algorithmic_bytes": nb_g,
        "traffic_ratio": None if tr16 is None else round(tr16["hbm_bytes_per_forward"] / nb_g, 3),
        "avg_launch_us": round(ms_g / n_g * 1e3, 2),
        "method": "the forward's GEMM launches captured on their own into one hipGraph, replayed 20x between HIP "
                  "events on the capture stream",
        "traffic_note": "HBM bytes per forward of these launches (rocprofv3 PMC pass, " + tr16["file"] + ")"
                        if tr16 else "no PMC pass committed for this workload"}
    fl = None if fp8 or loop.h * 8 != 1024 else load_traffic_floor()
    if fl is not None and tr16 is not None:
        # the lower bound any XCD-contiguous tile order has: each XCD's L2 misses once on every A / W panel its tiles
        # touch; traffic / floor is the part a tile order or L2 reuse could still remove
        res["roofline"]["traffic_floor_8xcd"] = round(fl[0])
        res["roofline"]["traffic_over_floor"] = round(tr16["hbm_bytes_per_forward"] / fl[0], 3)
        res["roofline"]["traffic_floor_note"] = "scripts/gemm_traffic_floor.py, " + fl[1]
    if "flash_attn" in fam:
        n_a, fl_a, _, ms_a = fam["flash_attn"]
        a_tf = fl_a / (ms_a / 1e3) / 1e12
        res["attention"] = {"bound": "mfma", "achieved": round(a_tf, 1), "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
                            "frac": round(a_tf / PEAK_BF16_TFLOPS, 4), "launches": n_a, "ms_per_forward": round(ms_a, 3),
                            "kernel": f"flash_attn_d64_kernel ({n_a} attentions per forward; with the default two-GEMM "
                                      "cross-attention (GEMM family) these are the self-attentions)"}
    if "gemm_e4m3" in fam:
        n_f, fl_f, _, ms_f = fam["gemm_e4m3"]
        f8_tf = fl_f / (ms_f / 1e3) / 1e12
        res["roofline_fp8"] = {"bound": "mfma", "achieved": round(f8_tf, 1), "peak": PEAK_FP8_TFLOPS,
                               "unit": "TFLOP/s", "frac": round(f8_tf / PEAK_FP8_TFLOPS, 4),
                               "traffic": None if tr is None or not fp8 else tr["hbm_bytes_per_forward"],
                               "traffic_note": ("HBM bytes per forward of the e4m3 launches (rocprofv3 PMC pass, "
                                                + tr["file"] + ")") if tr is not None and fp8 else
                               "no PMC pass committed for this workload",
                               "kernel": "gemm8_kernel on e4m3 operands (transformer Linears, e4m3 x e4m3 on "
                                         "v_mfma_scale_f32_16x16x128_f8f6f4; per-row scaled activations, the "
                                         "out-projections on MX block-scaled attention outputs)",
                               "launches": n_f, "algorithmic_flops": fl_f, "kernel_ms_per_forward": round(ms_f, 3)}
    flops = arch.unet_flops(loop.k, loop.k, loop.B, prompt_kv=False, cond_embed=False)
    res["forward_graph_ms"] = round(fam["_all"][3], 3)
    res["kernel_ms_per_forward"] = {k: round(v[3], 3) for k, v in fam.items() if not k.startswith("_")}
    return res, flops


def vae_leg(pipe, loop):
    from fdhip import arch, ops
    dec = pipe.vae.decoder_hip()
    h, w = loop.h, loop.w
    z = torch.empty((h * w, 4), dtype=torch.float16, device=loop.unet.device)
    ops.nchw_to_nhwc(loop.canvas, z, 1, 4, h * w, 1.0 / 0.13025)
    for _ in range(3):
        dec.decode_graphed(z, 1, h, w)
    torch.cuda.synchronize()
    times = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        dec.decode_graphed(z, 1, h, w)
        e1.record()
        torch.cuda.synchronize()
        times.append(e0.elapsed_time(e1))
    vae_ms = sorted(times)[2]
    fam = family_times(lambda: dec.decode(z, 1, h, w), ["gemm", "group_norm"], reps=5)
    res = {"vae_decode_ms": round(vae_ms, 2),
           "vae_decode_tflops": round(arch.vae_decode_flops(h, w) / (vae_ms / 1e3) / 1e12, 1)}
    if "group_norm" in fam:
        n_n, _, nb_n, ms_n = fam["group_norm"]
        gbs = nb_n / (ms_n / 1e3) / 1e9
        res["vae_norm"] = {"bound": "hbm", "achieved": round(gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                           "frac": round(gbs / PEAK_HBM_GBS, 4), "launches": n_n, "ms": round(ms_n, 3),
                           "algorithmic_bytes": nb_n, "kernel": "GroupNorm(+SiLU) of the 1024^2 VAE decode"}
    if "gemm" in fam:
        n_c, fl_c, _, ms_c = fam["gemm"]
        res["vae_conv"] = {"bound": "mfma", "achieved": round(fl_c / (ms_c / 1e3) / 1e12, 1), "peak": PEAK_BF16_TFLOPS,
                           "unit": "TFLOP/s", "frac": round(fl_c / (ms_c / 1e3) / 1e12 / PEAK_BF16_TFLOPS, 4),
                           "launches": n_c, "ms": round(ms_c, 3), "kernel": "fp16 implicit-GEMM convs of the decode"}
    res["vae_kernel_ms"] = {k: round(v[3], 3) for k, v in fam.items() if not k.startswith("_")}
    return res


# ------------------------------------------------------------------------------------------------ main
def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    if args.workload == "c4":
        args.fp8 = True  # configs[3] names fp8 UNet weights on the fp8 MFMA
    rc = maybe_launch(args, argv)
    if rc is not None:
        return rc
    world, rank, local = setup_dist()
    from fdhip import knobs
    from fdhip import lib as L
    knobs.apply_env()  # A/B runs set FD_* knobs in the environment; every non-default value is reported below
    L.require_device()
    dev = torch.device("cuda", local)
    if args.fp8 and args.unet_fp16:
        raise SystemExit("--fp8 and --unet-fp16 are exclusive")
    udt = "fp16" if args.unet_fp16 else "bf16"
    pipe = build_pipe(dev, args.fp8, world, torch.float16 if args.unet_fp16 else torch.bfloat16)
    result = {"n_gpus": world, "steps": args.steps, "warmup": args.warmup, "higher_is_better": True,
              "vs_baseline": None, "dtype": "fp8-e4m3+bf16" if args.fp8 else udt,
              "data": "synthetic (seeded random-init SDXL+FaithDiff weights, synthetic latents/conditions/images)",
              "knobs": knobs.changed()}
    if world > 1:  # rank 0 drew the weights, every other rank received them (FaithDiff_pipeline(process_group=))
        result["weights_broadcast"] = {"bytes": pipe.last_broadcast_bytes, "build_s": round(pipe.build_s, 2),
                                       "broadcast_s": round(pipe.last_broadcast_s, 3),
                                       "backend": dist.get_backend()}

    if args.workload in ("c3", "c4"):
        size, tag = (args.c3_size, "C3") if args.workload == "c3" else (args.c4_size, "C4")
        c3_run(pipe, world, rank, dev, size, 1, warm=False, tag=tag)  # warm-up: graphs captured
        reps = []
        barrier(world)
        for _ in range(max(1, args.steps // 20)):
            reps.append(c3_run(pipe, world, rank, dev, size, args.c3_steps, warm=False, tag=tag))
        r = reps[-1]
        what = (f"C3 tile-steps/sec @{size}px 20-step ({r['ntiles']} TLC tiles, tile-sharded over RCCL)"
                if tag == "C3" else f"C4 tile-steps/sec @{size}px output 20-step, fp8 UNet ({r['ntiles']} TLC "
                "tiles, tile-sharded over RCCL)")
        result.update({"metric": what,
                       "value": r["tile_steps_per_s"], "unit": "tile-steps/s", "scaling": "strong",
                       "ms_per_step": round(r["loop_s"] / r["steps"] * 1e3, 2),
                       "config": {"workload": r["workload"], "s_per_image": r["s_per_image"],
                                  "parallelism": f"tile-sharded x{world}"}, tag.lower(): r})
    elif args.workload == "c5":
        ims = list(range(rank, args.c5_images, world))
        imgs = [synthetic_image(args.size, args.size, 70 + i) for i in ims]
        prompts = [f"A restored photograph, number {i}, sharp and clean." for i in ims]
        run_batch(pipe, imgs, prompts, args.size, 2)  # warm: captures the batched UNet / VAE graphs
        barrier(world)
        t0 = time.perf_counter()
        tm, out, lat = run_batch(pipe, imgs, prompts, args.size, args.c5_steps)
        barrier(world)
        t = max_over_ranks(time.perf_counter() - t0, world, dev)
        stds = check_batch(out, lat, len(imgs))
        st = tm.step_ms()
        result.update({"metric": "C5 images/sec, 1024px 50-step, batch of 8 split over ranks",
                       "value": round(args.c5_images / t, 4), "unit": "images/s", "scaling": "strong",
                       "ms_per_step": round(float(np.median(st)), 2),
                       "config": {"workload": f"C5: {args.c5_images} images of {args.size}^2 x {args.c5_steps} "
                                              "Euler steps; each rank restores its images in ONE pipe(lr_img=[...]) "
                                              "call (their CFG pairs share UNet forwards, each with its own prompt)",
                                  "global_batch": args.c5_images, "images_per_rank": len(ims),
                                  "parallelism": f"replicas x{world}"},
                       "c5": {"s_total": round(t, 3), "loop_s": round(sum(st) / 1e3, 3),
                              "pre_loop_s": round(tm.span_ms("call_start", "loop_start") / 1e3, 3),
                              "decode_s": round(tm.span_ms("decode_start", "decode") / 1e3, 3),
                              "checked": {"latents_finite": True, "min_pixel_std": round(min(stds), 3)}}})
    else:
        loop = C2Loop(pipe, args.size, rank)
        for i in range(args.warmup):
            loop.step(i)
        barrier(world)
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        ev0.record()
        for i in range(args.steps):
            loop.step(i)
        ev1.record()
        barrier(world)
        wall = time.perf_counter() - t0
        t_max = max_over_ranks(wall, world, dev)
        for i in range(args.profile_steps):
            loop.step(i)
        torch.cuda.synchronize()
        ev_ms = ev0.elapsed_time(ev1)
        from fdhip import arch
        # the prompt's attn2 K/V projection and the tile's condition embedding run once per 20-step image
        # (HipUNet.set_context / cond_embed, C2Loop.per_image), as in __call__
        base = arch.unet_flops(loop.k, loop.k, loop.B, prompt_kv=False, cond_embed=False)
        flops = base + (arch.unet_flops(loop.k, loop.k, loop.B) - base) * ((args.steps + 19) // 20) / args.steps
        step_s = ev_ms / 1e3 / args.steps
        result.update({
            "metric": "denoise steps/sec @1024px 20-step + VAE decode ms",
            "value": round(args.steps * world / t_max, 4), "unit": "steps/s",
            "ms_per_step": round(t_max / args.steps * 1e3, 3), "scaling": "weak",
            "config": {"workload": f"C2: {args.size}x{args.size} single TLC tile, CFG batch 2, Euler step + blend, "
                                   f"UNet {'use_fp8: transformer Linears e4m3 MFMA, convs bf16' if args.fp8 else udt}"
                                   " (HipUNet.run: hipGraph replay), VAE fp16",
                       "model": "SDXL UNet + FaithDiff extras (2.58B params)", "global_batch": 2 * world,
                       "latent": [loop.h, loop.w], "parallelism": f"replicas x{world}"},
            "step_roofline": {"bound": "mfma", "achieved": round(flops / step_s / 1e12, 1), "peak": PEAK_BF16_TFLOPS,
                              "unit": "TFLOP/s", "frac": round(flops / step_s / 1e12 / PEAK_BF16_TFLOPS, 4),
                              "algorithmic_flops_per_step": flops, "event_ms_per_step": round(step_s * 1e3, 3)}})
        if not args.no_roofline:
            rl, _ = roofline_leg(loop, args.fp8)
            result.update(rl)
        if not args.no_vae:
            result.update(vae_leg(pipe, loop))
        del loop
        if not args.no_pipeline:
            result["pipeline"] = pipeline_leg(pipe, args.size)
        if not args.no_c3:
            result["c3"] = c3_run(pipe, world, rank, dev, args.c3_size, args.c3_steps)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            result["cpu_baseline"] = cpu_baseline(args.size)
        except Exception as e:  # the baseline must not sink the GPU measurement
            result["cpu_baseline"] = {"value": None, "error": repr(e)}
    if rank == 0:
        order = ["metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
                 "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"]
        line = {k: result[k] for k in order if k in result}
        line.update({k: v for k, v in result.items() if k not in line})
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
