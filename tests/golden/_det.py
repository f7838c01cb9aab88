"""Deterministic tensors shared by the golden generator and the tests (CPU torch RNG)."""
import os

import torch


def det_tensor(shape, seed, scale=1.0, offset=0.0, kind="randn"):
    g = torch.Generator().manual_seed(int(seed))
    if kind == "rand":
        t = torch.rand(shape, generator=g, dtype=torch.float32) * 2 - 1
    else:
        t = torch.randn(shape, generator=g, dtype=torch.float32)
    return t * scale + offset


def fill_module(module, seed, scale=None):
    """Overwrite every parameter with a seeded value (weights ~U(-1,1)/sqrt(fan_in), norms ~1)."""
    with torch.no_grad():
        for k, (name, p) in enumerate(sorted(module.named_parameters())):
            if p.ndim == 1 and ("ln" in name or "norm" in name) and name.endswith("weight"):
                p.copy_(det_tensor(p.shape, seed + k, 0.1, 1.0, "rand"))
            elif p.ndim == 1:
                p.copy_(det_tensor(p.shape, seed + k, 0.1, 0.0, "rand"))
            else:
                fan_in = p[0].numel()
                p.copy_(det_tensor(p.shape, seed + k, (scale or 1.0) / fan_in ** 0.5, 0.0, "rand"))
    return module


def synthetic_degraded(H, W, seed=0):
    """Seeded procedural RGB image (smooth field + edges) degraded by blur, x1/4 resize, noise, JPEG
    (dataloader/train_kernel.yml ranges), then LANCZOS back up, as test_wo_llava.py:78-81 does."""
    import io

    import numpy as np
    from PIL import Image, ImageFilter
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:H, 0:W].astype(np.float32)
    img = np.zeros((H, W, 3), np.float32)
    for c in range(3):
        for _ in range(4):
            fx, fy, ph = rng.uniform(0.5, 6, 2).tolist() + [rng.uniform(0, 6.28)]
            img[..., c] += np.sin(xx / W * fx * 6.28 + ph) * np.cos(yy / H * fy * 6.28)
    img += (((xx // 37) + (yy // 29)) % 2)[..., None] * 0.8
    img = (img - img.min()) / (img.max() - img.min())
    pil = Image.fromarray((img * 255).astype(np.uint8)).filter(ImageFilter.GaussianBlur(1.5))
    pil = pil.resize((W // 4, H // 4), Image.BICUBIC)
    arr = np.asarray(pil).astype(np.float32) + rng.normal(0, 5, (H // 4, W // 4, 3))
    pil = Image.fromarray(np.clip(arr, 0, 255).astype(np.uint8))
    buf = io.BytesIO()
    pil.save(buf, "JPEG", quality=75)
    pil = Image.open(io.BytesIO(buf.getvalue())).convert("RGB")
    return pil.resize((W, H), Image.LANCZOS)


def c2_inputs():
    """The seeded inputs of the C2 headline-parity case (BASELINE configs[1]: 1024^2, one TLC tile, 20 Euler
    steps, CFG 5, start_point 'lr'), shared by tests/golden/make_c2_golden.py and tests/test_pipeline_gpu.py:
    image, prompt embeddings (pos, neg, pooled pos, pooled neg), initial noise, VAE posterior draw."""
    H = W = 1024
    img = synthetic_degraded(H, W, 2)
    pe = det_tensor((1, 77, 2048), 9101)
    npe = det_tensor((1, 77, 2048), 9102)
    ppe = det_tensor((1, 1280), 9103)
    nppe = det_tensor((1, 1280), 9104)
    noise = det_tensor((1, 4, H // 8, W // 8), 9105)
    post = det_tensor((1, 4, H // 8, W // 8), 9106)
    return dict(H=H, W=W, img=img, pe=pe, npe=npe, ppe=ppe, nppe=nppe, noise=noise, post=post, steps=20,
                guidance=5.0, overlap=0.5, target=(1024, 1024), seed=0)


BAND_PNG = os.path.join(os.path.dirname(os.path.abspath(__file__)), "band", "band.png")


def band_inputs(upscale=1, steps=4):
    """The reference's one in-tree input (examples/band.png, 1079x778 RGBA) prepared exactly as
    test_wo_llava.py:65,78-82 does: convert('RGB'), resize by ``upscale`` with LANCZOS, check_image_size
    (bottom/right edge replication to a multiple of 8).  x1: 1080x784 -> a 135x98 latent, two ragged 128x98 TLC
    tiles (target 1024: 128-latent tiles clamped to the 98-row height), both on the UNet's forward_upsample_size
    path (98 = 2 * 49).  x4: 4316x3112 -> 4320x3112, a 540x389 latent.  The caption (LLaVA, OUT of scope) is
    replaced by seeded prompt embeddings; noise and the VAE posterior draw are explicit seeded tensors."""
    from PIL import Image
    from utils.image_process import check_image_size
    image = Image.open(BAND_PNG).convert("RGB")
    w, h = image.size
    image = image.resize((w * upscale, h * upscale), Image.LANCZOS)
    padded, w0, h0, W, H = check_image_size(image)
    pe = det_tensor((1, 77, 2048), 9201)
    npe = det_tensor((1, 77, 2048), 9202)
    ppe = det_tensor((1, 1280), 9203)
    nppe = det_tensor((1, 1280), 9204)
    noise = det_tensor((1, 4, H // 8, W // 8), 9205)
    post = det_tensor((1, 4, H // 8, W // 8), 9206)
    return dict(H=H, W=W, w0=w0, h0=h0, image=image, img=padded, pe=pe, npe=npe, ppe=ppe, nppe=nppe, noise=noise,
                post=post, steps=steps, guidance=5.0, overlap=0.5, target=(1024, 1024), seed=0)


# ----------------------------------------------------------------------------------------------------------------
# Cheap deterministic stand-ins for the diffusers-owned models, used to pin the reference's own __call__
# orchestration (pipeline_FaithDiff_tlc.py:1187-1459) against oracle/pipeline.py:run_pipeline
# (tests/golden/make_call_golden.py, tests/test_oracle_golden.py).  They are functions of every input the loop
# hands them -- CFG row order, tile position (time ids), timestep, image latents -- so a wrong orchestration
# changes the result; their own numerics are not what is pinned.
_TID_MIX = torch.tensor([[0.9, -0.4, 0.3, 0.2], [-0.5, 0.8, -0.1, 0.4], [0.7, 0.1, -0.6, 0.3],
                         [-0.2, 0.5, 0.4, -0.7], [0.3, -0.3, 0.2, 0.6], [0.1, 0.6, -0.5, -0.2]])


def standin_eps(x, t, ctx, text, tids, emb):
    """x (B,4,h,w), t scalar, ctx (B,L,D), text (B,P), tids (B,6), emb (B,Ce,h,w) -> eps (B,4,h,w) fp32."""
    B = x.shape[0]
    s = torch.tanh(ctx.float().mean(dim=1)[:, :4]).view(B, 4, 1, 1)
    p = torch.tanh(text.float()[:, :4]).view(B, 4, 1, 1)
    q = torch.tanh((tids.float() / 64.0) @ _TID_MIX).view(B, 4, 1, 1)
    tt = float(t) / 1000.0
    return torch.tanh(0.7 * x.float() + 0.3 * emb.float()[:, :4] + 0.5 * s + 0.2 * p + 0.1 * q + 0.05 * tt)


def standin_moments(x):
    """VAE encoder stand-in: (1,3,H,W) -> moments (1,8,H/8,W/8) (mean 4 | logvar 4)."""
    m = torch.nn.functional.avg_pool2d(x.float(), 8)
    mean = torch.cat([m, m[:, :1] * 0.5], 1)
    logvar = torch.cat([m * 2.0 - 3.0, m[:, 1:2] - 4.0], 1)
    return torch.cat([mean, logvar], 1)


def standin_features(x):
    """Denoise-encoder stand-in: (1,3,H,W) -> (1,8,H/8,W/8)."""
    m = torch.nn.functional.avg_pool2d(x.float(), 8)
    return torch.cat([m, torch.tanh(m * 3.0), m[:, :2] ** 2], 1)


def standin_decode(z):
    """VAE decoder stand-in: (1,4,h,w) -> (1,3,8h,8w)."""
    y = torch.nn.functional.interpolate(torch.tanh(z.float()[:, :3] * 0.5), scale_factor=8, mode="nearest")
    return y + 0.1 * z.float()[:, 3:4].repeat_interleave(8, 2).repeat_interleave(8, 3)


def call_cases():
    """(name, H, W, target, steps, guidance, rescale, start_point) of the orchestration pins."""
    return [("multi", 320, 192, (128, 128), 3, 5.0, 0.0, "lr"),     # 40x24 latent, 16x16 tiles: 4 x 2 grid
            ("ragged", 200, 136, (128, 128), 2, 5.0, 0.7, "lr"),    # 25x17 latent, snapped edge tiles, rescale
            ("clamped", 128, 128, (256, 256), 2, 3.0, 0.0, "noise")]  # 16x16 latent < 32 tile (quirk A.4)


def call_inputs(H, W, seed):
    img = det_tensor((1, 3, H, W), seed, 0.6).clamp(-1, 1)
    pe, npe = det_tensor((1, 77, 64), seed + 1), det_tensor((1, 77, 64), seed + 2)
    ppe, nppe = det_tensor((1, 32), seed + 3), det_tensor((1, 32), seed + 4)
    noise, post = det_tensor((1, 4, H // 8, W // 8), seed + 5), det_tensor((1, 4, H // 8, W // 8), seed + 6)
    return img, pe, npe, ppe, nppe, noise, post


# ----------------------------------------------------------------------------------------------------------------
# UNet forward / Encoder.encode / load_state_dict pins (tests/golden/make_unet_golden.py runs the reference's own
# UNet2DConditionModel.forward ext:480-697, Encoder.encode ext:122-148 and load_state_dict ext:444-478 unbound on the
# oracle's blocks; tests/test_unet_golden_cpu.py checks the oracle and the product's host logic against them).
UNET_WEIGHT_SEED = 1  # arch.random_init(arch.unet_param_shapes(), seed=1): the GPU UNet parity tests' weights


def unet_inputs(h, w, ntiles=1, seed=0):
    """(B, x, cond, ctx, text, tids) for a CFG-paired tile batch, as tests/test_unet_gpu.py feeds the UNet."""
    g = torch.Generator().manual_seed(seed)
    B = 2 * ntiles
    x = torch.randn(ntiles, 4, h, w, generator=g).repeat_interleave(2, 0)
    cond = torch.randn(ntiles, 512, h, w, generator=g).repeat_interleave(2, 0)
    ctx = torch.randn(2, 77, 2048, generator=g)
    text = torch.randn(2, 1280, generator=g).repeat(ntiles, 1)
    tids = torch.tensor([[1024.0, 1024.0, 64.0 * i, 0.0, 1024.0, 1024.0] for i in range(ntiles)]).repeat_interleave(2, 0)
    return B, x, cond, ctx, text, tids


def unet_golden_cases():
    """(name, h, w, ntiles, t, add_sample, with_embedding).  62x46 is not a multiple of 4, so the reference's
    forward_upsample_size path (ext:522-529, 665-666) fires: 62 -> 31 -> 16 on the way down, 16 -> 31 -> 62 up."""
    return [("s32", 32, 32, 1, 951.0, True, True),
            ("r40x24", 40, 24, 2, 501.0, True, True),
            ("odd62x46", 62, 46, 1, 951.0, True, True),
            ("noadd32", 32, 32, 1, 301.0, False, True),
            ("noemb24", 24, 24, 1, 51.0, True, False)]


def lsd_cases(extras, core_key, core_shape):
    """load_state_dict routing cases (ext:444-478): (name, state_dict, strict).  ``extras`` is a full extras +
    denoise_encoder state dict; ``core_key`` one real core key of shape ``core_shape``."""
    first = sorted(k for k in extras if k.startswith("spatial_ch_projs."))[-1]
    minus = {k: v for k, v in extras.items() if k != first}
    cne = "condition_embedding.conv_in.weight"
    bad_shape = dict(extras)
    bad_shape[cne] = torch.zeros(extras[cne].shape[0], 7, 3, 3)
    extra_key = dict(extras)
    extra_key["information_transformer_layes.5.ln_1.weight"] = torch.ones(640)
    agg = dict(extras)
    agg["agg_net.0.weight"] = torch.ones(4)
    core = {core_key: det_tensor(core_shape, 77), "foo.unknown.weight": torch.ones(3)}
    return [("full_strict", dict(extras), True),
            ("missing_strict", minus, True),
            ("missing_loose", minus, False),
            ("agg_strict", agg, True),
            ("agg_loose", agg, False),
            ("unknown_core_strict", {**extras, **core}, True),
            ("core_only_strict", core, True),
            ("bad_shape_loose", bad_shape, False),
            ("extra_key_strict", extra_key, True),
            ("extra_key_loose", extra_key, False)]
