"""Deterministic tensors shared by the golden generator and the tests (CPU torch RNG)."""
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
