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
