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
