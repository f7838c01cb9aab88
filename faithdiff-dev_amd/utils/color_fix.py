"""Colour correction after restoration (mirror of utils/color_fix.py:14-119; host CPU, as in the reference).

adain: per-channel mean / unbiased std (+1e-5 on the variance) renormalisation of the target towards
the source; wavelet: 5-level dilated 3x3 binomial blur decomposition, target high frequencies + source
low frequencies.  ToTensor / ToPILImage are restated with numpy (torchvision is not required):
ToTensor = uint8 HWC / 255 -> CHW float; ToPILImage on a float tensor = (x * 255).byte() (truncation).
"""
import numpy as np
import torch
import torch.nn.functional as F
from PIL import Image
from torch import Tensor


def _to_tensor(img):
    a = np.asarray(img.convert("RGB"), dtype=np.float32) / 255.0
    return torch.from_numpy(a.transpose(2, 0, 1).copy()).unsqueeze(0)


def _to_pil(t):
    a = t.squeeze(0).clamp(0.0, 1.0).mul(255).byte().permute(1, 2, 0).numpy()  # ToPILImage float path
    return Image.fromarray(a)


def calc_mean_std(feat: Tensor, eps=1e-5):
    size = feat.size()
    assert len(size) == 4, "The input feature should be 4D tensor."
    b, c = size[:2]
    feat_var = feat.reshape(b, c, -1).var(dim=2) + eps
    feat_std = feat_var.sqrt().reshape(b, c, 1, 1)
    feat_mean = feat.reshape(b, c, -1).mean(dim=2).reshape(b, c, 1, 1)
    return feat_mean, feat_std


def adaptive_instance_normalization(content_feat: Tensor, style_feat: Tensor):
    size = content_feat.size()
    style_mean, style_std = calc_mean_std(style_feat)
    content_mean, content_std = calc_mean_std(content_feat)
    normalized = (content_feat - content_mean.expand(size)) / content_std.expand(size)
    return normalized * style_std.expand(size) + style_mean.expand(size)


def wavelet_blur(image: Tensor, radius: int):
    k = torch.tensor([[0.0625, 0.125, 0.0625], [0.125, 0.25, 0.125], [0.0625, 0.125, 0.0625]], dtype=image.dtype)
    k = k[None, None].repeat(3, 1, 1, 1)
    image = F.pad(image, (radius, radius, radius, radius), mode="replicate")
    return F.conv2d(image, k, groups=3, dilation=radius)


def wavelet_decomposition(image: Tensor, levels=5):
    high = torch.zeros_like(image)
    for i in range(levels):
        low = wavelet_blur(image, 2 ** i)
        high += image - low
        image = low
    return high, low


def wavelet_reconstruction(content_feat: Tensor, style_feat: Tensor):
    content_high, _ = wavelet_decomposition(content_feat)
    _, style_low = wavelet_decomposition(style_feat)
    return content_high + style_low


def adain_color_fix(target: Image, source: Image):
    return _to_pil(adaptive_instance_normalization(_to_tensor(target), _to_tensor(source)))


def wavelet_color_fix(target: Image, source: Image):
    return _to_pil(wavelet_reconstruction(_to_tensor(target), _to_tensor(source)))
