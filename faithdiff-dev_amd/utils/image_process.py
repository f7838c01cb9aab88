"""Host pre-processing (mirror of utils/image_process.py:7-21).

check_image_size pads bottom/right to a multiple of 8 by edge replication; the reference calls
cv2.copyMakeBorder(BORDER_REPLICATE), which is np.pad(mode='edge') (cv2 is not needed here).
"""
import numpy as np
import torch
from PIL import Image


def check_image_size(x, padder_size=8):
    width, height = x.size
    mod_pad_h = (padder_size - height % padder_size) % padder_size
    mod_pad_w = (padder_size - width % padder_size) % padder_size
    x_np = np.array(x)
    pad = ((0, mod_pad_h), (0, mod_pad_w)) + ((0, 0),) * (x_np.ndim - 2)
    x = Image.fromarray(np.pad(x_np, pad, mode="edge"))
    return x, width, height, width + mod_pad_w, height + mod_pad_h


def image2tensor(img):
    """utils/image_process.py:23-26 (the BSRNet input, test.py:98): HWC uint8 (or HW) -> NCHW fp32 in [0, 1]."""
    a = np.asarray(img)
    if a.ndim == 2:
        a = a[:, :, None]
    return torch.from_numpy(np.ascontiguousarray(a)).permute(2, 0, 1).float().div(255.0).unsqueeze(0)


def tensor2image(img):
    """utils/image_process.py:29-33: NCHW / CHW tensor in [0, 1] -> HWC uint8 (round half to even, as numpy)."""
    a = img.detach().squeeze().float().clamp(0, 1).cpu().numpy()
    if a.ndim == 3:
        a = np.transpose(a, (1, 2, 0))
    return np.uint8((a * 255.0).round())
