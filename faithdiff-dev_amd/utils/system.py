"""Mirror of utils/system.py: torch_gc and quantize_8bit (fp8 e4m3 weight storage).

quantize_8bit(unet) marks the HIP UNet to store its GEMM/conv weights as OCP float8_e4m3fn (native on
gfx950), unscaled like the reference (utils/system.py:20); the denoise encoder stays fp16 (:24-26).
"""
import gc

import torch


def torch_gc():
    gc.collect()
    if torch.cuda.is_available():
        torch.cuda.empty_cache()


def quantize_8bit(unet):
    if unet is None:
        return
    unet.quantize_8bit()
    torch_gc()
