"""Mirror of utils/system.py: torch_gc and quantize_8bit (fp8 e4m3 weight storage).

quantize_8bit(unet) rounds every UNet weight to unscaled OCP float8_e4m3fn like the reference
(utils/system.py:20) and keeps 16-bit compute on those values (the reference's autocast arithmetic);
fp8_mfma=True opts in to the gfx950 e4m3 MFMA for the transformer Linears.  The denoise encoder stays fp16
(:24-26).
"""
import gc

import torch


def torch_gc():
    gc.collect()
    if torch.cuda.is_available():
        torch.cuda.empty_cache()


def quantize_8bit(unet, fp8_mfma=None):
    if unet is None:
        return
    unet.quantize_8bit(fp8_mfma=fp8_mfma)
    torch_gc()
