"""Checkpoint locations (mirror of CKPT_PTH.py).  The reference names HF repos; offline they resolve to a
local diffusers directory when one exists, else to the seeded random-init sentinel below."""
import os

RANDOM_INIT = "random-init"
SDXL_PATH = os.environ.get("FAITHDIFF_SDXL_PATH", RANDOM_INIT)
FAITHDIFF_PATH = os.environ.get("FAITHDIFF_PATH", RANDOM_INIT)
VAE_FP16_PATH = os.environ.get("FAITHDIFF_VAE_FP16_PATH", RANDOM_INIT)
LLAVA_CLIP_PATH = "openai/clip-vit-large-patch14-336"
LLAVA_MODEL_PATH = "liuhaotian/llava-v1.5-13b"
BSRNet_PATH = "./checkpoints/BSRNet.pth"
