"""Drop-in for FaithDiff/create_FaithDiff_model.py:11-37.

``FaithDiff_pipeline(sdxl_path, VAE_FP16_path, FaithDiff_path, use_fp8=False)`` builds the same
components the reference does (fp16 VAE, FaithDiff UNet with ``load_additional_layers``, optional fp8
weight storage, DDPM scheduler for the 'lr' start point, Euler scheduler, the pipeline) on the HIP path.
Paths that equal CKPT_PTH.RANDOM_INIT ('random-init') draw seeded random weights; otherwise local
diffusers directories / a local ``FaithDiff.bin`` are loaded with safe loaders (no hub download, no
pickle execution).  Extra keyword arguments (defaults keep the reference call working unchanged):
``seed`` (random-init seed), ``unet_dtype`` (bf16 per the north star; fp16 also supported),
``init_device`` ('cpu' for host-generated weights shared with the CPU oracle, 'cuda' for fast init),
``fp8_mfma`` (with ``use_fp8``: opt in to the e4m3 MFMA for the transformer Linears; default None = the
FD_FP8_MFMA env var, default off = the reference's 16-bit arithmetic on e4m3 weights), ``process_group`` (a
torch.distributed group whose ranks all call this together: rank 0 of the group alone reads the checkpoints (or
draws the random init), the others read nothing and receive every weight by broadcast over RCCL / gloo --
``pipe.last_broadcast_bytes``; the tokenizers' vocabulary files are still read by every rank).
"""
import torch

from utils.system import quantize_8bit

from .models.unet_2d_condition_vae_extension import RANDOM_INIT, RECEIVE, AutoencoderKL, UNet2DConditionModel
from .pipelines.pipeline_FaithDiff_tlc import FaithDiffStableDiffusionXLPipeline
from .schedulers import DDPMScheduler


def FaithDiff_pipeline(sdxl_path, VAE_FP16_path, FaithDiff_path, use_fp8=False, seed=0,
                       unet_dtype=torch.bfloat16, init_device="cpu", fp8_mfma=None, process_group=None):
    dtype = torch.float16
    tok_path = sdxl_path
    if process_group is not None:
        import torch.distributed as dist
        if dist.get_rank(process_group) != 0:  # a receiver: reads no weights, rank 0 broadcasts them below
            sdxl_path = VAE_FP16_path = FaithDiff_path = RECEIVE
    vae = AutoencoderKL.from_pretrained(VAE_FP16_path, seed=seed, init_device=init_device).to(dtype=dtype)
    unet = UNet2DConditionModel.from_pretrained(sdxl_path, subfolder="unet", variant="fp16", seed=seed,
                                                init_device=init_device)
    fd_path = FaithDiff_path
    if fd_path not in (RANDOM_INIT, RECEIVE) and not str(fd_path).endswith((".bin", ".safetensors")):
        fd_path = f"{fd_path}/FaithDiff.bin"
    unet.load_additional_layers(weight_path=fd_path, dtype=dtype, init_device=init_device)
    if use_fp8:
        quantize_8bit(unet, fp8_mfma=fp8_mfma)
    unet.to(dtype=unet_dtype)
    from .models.clip_text import load_tokenizer
    pipe = FaithDiffStableDiffusionXLPipeline.from_pretrained(
        sdxl_path, vae=vae, add_sample=True, denoise_encoder=unet.denoise_encoder, DDPM_scheduler=DDPMScheduler(),
        add_watermarker=False, torch_dtype=dtype, variant="fp16", unet=unet, seed=seed,
        tokenizer=load_tokenizer(tok_path, "tokenizer", pad_token_id=49407),
        tokenizer_2=load_tokenizer(tok_path, "tokenizer_2", pad_token_id=0))
    pipe.unet = unet
    if process_group is not None:
        pipe.broadcast_weights(process_group)
    return pipe


def create_bsrnet(bsrnet_path, seed=0):
    """create_FaithDiff_model.py:39-42: RRDBNet(3, 3, 64, 23, 32, sf=4) with its weights loaded strictly -- from a
    local .pth (torch.load(weights_only=True)) or .safetensors file, or seeded random weights for 'random-init'."""
    from .models.bsrnet_arch import BSRNet
    from .models.unet_2d_condition_vae_extension import _load_file
    from fdhip import arch
    bsrnet = BSRNet(in_nc=3, out_nc=3, nf=64, nb=23, gc=32, sf=4)
    if bsrnet_path == RANDOM_INIT:
        sd = arch.random_init(arch.bsrnet_param_shapes(23), seed=seed + 31, gain=0.25)
    else:
        sd = _load_file(str(bsrnet_path))
    bsrnet.load_state_dict(sd, strict=True)
    return bsrnet
