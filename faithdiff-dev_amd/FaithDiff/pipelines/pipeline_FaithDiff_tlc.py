"""Drop-in for FaithDiff/pipelines/pipeline_FaithDiff_tlc.py on MI355X.

``FaithDiffStableDiffusionXLPipeline.__call__`` keeps the reference signature (:1008-1042) and output
(``.images``), and the same algorithm (:1187-1459): encode prompt (CFG always on, "" encoded, :1231-1243)
-> preprocess (:1246) -> Euler timesteps (:1249) -> denoise encoder (:1250-1255) -> TLC grids of the
image latents (:1257) -> noise * init sigma (:1261-1270) -> start_point 'lr': VAE posterior sample *
0.13025, DDPM add_noise at t = 999 (:1271-1276) -> per step, per tile: CFG pair, scale_model_input,
add_time_ids = [orig_h, orig_w, tile_i, tile_j, tgt_h, tgt_w] (latent-grid offsets), UNet, CFG (+
rescale), Euler step, then the gaussian fp32 blend (:1324-1409) -> latents / 0.13025 -> fp16 VAE decode
(:1411-1442) -> postprocess (:1451).

What differs (MI355X-first, documented in DESIGN.md): the latent state stays fp32 between steps (the
reference rounds it to fp16 at :1409); several tiles share one UNet forward (rows are independent
except the extras' batch-axis MHA, which is grouped per tile); the per-element loop work is fused
device kernels (fd_tlc_*); tiles can be sharded over ranks (tile_parallel.py); the CLIP text encoders
run on the HIP kernels (fdhip/clip.py) when built by from_pretrained, with a seeded synthetic stand-in
only for pipelines constructed without them.
"""
import inspect
import time
import zlib
from types import SimpleNamespace
from typing import Any, Callable, Dict, List, Optional, Tuple, Union

import numpy as np
import PIL.Image
import torch
import torch.distributed as dist

from fdhip import knobs, ops

from ..schedulers import DDPMScheduler, EulerDiscreteScheduler
from .pipeline_output import FaithDiffStableDiffusionXLPipelineOutput
from .tile_parallel import TileShard, broadcast, broadcast_state_dict, run_tile_loop, staging_device
from .tlc import TileGrid, max_tile_batch, tile_batches


class SyntheticTextEncoder:
    """Seeded stand-in for CLIP-L + OpenCLIP-bigG: prompt -> (1, 77, 2048) hidden states
    (``hidden_states[-2]`` concat) and (1, 1280) pooled embedding, deterministic in the prompt text.
    The empty negative prompt is *encoded* like any other prompt, as in the reference (:622-675)."""

    def __call__(self, prompt: str):
        g = torch.Generator().manual_seed(zlib.crc32(prompt.encode("utf-8")) & 0x7FFFFFFF)
        return torch.randn(1, 77, 2048, generator=g), torch.randn(1, 1280, generator=g)


def randn_tensor(shape, generator=None, device=None, dtype=torch.float32):
    """diffusers.utils.torch_utils.randn_tensor semantics: draw on the generator's device."""
    if isinstance(generator, list):
        generator = generator[0]
    gdev = generator.device if generator is not None else torch.device(device)
    return torch.randn(shape, generator=generator, device=gdev, dtype=dtype).to(device)


def retrieve_timesteps(scheduler, num_inference_steps=None, device=None, timesteps=None, **kwargs):
    """:331-372."""
    if timesteps is not None:
        if "timesteps" not in set(inspect.signature(scheduler.set_timesteps).parameters.keys()):
            raise ValueError(f"The current scheduler class {scheduler.__class__}'s `set_timesteps` does not support "
                             "custom timestep schedules.")
        scheduler.set_timesteps(timesteps=timesteps, device=device, **kwargs)
        return scheduler.timesteps, len(scheduler.timesteps)
    scheduler.set_timesteps(num_inference_steps, device=device, **kwargs)
    return scheduler.timesteps, num_inference_steps


class FaithDiffStableDiffusionXLPipeline:
    model_cpu_offload_seq = "text_encoder->text_encoder_2->denoise_encoder->unet->vae"
    _optional_components = ["tokenizer", "tokenizer_2", "text_encoder", "text_encoder_2", "feature_extractor"]
    _callback_tensor_inputs = ["latents", "prompt_embeds", "negative_prompt_embeds", "add_text_embeds",
                               "add_time_ids", "negative_pooled_prompt_embeds", "negative_add_time_ids"]

    def __init__(self, vae, denoise_encoder, text_encoder=None, text_encoder_2=None, tokenizer=None,
                 tokenizer_2=None, unet=None, scheduler=None, DDPM_scheduler=None, force_zeros_for_empty_prompt=True,
                 add_watermarker=None):
        self.vae = vae
        self.denoise_encoder = denoise_encoder
        self.text_encoder = text_encoder or SyntheticTextEncoder()
        self.text_encoder_2 = text_encoder_2
        self.tokenizer, self.tokenizer_2 = tokenizer, tokenizer_2
        self.unet = unet
        self.scheduler = scheduler or EulerDiscreteScheduler()
        self.DDPM_scheduler = DDPM_scheduler or DDPMScheduler()
        self.config = SimpleNamespace(force_zeros_for_empty_prompt=force_zeros_for_empty_prompt)
        self.vae_scale_factor = 2 ** (len(self.vae.config.block_out_channels) - 1)
        self.default_sample_size = 128
        self.watermark = None
        self.device = torch.device("cpu")
        # TLC tiles per UNet forward (B = 2 * tile_batch rows; C3 4096^2: 4 -> 13 tiles = 51.6 -> 53.2 tile-steps/s,
        # scripts/tb_sweep.sh; C4 225 tiles: 13 -> 25 = 70.1 -> 72.2 tile-steps/s, profiles/r05ad_tile_batch_ab.txt).
        # 25 keeps the largest activation (the 128^2 level's 2 * 25 * 16384 rows x 1280) at 1.05e9 elements, half of
        # the 32-bit index range the kernels' offsets assume.  FD_TILE_BATCH overrides (A/B timing)
        self.tile_batch = knobs.get("FD_TILE_BATCH")
        # FD_TILE_BALANCE=1: a rank's tiles in ceil(count / tile_batch) batches of equal size (+-1) instead of full
        # batches and a short remainder (C4 225 tiles: 17 x 13 + 4 -> 9 x 13 + 9 x 12)
        self.tile_balance = knobs.get("FD_TILE_BALANCE")
        self.process_group = None    # torch.distributed group for tile parallelism (None: single GPU)
        self.last_timings = {}
        self._weights_group = None   # the group broadcast_weights last synchronised the weights over
        self.last_broadcast_bytes = 0
        self.last_broadcast_s = 0.0

    # ------------------------------------------------------------------ construction
    @classmethod
    def from_pretrained(cls, sdxl_path, vae=None, denoise_encoder=None, DDPM_scheduler=None, add_sample=True,
                        add_watermarker=False, torch_dtype=None, variant=None, unet=None, seed=0, **kwargs):
        """Like diffusers' from_pretrained of the SDXL directory: the two CLIP text encoders and tokenizers come
        from ``sdxl_path`` (text_encoder/, text_encoder_2/, tokenizer/, tokenizer_2/; 'random-init' = seeded
        weights of the real architecture + the framing-only fallback tokenizer), unless passed in."""
        from ..models.clip_text import CLIPTextModel, CLIPTextModelWithProjection, load_tokenizer
        te = kwargs.get("text_encoder") or CLIPTextModel.from_pretrained(sdxl_path, "text_encoder", seed=seed + 11)
        te2 = kwargs.get("text_encoder_2") or CLIPTextModelWithProjection.from_pretrained(sdxl_path, "text_encoder_2",
                                                                                           seed=seed + 13)
        tok = kwargs.get("tokenizer") or load_tokenizer(sdxl_path, "tokenizer", pad_token_id=49407)
        tok2 = kwargs.get("tokenizer_2") or load_tokenizer(sdxl_path, "tokenizer_2", pad_token_id=0)
        return cls(vae=vae, denoise_encoder=denoise_encoder, unet=unet, scheduler=EulerDiscreteScheduler(),
                   DDPM_scheduler=DDPM_scheduler or DDPMScheduler(), add_watermarker=add_watermarker,
                   text_encoder=te, text_encoder_2=te2, tokenizer=tok, tokenizer_2=tok2)

    def to(self, device=None, dtype=None):
        dev = torch.device(device) if device is not None else self.device
        if dev.type == "cuda" and dev.index is not None:
            torch.cuda.set_device(dev)
        self.device = dev
        for m in (self.vae, self.denoise_encoder, self.unet, self.text_encoder_2,
                  None if isinstance(self.text_encoder, SyntheticTextEncoder) else self.text_encoder):
            if m is not None:
                m.to(device=dev)
        return self

    @property
    def _execution_device(self):
        return self.device

    def enable_model_cpu_offload(self, *a, **k):
        """No-op: 288 GB of HBM3E hold the UNet, VAE and encoders (reference README:59-60 needs offload on
        <12 GB parts)."""

    def set_encoder_tile_settings(self, denoise_encoder_tile_sample_min_size=1024,
                                  denoise_encoder_sample_overlap_factor=0.25, vae_sample_size=1024,
                                  vae_tile_overlap_factor=0.25):
        """:888-896 (note: does not recompute denoise_encoder.tile_latent_min_size, as in the reference)."""
        self.denoise_encoder.tile_sample_min_size = denoise_encoder_tile_sample_min_size
        self.denoise_encoder.tile_overlap_factor = denoise_encoder_sample_overlap_factor
        self.vae.config.sample_size = vae_sample_size
        self.vae.tile_overlap_factor = vae_tile_overlap_factor

    def enable_vae_tiling(self):
        self.vae.enable_tiling()
        self.denoise_encoder.enable_tiling()

    def disable_vae_tiling(self):
        self.vae.disable_tiling()
        self.denoise_encoder.disable_tiling()

    def enable_tile_parallel(self, group=None, sync_weights=True):
        """Shard TLC tiles over the ranks of `group` (default WORLD) with one all-gather per step; the tiled VAE
        encode / decode and the tiled denoise encoder shard their tiles the same way (fdhip.tiling.map_tiles).
        The tiles of one image must all see the same model: with ``sync_weights`` (default) every rank's weights
        first become rank 0's (broadcast_weights) unless the pipeline was built or synced over this group already.
        ``sync_weights=False`` skips that transfer for callers that loaded the same checkpoint on every rank (the
        reference flow: each process reads the same files) -- their weights are already equal."""
        self.process_group = group if group is not None else dist.group.WORLD
        if sync_weights and self._weights_group is not self.process_group:
            self.broadcast_weights(self.process_group)
        for m in (self.vae, self.denoise_encoder):
            if m is not None:
                m.process_group = self.process_group

    def _weight_owners(self):
        te = None if isinstance(self.text_encoder, SyntheticTextEncoder) else self.text_encoder
        return [("unet", self.unet), ("vae", self.vae), ("denoise_encoder", self.denoise_encoder),
                ("text_encoder", te), ("text_encoder_2", self.text_encoder_2)]

    def broadcast_weights(self, group=None, src=0):
        """Every component's weights (UNet + FaithDiff extras, VAE, denoise encoder, both text encoders) become
        rank `src`'s over `group` -- one manifest + bucketed broadcasts per component over RCCL (gloo on CPU),
        before anything is packed for the kernels (packed modules built earlier are dropped and rebuilt from the
        received weights on next use).  Returns the bytes broadcast (also in ``last_broadcast_bytes``)."""
        group = group if group is not None else dist.group.WORLD
        if dist.get_world_size(group) == 1:  # nothing to synchronise
            self._weights_group, self.last_broadcast_bytes = group, 0
            return 0
        dev = staging_device(group)
        # every rank must still hold every component's host weights; agree on it collectively first, so that a
        # rank that released them (release_host_weights) makes ALL ranks raise instead of leaving the others
        # blocked in a broadcast it never joins
        owners = [(name, m, getattr(m, "_sd", None)) for name, m in self._weight_owners()]
        released = [name for name, _, sd in owners if sd is not None and not sd]
        flag = torch.tensor([len(released)], dtype=torch.int64, device=dev)
        dist.all_reduce(flag, group=group)
        if int(flag.item()):
            raise RuntimeError("broadcast_weights: host weights were released (release_host_weights) before they "
                               f"were synchronised over the group (this rank: {released or 'none'})")
        total = 0
        t0 = time.perf_counter()
        for name, m, sd in owners:
            if sd is None:
                continue
            total += broadcast_state_dict(sd, group, src, device=dev)
            for attr in ("_hip", "_enc", "_dec"):
                if getattr(m, attr, None) is not None:
                    setattr(m, attr, None)
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        self._weights_group = group
        self.last_broadcast_bytes, self.last_broadcast_s = total, time.perf_counter() - t0
        return total

    # ------------------------------------------------------------------ properties (:915-948)
    @property
    def guidance_scale(self):
        return self._guidance_scale

    @property
    def guidance_rescale(self):
        return self._guidance_rescale

    @property
    def clip_skip(self):
        return self._clip_skip

    @property
    def do_classifier_free_guidance(self):
        return self._guidance_scale > 1 and self.unet.config.time_cond_proj_dim is None

    @property
    def cross_attention_kwargs(self):
        return self._cross_attention_kwargs

    @property
    def denoising_end(self):
        return self._denoising_end

    @property
    def num_timesteps(self):
        return self._num_timesteps

    @property
    def interrupt(self):
        return self._interrupt

    # ------------------------------------------------------------------ inputs
    def encode_prompt(self, prompt, prompt_2=None, device=None, num_images_per_prompt=1,
                      do_classifier_free_guidance=True, negative_prompt=None, negative_prompt_2=None,
                      prompt_embeds=None, negative_prompt_embeds=None, pooled_prompt_embeds=None,
                      negative_pooled_prompt_embeds=None, lora_scale=None, clip_skip=None):
        """:485-717.  With the two CLIP encoders (HIP, FaithDiff/models/clip_text.py): tokenize each prompt with
        its tokenizer (max_length 77, truncation), keep hidden_states[-2] (or -(clip_skip + 2)) of both and concat
        (:587-615), the pooled output is text_encoder_2's projected EOS row (:608); the negative prompt ("" when
        None and force_zeros is off) is *encoded* the same way (:622-675).  Without them (pipelines built around
        pre-computed embeddings) the seeded synthetic stand-in is used."""
        if self.text_encoder_2 is None:
            if prompt_embeds is None:
                if isinstance(prompt, list):
                    prompt = prompt[0]
                prompt_embeds, pooled_prompt_embeds = self.text_encoder(prompt)
            zero_out = negative_prompt is None and self.config.force_zeros_for_empty_prompt
            if do_classifier_free_guidance and negative_prompt_embeds is None and zero_out:
                negative_prompt_embeds = torch.zeros_like(prompt_embeds)
                negative_pooled_prompt_embeds = torch.zeros_like(pooled_prompt_embeds)
            elif do_classifier_free_guidance and negative_prompt_embeds is None:
                neg = negative_prompt or ""
                if isinstance(neg, list):
                    neg = neg[0]
                negative_prompt_embeds, negative_pooled_prompt_embeds = self.text_encoder(neg)
            return prompt_embeds, negative_prompt_embeds, pooled_prompt_embeds, negative_pooled_prompt_embeds

        tokenizers = [self.tokenizer, self.tokenizer_2] if self.tokenizer is not None else [self.tokenizer_2]
        encoders = [self.text_encoder, self.text_encoder_2] if self.tokenizer is not None else [self.text_encoder_2]
        prompt = [prompt] if isinstance(prompt, str) else prompt
        batch_size = len(prompt) if prompt is not None else prompt_embeds.shape[0]

        def run(texts_per_encoder, skips):
            """One forward per encoder over every text group given (each group: len(texts) rows); group g keeps
            hidden_states[-2] (skip None) or [-(skip + 2)] and the final encoder's pooled row (:587-615).  The
            prompt and the negative prompt go through as one batch (the reference encodes them in two passes,
            :587-615 / :651-675): half the weight streaming and launches, and -- run as row groups of equal size
            -- bitwise the rows each pass gives alone."""
            sizes = [len(t) for t in texts_per_encoder[0]]
            embs, pooled = [[] for _ in sizes], None
            for groups, tok, enc in zip(texts_per_encoder, tokenizers, encoders):
                ids = torch.cat([tok(texts, padding="max_length", max_length=tok.model_max_length, truncation=True,
                                     return_tensors="pt").input_ids for texts in groups], 0)
                rg = sum(sizes)  # every prompt its own group of 77 rows: bitwise its solo pass
                out = enc(ids, output_hidden_states=True, row_groups=rg) if hasattr(enc, "hip") else \
                    enc(ids, output_hidden_states=True)
                pooled = out[0]  # only the final encoder's pooled output is kept (:607-608)
                r0 = 0
                for g, (n, skip) in enumerate(zip(sizes, skips)):
                    h = out.hidden_states[-2] if skip is None else out.hidden_states[-(skip + 2)]
                    embs[g].append(h[r0:r0 + n])
                    r0 += n
            res, r0 = [], 0
            for g, n in enumerate(sizes):
                res.append((torch.cat(embs[g], dim=-1), pooled[r0:r0 + n]))
                r0 += n
            return res

        zero_out = negative_prompt is None and self.config.force_zeros_for_empty_prompt
        encode_neg = do_classifier_free_guidance and negative_prompt_embeds is None and not zero_out
        if encode_neg:
            negative_prompt = negative_prompt or ""
            negative_prompt_2 = negative_prompt_2 or negative_prompt
            negative_prompt = batch_size * [negative_prompt] if isinstance(negative_prompt, str) else negative_prompt
            negative_prompt_2 = (batch_size * [negative_prompt_2] if isinstance(negative_prompt_2, str)
                                 else negative_prompt_2)
            if prompt is not None and type(prompt) is not type(negative_prompt):
                raise TypeError(f"`negative_prompt` should be the same type to `prompt`, but got "
                                f"{type(negative_prompt)} != {type(prompt)}.")
            if batch_size != len(negative_prompt):
                raise ValueError(f"`negative_prompt`: {negative_prompt} has batch size {len(negative_prompt)}, but "
                                 f"`prompt`: {prompt} has batch size {batch_size}. Please make sure that passed "
                                 "`negative_prompt` matches the batch size of `prompt`.")
        if prompt_embeds is None:
            prompt_2 = prompt_2 or prompt
            prompt_2 = [prompt_2] if isinstance(prompt_2, str) else prompt_2
            if encode_neg:
                (prompt_embeds, pooled_prompt_embeds), (negative_prompt_embeds, negative_pooled_prompt_embeds) = run(
                    [[prompt, negative_prompt], [prompt_2, negative_prompt_2]], [clip_skip, None])
                return prompt_embeds, negative_prompt_embeds, pooled_prompt_embeds, negative_pooled_prompt_embeds
            (prompt_embeds, pooled_prompt_embeds), = run([[prompt], [prompt_2]], [clip_skip])
        if do_classifier_free_guidance and negative_prompt_embeds is None and zero_out:
            negative_prompt_embeds = torch.zeros_like(prompt_embeds)
            negative_pooled_prompt_embeds = torch.zeros_like(pooled_prompt_embeds)
        elif encode_neg:
            (negative_prompt_embeds, negative_pooled_prompt_embeds), = run(
                [[negative_prompt], [negative_prompt_2]], [None])
        return prompt_embeds, negative_prompt_embeds, pooled_prompt_embeds, negative_pooled_prompt_embeds

    def check_inputs(self, lr_img, prompt, prompt_2, height, width, callback_steps, negative_prompt=None,
                     negative_prompt_2=None, prompt_embeds=None, negative_prompt_embeds=None,
                     pooled_prompt_embeds=None, negative_pooled_prompt_embeds=None,
                     callback_on_step_end_tensor_inputs=None):
        """:738-817 (same ValueErrors)."""
        if lr_img is None:
            raise ValueError("`lr_image` must be provided!")
        if height % 8 != 0 or width % 8 != 0:
            raise ValueError(f"`height` and `width` have to be divisible by 8 but are {height} and {width}.")
        if callback_steps is not None and (not isinstance(callback_steps, int) or callback_steps <= 0):
            raise ValueError(f"`callback_steps` has to be a positive integer but is {callback_steps} of type "
                             f"{type(callback_steps)}.")
        if callback_on_step_end_tensor_inputs is not None and not all(
                k in self._callback_tensor_inputs for k in callback_on_step_end_tensor_inputs):
            raise ValueError(f"`callback_on_step_end_tensor_inputs` has to be in {self._callback_tensor_inputs}")
        if prompt is not None and prompt_embeds is not None:
            raise ValueError("Cannot forward both `prompt` and `prompt_embeds`. Please make sure to only forward one "
                             "of the two.")
        elif prompt_2 is not None and prompt_embeds is not None:
            raise ValueError("Cannot forward both `prompt_2` and `prompt_embeds`.")
        elif prompt is None and prompt_embeds is None:
            raise ValueError("Provide either `prompt` or `prompt_embeds`. Cannot leave both `prompt` and "
                             "`prompt_embeds` undefined.")
        elif prompt is not None and not isinstance(prompt, (str, list)):
            raise ValueError(f"`prompt` has to be of type `str` or `list` but is {type(prompt)}")
        elif prompt_2 is not None and not isinstance(prompt_2, (str, list)):
            raise ValueError(f"`prompt_2` has to be of type `str` or `list` but is {type(prompt_2)}")
        if negative_prompt is not None and negative_prompt_embeds is not None:
            raise ValueError("Cannot forward both `negative_prompt` and `negative_prompt_embeds`.")
        elif negative_prompt_2 is not None and negative_prompt_embeds is not None:
            raise ValueError("Cannot forward both `negative_prompt_2` and `negative_prompt_embeds`.")
        if prompt_embeds is not None and negative_prompt_embeds is not None:
            if prompt_embeds.shape != negative_prompt_embeds.shape:
                raise ValueError("`prompt_embeds` and `negative_prompt_embeds` must have the same shape when passed "
                                 f"directly, but got: {prompt_embeds.shape} != {negative_prompt_embeds.shape}.")
        if prompt_embeds is not None and pooled_prompt_embeds is None:
            raise ValueError("If `prompt_embeds` are provided, `pooled_prompt_embeds` also have to be passed.")
        if negative_prompt_embeds is not None and negative_pooled_prompt_embeds is None:
            raise ValueError("If `negative_prompt_embeds` are provided, `negative_pooled_prompt_embeds` also have to "
                             "be passed.")

    def _preprocess(self, img, height, width):
        """VaeImageProcessor.preprocess (:1246): PIL (resized to (width, height) if needed, LANCZOS) ->
        [-1, 1], laid out NHWC [H*W, 3] fp16 on the device (the host does only the uint8 -> float map)."""
        if isinstance(img, list):
            img = img[0]
        if isinstance(img, torch.Tensor):
            t = img.float()
            if t.ndim == 4:
                t = t[0]
            if t.shape[0] == 3:
                t = t.permute(1, 2, 0)
            arr = t.cpu().numpy()
        else:
            if not isinstance(img, PIL.Image.Image):
                raise ValueError(f"`image` has to be of type `torch.Tensor`, `PIL.Image.Image` or list but is "
                                 f"{type(img)}")
            if img.size != (width, height):
                img = img.resize((width, height), resample=PIL.Image.LANCZOS)
            # the uint8 pixels go to the device (a quarter of the fp32 bytes) and are mapped there with the
            # same fp32 operations numpy would do (x / 255 * 2 - 1, each correctly rounded): ~4 ms of host
            # numpy per 1024^2 image otherwise
            u8 = torch.from_numpy(np.ascontiguousarray(np.asarray(img.convert("RGB"), dtype=np.uint8)))
            x = u8.reshape(-1, 3).to(self.device).to(torch.float32)
            return (x / 255.0 * 2.0 - 1.0).to(torch.float16)
        x = torch.from_numpy(np.ascontiguousarray(arr)).reshape(-1, 3)
        return x.to(self.device, torch.float16)

    def prepare_latents(self, batch_size, num_channels_latents, height, width, dtype, device, generator,
                        latents=None):
        """:820-835 -- returns the *unscaled* noise; the init sigma is applied on device in the fused kernel."""
        shape = (batch_size, num_channels_latents, height // self.vae_scale_factor, width // self.vae_scale_factor)
        if isinstance(generator, list) and len(generator) != batch_size:
            raise ValueError(f"You have passed a list of generators of length {len(generator)}, but requested an "
                             f"effective batch size of {batch_size}.")
        if latents is None:
            return randn_tensor(shape, generator=generator, device=device, dtype=torch.float32)
        return latents.to(device=device, dtype=torch.float32)

    # ------------------------------------------------------------------ the call
    @torch.no_grad()
    def __call__(self, lr_img=None, prompt: Union[str, List[str]] = None, prompt_2=None, height: Optional[int] = None,
                 width: Optional[int] = None, num_inference_steps: int = 50, start_point: Optional[str] = "noise",
                 timesteps: List[int] = None, denoising_end: Optional[float] = None, overlap: float = 0.5,
                 guidance_scale: float = 5.0, negative_prompt=None, negative_prompt_2=None,
                 num_images_per_prompt: Optional[int] = 1, eta: float = 0.0, generator=None,
                 latents: Optional[torch.Tensor] = None, prompt_embeds=None, negative_prompt_embeds=None,
                 pooled_prompt_embeds=None, negative_pooled_prompt_embeds=None, output_type: Optional[str] = "pil",
                 return_dict: bool = True, cross_attention_kwargs: Optional[Dict[str, Any]] = None,
                 guidance_rescale: float = 0.0, original_size: Optional[Tuple[int, int]] = None,
                 target_size: Optional[Tuple[int, int]] = None, clip_skip: Optional[int] = None,
                 callback_on_step_end: Optional[Callable[[int, int, Dict], None]] = None,
                 callback_on_step_end_tensor_inputs: List[str] = ["latents"], add_sample: bool = True, **kwargs):
        if num_images_per_prompt not in (None, 1):
            # the reference's TLC loop restores one latent canvas per call (pipeline:1278-1409)
            raise NotImplementedError("num_images_per_prompt > 1 is not supported by the TLC tile loop; pass a list "
                                      "of images (lr_img=[...]) instead")
        if isinstance(lr_img, (list, tuple)) and len(lr_img) > 1:
            return self._call_images(
                lr_img, prompt, prompt_2=prompt_2, height=height, width=width,
                num_inference_steps=num_inference_steps, start_point=start_point, timesteps=timesteps,
                denoising_end=denoising_end, overlap=overlap, guidance_scale=guidance_scale,
                negative_prompt=negative_prompt, negative_prompt_2=negative_prompt_2, generator=generator,
                latents=latents, prompt_embeds=prompt_embeds, negative_prompt_embeds=negative_prompt_embeds,
                pooled_prompt_embeds=pooled_prompt_embeds, negative_pooled_prompt_embeds=negative_pooled_prompt_embeds,
                output_type=output_type, return_dict=return_dict, cross_attention_kwargs=cross_attention_kwargs,
                guidance_rescale=guidance_rescale, original_size=original_size, target_size=target_size,
                clip_skip=clip_skip, callback_on_step_end=callback_on_step_end,
                callback_on_step_end_tensor_inputs=callback_on_step_end_tensor_inputs, add_sample=add_sample,
                **kwargs)
        callback = kwargs.pop("callback", None)
        callback_steps = kwargs.pop("callback_steps", None)
        posterior_noise = kwargs.pop("posterior_noise", None)  # explicit VAE posterior draw (parity tests)
        timer = kwargs.pop("timer", None)
        # eps_hook(step, tile_begin, ntiles, eps): observation hook for the teacher-forced parity tests -- sees each
        # UNet call's noise prediction (NHWC [ntiles * cfg * kh * kw, 4], CFG rows uncond-first; the graph's static
        # output, valid only inside the call) before the CFG + Euler step consumes it
        eps_hook = kwargs.pop("eps_hook", None)

        height = height or self.default_sample_size * self.vae_scale_factor
        width = width or self.default_sample_size * self.vae_scale_factor
        original_size = original_size or (height, width)
        target_size = target_size or (height, width)
        self.check_inputs(lr_img, prompt, prompt_2, height, width, callback_steps, negative_prompt, negative_prompt_2,
                          prompt_embeds, negative_prompt_embeds, pooled_prompt_embeds, negative_pooled_prompt_embeds,
                          callback_on_step_end_tensor_inputs)
        self._guidance_scale = guidance_scale
        self._guidance_rescale = guidance_rescale
        self._clip_skip = clip_skip
        self._cross_attention_kwargs = cross_attention_kwargs
        self._denoising_end = denoising_end
        self._interrupt = False
        dev = self.device
        if dev.type != "cuda":
            raise RuntimeError("FaithDiff on MI355X: call pipe.to('cuda') (there is no CPU execution path)")
        unet = self.unet.hip()

        # 3. prompts (CFG always requested from encode_prompt, :1240)
        pe, npe, ppe, nppe = self.encode_prompt(prompt, do_classifier_free_guidance=True,
                                                negative_prompt=negative_prompt, prompt_embeds=prompt_embeds,
                                                negative_prompt_embeds=negative_prompt_embeds,
                                                pooled_prompt_embeds=pooled_prompt_embeds,
                                                negative_pooled_prompt_embeds=negative_pooled_prompt_embeds)
        cfg = 2 if self.do_classifier_free_guidance else 1
        if cfg == 2:
            ctx = torch.cat([npe.float(), pe.float()], 0)
            text = torch.cat([nppe.float(), ppe.float()], 0)
        else:
            ctx, text = pe.float(), ppe.float()

        # 4. image + timesteps
        x_img = self._preprocess(lr_img, height, width)
        ts, num_inference_steps = retrieve_timesteps(self.scheduler, num_inference_steps, dev, timesteps)
        if denoising_end is not None and isinstance(denoising_end, float) and 0 < denoising_end < 1:
            cutoff = int(round(self.scheduler.config.num_train_timesteps
                               - denoising_end * self.scheduler.config.num_train_timesteps))
            num_inference_steps = len([t for t in ts if t >= cutoff])
        sig = self.scheduler.sigmas
        self._num_timesteps = num_inference_steps
        h, w = height // 8, width // 8

        # 5. denoise-encoder image latents (:1250-1255) -> TLC tiles (:1257)
        grid = TileGrid(h, w, (target_size[0] // 8, target_size[1] // 8), overlap)
        kh, kw, N = grid.kh, grid.kw, grid.ntiles
        shard = TileShard(N, self.process_group)
        img_lat = self.denoise_encoder.encode_nhwc(x_img, height, width)  # [h*w, 512] fp16
        rows_t = torch.tensor(grid.rows, dtype=torch.int32, device=dev)
        cols_t = torch.tensor(grid.cols, dtype=torch.int32, device=dev)
        cond_dt = unet.dtype
        img_lat_c = torch.empty_like(img_lat, dtype=cond_dt)
        ops.unary(img_lat, img_lat_c)
        cond_tiles = None
        if shard.count:
            cond_tiles = torch.empty((shard.count * cfg, kh * kw, 512), dtype=cond_dt, device=dev)
            ops.tlc_grids_nhwc(img_lat_c, rows_t, cols_t, h, w, 512, kh, kw, shard.begin, shard.count, cfg,
                               cond_tiles)
        del img_lat_c

        # 6. initial latent canvas (:1261-1278): noise * init_sigma [+ DDPM(add_noise) of the VAE sample]
        noise = self.prepare_latents(1, 4, height, width, torch.float32, dev, generator, latents)
        canvas = torch.empty((4, h, w), dtype=torch.float32, device=dev)
        init_sigma = float(self.scheduler.init_noise_sigma)
        if start_point == "lr":
            moments = self.vae.encode_moments_nhwc(x_img, height, width)
            eps_post = (posterior_noise.to(dev, torch.float32) if posterior_noise is not None
                        else torch.randn((1, 4, h, w), device=dev, dtype=torch.float32))
            a, b = self.DDPM_scheduler.add_noise_coefficients(999)
            ops.vae_sample_add_noise(moments, eps_post.contiguous(), noise.contiguous(), canvas, h * w,
                                     self.vae.config.scaling_factor, init_sigma, a, b, True)
        else:
            ops.vae_sample_add_noise(None, None, noise.contiguous(), canvas, h * w, 1.0, init_sigma, 0.0, 1.0, False)
        if shard.world > 1:
            broadcast(canvas, dist.get_global_rank(self.process_group, 0), self.process_group)

        # 7. per-row conditioning, computed once per image
        unet.set_context(ctx.to(dev))
        # capped where the widest activation of one forward would leave the kernels' 32-bit offset range
        tb = max(1, min(self.tile_batch, shard.count or 1, max_tile_batch(kh, kw, cfg)))
        # the FaithDiff condition embedding (ext:528-534) of every tile's image latents: fixed across the denoise
        # loop, so computed once per image here (the reference recomputes it inside every UNet call, :1350),
        # per tile batch, bitwise what the forward would compute (HipUNet.cond_embed)
        cond_emb = False
        if cond_tiles is not None and unet.has_extras:
            ie_tiles = torch.empty((cond_tiles.shape[0], kh * kw, 320), dtype=cond_dt, device=dev)
            # the same tile batches as the denoise loop below (every kernel is bitwise batch-invariant, but the
            # hoisted embedding then rides in exactly the batches the loop's forwards would have used)
            for c0, n in tile_batches(shard.count, tb, self.tile_balance):
                r0, r1 = c0 * cfg, (c0 + n) * cfg
                unet.cond_embed(cond_tiles[r0:r1].reshape(-1, 512), r1 - r0, kh, kw,
                                out=ie_tiles[r0:r1].reshape(-1, 320))
            cond_tiles, cond_emb = ie_tiles, True
        B = tb * cfg
        text_rows = text.to(dev).repeat(tb, 1).contiguous()  # [B, 1280]
        tids_all = torch.tensor([[original_size[0], original_size[1], i, j, target_size[0], target_size[1]]
                                 for (i, j) in [grid.origin(t) for t in range(N)]], dtype=torch.float32)
        tids_all = tids_all.repeat_interleave(cfg, 0).to(dev)  # [N*cfg, 6]
        t_rows = torch.tensor(np.repeat(ts[:num_inference_steps], B), dtype=torch.float32, device=dev).view(-1, B)
        weights = torch.tensor(grid.weights(), dtype=torch.float64, device=dev)
        xin = torch.empty((B * kh * kw, 4), dtype=cond_dt, device=dev)
        canvas_next = torch.empty_like(canvas)
        state = {"canvas": canvas, "next": canvas_next}

        def compute(i, begin, count, out):
            s, s_next = float(sig[i]), float(sig[i + 1])
            for c0, n in tile_batches(count, tb, self.tile_balance):
                rows = n * cfg
                cond = cond_tiles[c0 * cfg:(c0 + n) * cfg].reshape(rows * kh * kw, cond_tiles.shape[-1])
                tid = tids_all[(begin + c0) * cfg:(begin + c0 + n) * cfg]
                # once run()'s graph for this batch shape is captured, the latent tiles and the step's timesteps go
                # straight into its static inputs (one launch, fd_tlc_scale_input_t; no input copies for them)
                st = unet.graph_inputs(rows, kh, kw, add_sample=add_sample, cond_embedded=cond_emb)
                x_in, t_in = (st[0], st[1]) if st is not None else (xin[:rows * kh * kw], t_rows[i, :rows])
                ops.tlc_scale_input(state["canvas"], rows_t, cols_t, h, w, kh, kw, begin + c0, n, cfg, s, x_in,
                                    t_out=t_in if st is not None else None, timestep=float(ts[i]))
                # one hipGraph replay per tile batch after the first two steps (HipUNet.run, fdhip/graphs.py)
                eps = unet.run(x_in, t_in, tid, text_rows[:rows], cond, rows, kh, kw,
                               add_sample=add_sample, cond_embedded=cond_emb)
                if eps_hook is not None:
                    eps_hook(i, begin + c0, n, eps)
                ops.tlc_cfg_euler_step(eps, state["canvas"], rows_t, cols_t, h, w, kh, kw, begin + c0, n, cfg,
                                       guidance_scale, guidance_rescale, s, s_next, out[c0:c0 + n])

        def blend(tiles):
            ops.tlc_blend(tiles.contiguous(), weights, rows_t, cols_t, 4, h, w, kh, kw, state["next"])
            state["canvas"], state["next"] = state["next"], state["canvas"]
            return state["canvas"]

        def on_step(i, cv):
            if timer is not None:
                timer("step", i)
            if callback_on_step_end is not None:
                cb = {k: (cv.view(1, 4, h, w) if k == "latents" else None) for k in callback_on_step_end_tensor_inputs}
                out = callback_on_step_end(self, i, ts[i], cb)
                if out is not None and out.get("latents") is not None:
                    state["canvas"].copy_(out["latents"].reshape(4, h, w))
            if callback is not None and callback_steps and i % callback_steps == 0:
                callback(i, ts[i], cv.view(1, 4, h, w))

        if timer is not None:  # timer(label, i): measurement hook (bench.py records a HIP event per call)
            timer("loop_start", 0)
        final = run_tile_loop(num_inference_steps, shard, (4, kh, kw), compute, blend, dev, on_step=on_step,
                              timer=timer)
        if final is None:
            final = canvas
        lat = final.view(1, 4, h, w)
        if output_type == "latent":
            image = lat.clone()
        else:
            if timer is not None:
                timer("decode_start", 0)
            z = torch.empty((h * w, 4), dtype=self.vae.dtype, device=dev)
            ops.nchw_to_nhwc(final, z, 1, 4, h * w, 1.0 / self.vae.config.scaling_factor)
            y = self.vae.decode_nhwc(z, h, w)  # NHWC [H*W, 3] fp16
            if timer is not None:
                timer("decode", 0)
            image = self._postprocess(y, height, width, output_type)
        ops.split_k_health()  # a timed-out split-K hand-off (never expected) raises here, counters reset
        if not return_dict:
            return (image,)
        return FaithDiffStableDiffusionXLPipelineOutput(images=image)

    @torch.no_grad()
    def _call_images(self, imgs, prompt, prompt_2=None, height=None, width=None, num_inference_steps=50,
                     start_point="noise", timesteps=None, denoising_end=None, overlap=0.5, guidance_scale=5.0,
                     negative_prompt=None, negative_prompt_2=None, generator=None, latents=None, prompt_embeds=None,
                     negative_prompt_embeds=None, pooled_prompt_embeds=None, negative_pooled_prompt_embeds=None,
                     output_type="pil", return_dict=True, cross_attention_kwargs=None, guidance_rescale=0.0,
                     original_size=None, target_size=None, clip_skip=None, callback_on_step_end=None,
                     callback_on_step_end_tensor_inputs=("latents",), add_sample=True, **kwargs):
        """Several images of one size in one call (BASELINE configs[4], C5: a batch of 1024^2 restorations; the
        reference restores one image per pipe() call, test_wo_llava.py:53-97).  When each image is a single TLC
        tile (target_size covers the image latent), the images' CFG pairs share UNet forwards (tile_batch images
        per forward), each pair attending to its own prompt (HipUNet.set_context with several prompt pairs), with
        the per-image work -- prompt encoding, preprocess, denoise encoder, VAE encode / decode, the CFG + Euler
        step and the blend -- unchanged: every image is bitwise the result of its own pipe() call with the same
        prompt, noise (``latents`` [n, 4, h, w]) and posterior draw (``posterior_noise`` [n, 4, h, w]); GPU test.
        Images with several TLC tiles are restored one call at a time.  Per-image tensors (latents, posterior
        noise, the four precomputed embeddings) carry one row per image; prompt lists one entry per image; every
        other argument (clip_skip, cross_attention_kwargs, the step callbacks) applies to every image."""
        nimg = len(imgs)

        def per_image(x, what):
            if x is None or isinstance(x, str):
                return [x] * nimg
            if len(x) != nimg:
                raise ValueError(f"{nimg} images need {nimg} {what} (got {len(x)})")
            return list(x) if not torch.is_tensor(x) else [x[i:i + 1] for i in range(nimg)]
        prompts, prompts_2 = per_image(prompt, "prompts"), per_image(prompt_2, "prompt_2 entries")
        negs, negs_2 = per_image(negative_prompt, "negative prompts"), per_image(negative_prompt_2, "negative_prompt_2")
        embeds = [per_image(e, "embedding rows") for e in (prompt_embeds, negative_prompt_embeds, pooled_prompt_embeds,
                                                           negative_pooled_prompt_embeds)]
        posterior_noise = kwargs.pop("posterior_noise", None)
        timer = kwargs.pop("timer", None)
        callback = kwargs.pop("callback", None)
        callback_steps = kwargs.pop("callback_steps", None)
        height = height or self.default_sample_size * self.vae_scale_factor
        width = width or self.default_sample_size * self.vae_scale_factor
        original_size = original_size or (height, width)
        target_size = target_size or (height, width)
        h, w = height // 8, width // 8
        grid = TileGrid(h, w, (target_size[0] // 8, target_size[1] // 8), overlap)

        def pick(x, i):
            return None if x is None else x[i:i + 1] if torch.is_tensor(x) else x[i]
        if grid.ntiles != 1 or self.process_group is not None:
            outs = []
            for i in range(nimg):
                o = self(lr_img=imgs[i], prompt=prompts[i], prompt_2=prompts_2[i], height=height, width=width,
                         num_inference_steps=num_inference_steps, start_point=start_point, timesteps=timesteps,
                         denoising_end=denoising_end, overlap=overlap, guidance_scale=guidance_scale,
                         negative_prompt=negs[i], negative_prompt_2=negs_2[i], generator=generator,
                         latents=pick(latents, i), prompt_embeds=embeds[0][i], negative_prompt_embeds=embeds[1][i],
                         pooled_prompt_embeds=embeds[2][i], negative_pooled_prompt_embeds=embeds[3][i],
                         output_type=output_type, return_dict=True, cross_attention_kwargs=cross_attention_kwargs,
                         guidance_rescale=guidance_rescale, original_size=original_size, target_size=target_size,
                         clip_skip=clip_skip, callback_on_step_end=callback_on_step_end,
                         callback_on_step_end_tensor_inputs=callback_on_step_end_tensor_inputs,
                         add_sample=add_sample, posterior_noise=pick(posterior_noise, i), timer=timer,
                         callback=callback, callback_steps=callback_steps, **kwargs)
                outs.extend(o.images if isinstance(o.images, list) else [o.images])
            return FaithDiffStableDiffusionXLPipelineOutput(images=outs) if return_dict else (outs,)
        for i in range(nimg):
            self.check_inputs(imgs[i], prompts[i], prompts_2[i], height, width, callback_steps, negs[i], negs_2[i],
                              *[e[i] for e in embeds], callback_on_step_end_tensor_inputs)
        self._guidance_scale, self._guidance_rescale = guidance_scale, guidance_rescale
        self._clip_skip, self._cross_attention_kwargs, self._denoising_end = clip_skip, cross_attention_kwargs, \
            denoising_end
        self._interrupt = False
        dev = self.device
        if dev.type != "cuda":
            raise RuntimeError("FaithDiff on MI355X: call pipe.to('cuda') (there is no CPU execution path)")
        unet = self.unet.hip()
        cfg = 2 if self.do_classifier_free_guidance else 1
        # prompts: one encoder pass over every image's prompt and negative prompt (each prompt its own row group)
        def joined(col):
            return None if col[0] is None else torch.cat(col, 0)
        pe, npe, ppe, nppe = self.encode_prompt(
            None if prompts[0] is None else prompts, prompt_2=None if prompts_2[0] is None else prompts_2,
            do_classifier_free_guidance=True, negative_prompt=negs if any(n is not None for n in negs) else None,
            negative_prompt_2=None if negs_2[0] is None else negs_2, prompt_embeds=joined(embeds[0]),
            negative_prompt_embeds=joined(embeds[1]), pooled_prompt_embeds=joined(embeds[2]),
            negative_pooled_prompt_embeds=joined(embeds[3]), clip_skip=clip_skip)
        if cfg == 2:
            ctx = torch.stack([npe.float(), pe.float()], 1).reshape(2 * nimg, *pe.shape[1:])
            text = torch.stack([nppe.float(), ppe.float()], 1).reshape(2 * nimg, -1)
        else:
            ctx, text = pe.float(), ppe.float()
        ts, num_inference_steps = retrieve_timesteps(self.scheduler, num_inference_steps, dev, timesteps)
        if denoising_end is not None and isinstance(denoising_end, float) and 0 < denoising_end < 1:
            cutoff = int(round(self.scheduler.config.num_train_timesteps
                               - denoising_end * self.scheduler.config.num_train_timesteps))
            num_inference_steps = len([t for t in ts if t >= cutoff])
        sig = self.scheduler.sigmas
        self._num_timesteps = num_inference_steps
        kh, kw = grid.kh, grid.kw
        rows_t = torch.tensor(grid.rows, dtype=torch.int32, device=dev)
        cols_t = torch.tensor(grid.cols, dtype=torch.int32, device=dev)
        cond_dt = unet.dtype
        cond_tiles = torch.empty((nimg * cfg, kh * kw, 512), dtype=cond_dt, device=dev)
        canvas = torch.empty((nimg, 4, h, w), dtype=torch.float32, device=dev)
        init_sigma = float(self.scheduler.init_noise_sigma)
        a, b = self.DDPM_scheduler.add_noise_coefficients(999)
        if timer is not None:
            timer("images_start", 0)
        for i in range(nimg):  # per image, exactly as __call__: preprocess, denoise encoder, grids, start latents
            x_img = self._preprocess(imgs[i], height, width)
            img_lat = self.denoise_encoder.encode_nhwc(x_img, height, width)  # the graph's buffer: used right away
            img_lat_c = torch.empty_like(img_lat, dtype=cond_dt)
            ops.unary(img_lat, img_lat_c)
            ops.tlc_grids_nhwc(img_lat_c, rows_t, cols_t, h, w, 512, kh, kw, 0, 1, cfg, cond_tiles[i * cfg:])
            noise = self.prepare_latents(1, 4, height, width, torch.float32, dev, generator, pick(latents, i))
            if start_point == "lr":
                moments = self.vae.encode_moments_nhwc(x_img, height, width)
                pn = pick(posterior_noise, i)
                eps_post = (pn.to(dev, torch.float32) if pn is not None
                            else torch.randn((1, 4, h, w), device=dev, dtype=torch.float32))
                ops.vae_sample_add_noise(moments, eps_post.contiguous(), noise.contiguous(), canvas[i], h * w,
                                         self.vae.config.scaling_factor, init_sigma, a, b, True)
            else:
                ops.vae_sample_add_noise(None, None, noise.contiguous(), canvas[i], h * w, 1.0, init_sigma, 0.0, 1.0,
                                         False)
        unet.set_context(ctx.to(dev), ncfg=cfg)
        tb = max(1, min(self.tile_batch, nimg, max_tile_batch(kh, kw, cfg)))
        cond_emb = False
        if unet.has_extras:  # the condition embedding of every image's tile, once per call (HipUNet.cond_embed)
            ie = torch.empty((nimg * cfg, kh * kw, 320), dtype=cond_dt, device=dev)
            for c0 in range(0, nimg, tb):
                r0, r1 = c0 * cfg, min(c0 + tb, nimg) * cfg
                unet.cond_embed(cond_tiles[r0:r1].reshape(-1, 512), r1 - r0, kh, kw, out=ie[r0:r1].reshape(-1, 320))
            cond_tiles, cond_emb = ie, True
        text_rows = text.to(dev).contiguous()  # [nimg*cfg, 1280]
        tids = torch.tensor([[original_size[0], original_size[1], *grid.origin(0), target_size[0], target_size[1]]],
                            dtype=torch.float32).repeat(tb * cfg, 1).to(dev)
        t_rows = torch.tensor(np.repeat(ts[:num_inference_steps], tb * cfg), dtype=torch.float32,
                              device=dev).view(-1, tb * cfg)
        weights = torch.tensor(grid.weights(), dtype=torch.float64, device=dev)
        xin = torch.empty((tb * cfg * kh * kw, 4), dtype=cond_dt, device=dev)
        tiles = torch.empty((nimg, 1, 4, kh, kw), dtype=torch.float32, device=dev)
        nxt = torch.empty_like(canvas)
        if timer is not None:
            timer("loop_start", 0)
        for st in range(num_inference_steps):
            s_, sn = float(sig[st]), float(sig[st + 1])
            for c0 in range(0, nimg, tb):
                n = min(tb, nimg - c0)
                rows, per = n * cfg, cfg * kh * kw
                for j in range(n):
                    ops.tlc_scale_input(canvas[c0 + j], rows_t, cols_t, h, w, kh, kw, 0, 1, cfg, s_,
                                        xin[j * per:(j + 1) * per])
                cond = cond_tiles[c0 * cfg:(c0 + n) * cfg].reshape(rows * kh * kw, cond_tiles.shape[-1])
                eps = unet.run(xin[:rows * kh * kw], t_rows[st, :rows], tids[:rows], text_rows[c0 * cfg:(c0 + n) * cfg],
                               cond, rows, kh, kw, add_sample=add_sample, cond_embedded=cond_emb, kv_pair0=c0)
                for j in range(n):
                    ops.tlc_cfg_euler_step(eps[j * per:(j + 1) * per], canvas[c0 + j], rows_t, cols_t, h, w, kh, kw,
                                           0, 1, cfg, guidance_scale, guidance_rescale, s_, sn, tiles[c0 + j])
            for i in range(nimg):
                ops.tlc_blend(tiles[i], weights, rows_t, cols_t, 4, h, w, kh, kw, nxt[i])
            canvas, nxt = nxt, canvas
            if timer is not None:
                timer("step", st)
            if callback_on_step_end is not None:
                cb = {k: (canvas if k == "latents" else None) for k in callback_on_step_end_tensor_inputs}
                out = callback_on_step_end(self, st, ts[st], cb)
                if out is not None and out.get("latents") is not None:
                    canvas.copy_(out["latents"].reshape(nimg, 4, h, w))
            if callback is not None and callback_steps and st % callback_steps == 0:
                callback(st, ts[st], canvas)
        if output_type == "latent":
            images = canvas.clone()
        else:
            if timer is not None:
                timer("decode_start", 0)
            images = []
            for i in range(nimg):
                z = torch.empty((h * w, 4), dtype=self.vae.dtype, device=dev)
                ops.nchw_to_nhwc(canvas[i], z, 1, 4, h * w, 1.0 / self.vae.config.scaling_factor)
                y = self.vae.decode_nhwc(z, h, w)
                im = self._postprocess(y, height, width, output_type)
                images.extend(im if isinstance(im, list) else [im])
            if timer is not None:
                timer("decode", 0)
        ops.split_k_health()
        if not return_dict:
            return (images,)
        return FaithDiffStableDiffusionXLPipelineOutput(images=images)

    def _postprocess(self, y, H, W, output_type):
        """VaeImageProcessor.postprocess (:1451)."""
        if output_type == "pt":
            out = torch.empty((1, 3, H, W), dtype=y.dtype, device=y.device)
            ops.nhwc_to_nchw(y, out, 1, 3, H * W)
            return (out.float() / 2 + 0.5).clamp(0, 1)
        u8 = torch.empty((H * W, 3), dtype=torch.uint8, device=y.device)
        ops.postprocess_u8(y, u8)
        arr = u8.view(H, W, 3).cpu().numpy()
        if output_type == "np":
            return arr[None].astype(np.float32) / 255.0
        return [PIL.Image.fromarray(arr)]
