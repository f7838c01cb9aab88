"""Drop-in for FaithDiff/models/unet_2d_condition_vae_extension.py on the MI355X HIP path.

``UNet2DConditionModel`` keeps the reference's operator surface -- ``from_pretrained``,
``load_additional_layers`` (ext:405-433) with the prefix-split state dict (core non-strict, extras
strict; ext:444-478), ``to``, ``config``/``dtype`` and ``forward(sample, timestep, encoder_hidden_states,
..., added_cond_kwargs, input_embedding, add_sample, return_dict)`` (ext:480-697) -- but computes on
``fdhip.unet.HipUNet`` (NHWC bf16 MFMA kernels).  ``Encoder`` is the denoise encoder (ext:39-196) on
``fdhip.vae.HipEncoder``; ``AutoencoderKL`` is the fp16 VAE.

Weights: a local diffusers directory / file is loaded with safe loaders only (safetensors, or
``torch.load(weights_only=True)`` -- the reference's ``weights_only=False`` pickle load at ext:427 is not
reproduced); the ``random-init`` sentinel (CKPT_PTH) draws seeded random weights (fdhip.arch).
"""
import os
from types import SimpleNamespace

import torch

from fdhip import arch, knobs, ops
from fdhip import lib as L

RANDOM_INIT = "random-init"
# Path sentinel for a rank that builds a pipeline collectively (FaithDiff_pipeline(process_group=...)) and is not
# the source: it reads nothing and allocates the architecture's tensors, which rank 0 then broadcasts.
RECEIVE = "receive-from-rank0"


def _empty(shapes, device="cpu"):
    return {k: torch.empty(s, dtype=torch.float32, device=device) for k, s in shapes.items()}


def _load_file(path):
    if path.endswith(".safetensors"):
        from safetensors.torch import load_file
        return load_file(path)
    return torch.load(path, map_location="cpu", weights_only=True)


def _find_weights(root, subfolder, variant=None):
    d = os.path.join(root, subfolder) if subfolder else root
    names = []
    if variant:
        names += [f"diffusion_pytorch_model.{variant}.safetensors", f"diffusion_pytorch_model.{variant}.bin"]
    names += ["diffusion_pytorch_model.safetensors", "diffusion_pytorch_model.bin"]
    for n in names:
        p = os.path.join(d, n)
        if os.path.exists(p):
            return p
    raise FileNotFoundError(f"no diffusers weights under {d} (looked for {names}); use '{RANDOM_INIT}' offline")


def _check_keys(sd, shapes, strict, what):
    missing = [k for k in shapes if k not in sd]
    unexpected = [k for k in sd if k not in shapes]
    bad = [k for k in shapes if k in sd and tuple(sd[k].shape) != tuple(shapes[k])]
    if bad or (strict and (missing or unexpected)):
        raise RuntimeError(f"Error(s) in loading state_dict for {what}: missing={missing[:5]} "
                           f"unexpected={unexpected[:5]} shape_mismatch={bad[:5]}")
    return missing


class UNet2DConditionModel:
    """FaithDiff UNet (SDXL core + extras) executing on HIP."""

    EXTRA_PREFIXES = ("denoise_encoder.", "information_transformer_layes.", "condition_embedding.", "agg_net.",
                      "spatial_ch_projs.")

    def __init__(self, core_state_dict, seed=0):
        self.config = SimpleNamespace(sample_size=128, in_channels=4, out_channels=4, time_cond_proj_dim=None,
                                      block_out_channels=(320, 640, 1280), cross_attention_dim=2048,
                                      addition_time_embed_dim=256, projection_class_embeddings_input_dim=2816)
        self._sd = dict(core_state_dict)
        self._seed = seed
        self._dtype = torch.float32
        self._device = torch.device("cpu")
        self._hip = None
        self._fp8 = False
        self._fp8_mfma = None
        self.denoise_encoder = None
        self.information_transformer_layes = None
        self.condition_embedding = None
        self.agg_net = None
        self.spatial_ch_projs = None

    # ------------------------------------------------------------------ construction / loading
    @classmethod
    def from_pretrained(cls, path, subfolder="unet", variant=None, seed=0, init_device="cpu", **kwargs):
        shapes = arch.unet_param_shapes(with_extras=False)
        if path == RANDOM_INIT:
            sd = arch.random_init(shapes, seed=seed, device=init_device)
        elif path == RECEIVE:
            sd = _empty(shapes, init_device)
        else:
            sd = _load_file(_find_weights(path, subfolder, variant))
            _check_keys(sd, shapes, True, "UNet2DConditionModel")
        return cls(sd, seed=seed)

    def load_additional_layers(self, dtype=torch.float16, channel=512, weight_path=None, init_device="cpu"):
        """ext:405-433: build the extras (+ denoise encoder), then load ``weight_path`` if given."""
        ext_shapes = {k: v for k, v in arch.unet_param_shapes(True).items() if k.startswith(self.EXTRA_PREFIXES)}
        den_shapes = arch.encoder_param_shapes("denoise_encoder.", with_out=False)
        if weight_path is None or weight_path == RANDOM_INIT:
            extra = arch.random_init({**ext_shapes, **den_shapes}, seed=self._seed + 7, device=init_device)
        elif weight_path == RECEIVE:
            extra = _empty({**ext_shapes, **den_shapes}, init_device)
        else:
            extra = _load_file(weight_path)
        self.load_state_dict(extra, strict=True)
        self._dtype = dtype or self._dtype

    def load_state_dict(self, state_dict, strict=True):
        """ext:444-478: prefix split; core non-strict, every present extras group strict."""
        ext_shapes = {k: v for k, v in arch.unet_param_shapes(True).items() if k.startswith(self.EXTRA_PREFIXES)}
        den_shapes = arch.encoder_param_shapes("denoise_encoder.", with_out=False)
        core = {k: v for k, v in state_dict.items() if not k.startswith(self.EXTRA_PREFIXES)}
        _check_keys(core, arch.unet_param_shapes(False), False, "UNet2DConditionModel")
        self._sd.update(core)
        groups = {"information_transformer_layes.": {}, "condition_embedding.": {}, "spatial_ch_projs.": {},
                  "denoise_encoder.": {}, "agg_net.": {}}
        for k, v in state_dict.items():
            for p in groups:
                if k.startswith(p):
                    groups[p][k] = v
        for p, d in groups.items():
            if not d:
                continue
            if p == "agg_net.":
                # the reference's agg_net is an empty nn.ModuleList (ext:402-403): every key is unexpected
                if strict:
                    raise RuntimeError(f"Error(s) in loading state_dict for ModuleList: unexpected={sorted(d)[:5]}")
                continue
            want = den_shapes if p == "denoise_encoder." else {k: s for k, s in ext_shapes.items() if k.startswith(p)}
            _check_keys(d, want, strict, p[:-1])
            if p == "denoise_encoder.":
                self.denoise_encoder = Encoder({k[len(p):]: v for k, v in d.items()})
            else:
                self._sd.update(d)
        self.information_transformer_layes = "information_transformer_layes.0.ln_1.weight" in self._sd or None
        self.condition_embedding = "condition_embedding.conv_in.weight" in self._sd or None
        self.spatial_ch_projs = "spatial_ch_projs.weight" in self._sd or None
        self._hip = None

    def quantize_8bit(self, fp8_mfma=None):
        """utils/system.py:13-32: every UNet parameter (core + extras, incl. norms and biases) becomes unscaled
        float8_e4m3fn.  By default compute stays 16-bit on the exact e4m3 values (bf16 here, fp16 under the
        reference's autocast, pipeline:1349) -- the reference's arithmetic.  ``fp8_mfma=True`` (or
        FD_FP8_MFMA=1) opts in to the CDNA4 e4m3 MFMA for the transformer Linears, which ALSO quantizes their
        activations per row to e4m3: a numerics change the reference does not make.  The
        denoise encoder stays fp16 (:24-26).  See fdhip.arch.quantize_e4m3."""
        self._fp8 = True
        if fp8_mfma is not None:
            self._fp8_mfma = bool(fp8_mfma)
        self._hip = None

    # ------------------------------------------------------------------ device
    @property
    def dtype(self):
        return self._dtype

    @property
    def device(self):
        return self._device

    def to(self, device=None, dtype=None, **kwargs):
        if isinstance(device, torch.dtype):
            device, dtype = None, device
        if dtype is not None and dtype != self._dtype:
            self._dtype = dtype
            self._hip = None
        if device is not None:
            self._device = torch.device(device)
            if self._device.type == "cuda" and self._device.index is None:
                self._device = torch.device("cuda", torch.cuda.current_device())
        if self.denoise_encoder is not None:
            self.denoise_encoder.to(device=device)
        return self

    def hip(self):
        """The packed HIP module (built on first use on a CUDA/HIP device; no CPU execution exists)."""
        if self._hip is None:
            if self._device.type != "cuda":
                raise RuntimeError("the FaithDiff UNet runs only on an MI355X (gfx950); call .to('cuda') first")
            from fdhip.unet import HipUNet
            cdt = torch.bfloat16 if self._dtype in (torch.float32, torch.bfloat16, torch.float8_e4m3fn) \
                else self._dtype
            sd = arch.quantize_e4m3(self._sd) if self._fp8 else self._sd
            # default: 16-bit MFMA on the widened e4m3 values (exactly the reference's autocast arithmetic);
            # opt-in (quantize_8bit(fp8_mfma=True) or FD_FP8_MFMA=1): transformer Linears on the e4m3 MFMA
            opt = self._fp8_mfma if self._fp8_mfma is not None else knobs.get("FD_FP8_MFMA") == 1
            fp8_mfma = self._fp8 and opt
            self._hip = HipUNet(sd, self._device, cdt, fp8_mfma=fp8_mfma)
        return self._hip

    def release_host_weights(self):
        self.hip()
        self._sd = {}

    # ------------------------------------------------------------------ reference-compatible forward
    def __call__(self, *a, **k):
        return self.forward(*a, **k)

    @torch.no_grad()
    def forward(self, sample, timestep, encoder_hidden_states, class_labels=None, timestep_cond=None,
                attention_mask=None, cross_attention_kwargs=None, added_cond_kwargs=None,
                down_block_additional_residuals=None, mid_block_additional_residual=None,
                down_intrablock_additional_residuals=None, encoder_attention_mask=None, input_embedding=None,
                add_sample=True, return_dict=True, use_condition_embedding=True):
        """NCHW in / NCHW out like ext:480-697 (the pipeline itself calls the NHWC fast path)."""
        if any(a is not None for a in (class_labels, timestep_cond, attention_mask, down_block_additional_residuals,
                                       mid_block_additional_residual, down_intrablock_additional_residuals,
                                       encoder_attention_mask)):
            raise NotImplementedError("ControlNet / T2I-adapter residuals, masks and class labels are not part of "
                                      "the FaithDiff hot path")
        if not use_condition_embedding:
            raise NotImplementedError("use_condition_embedding=False is not on the FaithDiff hot path")
        hip = self.hip()
        dev, cdt = hip.device, hip.dtype
        B, _, H, W = sample.shape
        x = torch.empty((B * H * W, 4), dtype=cdt, device=dev)
        ops.nchw_to_nhwc(sample.to(dev).contiguous(), x, B, 4, H * W)
        cond = None
        if input_embedding is not None:
            cond = torch.empty((B * H * W, input_embedding.shape[1]), dtype=cdt, device=dev)
            ops.nchw_to_nhwc(input_embedding.to(dev).contiguous(), cond, B, input_embedding.shape[1], H * W)
        ctx = encoder_hidden_states.to(dev)
        hip.set_context(ctx)  # per-sample rows: kv_mod = B, and the extras' MHA spans all B rows (ext:577)
        t = torch.as_tensor(timestep, dtype=torch.float32, device=dev).reshape(-1).expand(B).contiguous()
        tids = added_cond_kwargs["time_ids"].to(dev, torch.float32).contiguous()
        text = added_cond_kwargs["text_embeds"].to(dev, torch.float32).contiguous()
        eps = hip.forward(x, t, tids, text, cond, B, H, W, add_sample=add_sample)
        out = torch.empty((B, 4, H, W), dtype=sample.dtype if sample.dtype != torch.float64 else torch.float32,
                          device=dev)
        ops.nhwc_to_nchw(eps, out, B, 4, H * W)
        return (out,) if not return_dict else SimpleNamespace(sample=out)


class Encoder:
    """FaithDiff denoise encoder (ext:39-196): VAE encoder trunk without conv_out, fp16, optional tiling."""

    def __init__(self, state_dict):
        self._sd = state_dict
        self.dtype = torch.float16
        self._device = torch.device("cpu")
        self._hip = None
        self.tile_sample_min_size = 1024
        self.tile_latent_min_size = int(self.tile_sample_min_size / 8)
        self.tile_overlap_factor = 0.25
        self.use_tiling = False
        self.process_group = None  # set by pipe.enable_tile_parallel: tiles sharded over its ranks

    def enable_tiling(self):
        self.use_tiling = True

    def disable_tiling(self):
        self.use_tiling = False

    def to(self, device=None, dtype=None, **kwargs):
        if device is not None and not isinstance(device, torch.dtype):
            self._device = torch.device(device)
            if self._device.type == "cuda" and self._device.index is None:
                self._device = torch.device("cuda", torch.cuda.current_device())
        return self

    def hip(self):
        if self._hip is None:
            if self._device.type != "cuda":
                raise RuntimeError("the denoise encoder runs only on an MI355X (gfx950); call .to('cuda') first")
            from fdhip.vae import HipEncoder
            self._hip = HipEncoder(self._sd, "", with_out=False, device=self._device, dtype=self.dtype)
        return self._hip

    def encode_nhwc(self, x, H, W):
        """x NHWC fp16 [H*W, 3] -> NHWC fp16 [(H/8)*(W/8), 512] (tiled per ext:164-196 when enabled)."""
        if self.use_tiling and (W > self.tile_latent_min_size or H > self.tile_latent_min_size):
            from fdhip.tiling import tiled_encoder_forward
            return tiled_encoder_forward(self, x, H, W, self.process_group)
        return self.hip().encode_graphed(x, 1, H, W)

    def __call__(self, sample):
        """NCHW [1,3,H,W] -> NCHW [1,512,H/8,W/8] (reference signature, ext:192-196)."""
        _, _, H, W = sample.shape
        x = torch.empty((H * W, 3), dtype=self.dtype, device=self._device)
        ops.nchw_to_nhwc(sample.to(self._device).contiguous(), x, 1, 3, H * W)
        y = self.encode_nhwc(x, H, W)
        out = torch.empty((1, 512, H // 8, W // 8), dtype=self.dtype, device=self._device)
        ops.nhwc_to_nchw(y, out, 1, 512, (H // 8) * (W // 8))
        return out


class _LatentDist:
    def __init__(self, vae, moments, h, w):
        self.vae, self.moments, self.h, self.w = vae, moments, h, w

    def sample(self, generator=None):
        dev = self.moments.device
        eps = torch.randn((1, 4, self.h, self.w), generator=generator, device=dev, dtype=torch.float32)
        out = torch.empty((1, 4, self.h, self.w), dtype=torch.float32, device=dev)
        ops.vae_sample_add_noise(self.moments, eps, eps, out, self.h * self.w, 1.0, 0.0, 1.0, 0.0, True)
        return out


class AutoencoderKL:
    """sdxl-vae-fp16-fix on HIP (fp16).  encode -> .latent_dist.sample(); decode(z) -> (image,)."""

    def __init__(self, state_dict):
        self._sd = state_dict
        self.config = SimpleNamespace(scaling_factor=0.13025, latent_channels=4,
                                      block_out_channels=(128, 256, 512, 512), force_upcast=False, latents_mean=None,
                                      latents_std=None, sample_size=1024)
        self.dtype = torch.float16
        self._device = torch.device("cpu")
        self._enc = self._dec = None
        self.use_tiling = False
        self.process_group = None  # set by pipe.enable_tile_parallel: tiled encode / decode sharded over its ranks
        self.tile_overlap_factor = 0.25
        # diffusers sets these from config.sample_size at construction; later config changes (as
        # set_encoder_tile_settings makes, pipeline:895) do not move them -- reproduced.
        self.tile_sample_min_size = self.config.sample_size
        self.tile_latent_min_size = int(self.config.sample_size / 8)

    @classmethod
    def from_pretrained(cls, path, subfolder=None, seed=0, init_device="cpu", **kwargs):
        shapes = arch.vae_param_shapes()
        if path == RANDOM_INIT:
            sd = arch.random_init(shapes, seed=seed + 3, device=init_device)
        elif path == RECEIVE:
            sd = _empty(shapes, init_device)
        else:
            sd = _load_file(_find_weights(path, subfolder or ""))
            _check_keys(sd, shapes, True, "AutoencoderKL")
        return cls(sd)

    def enable_tiling(self):
        self.use_tiling = True

    def disable_tiling(self):
        self.use_tiling = False

    def to(self, device=None, dtype=None, **kwargs):
        if isinstance(device, torch.dtype):
            device, dtype = None, device
        if device is not None:
            self._device = torch.device(device)
            if self._device.type == "cuda" and self._device.index is None:
                self._device = torch.device("cuda", torch.cuda.current_device())
        if dtype is not None:
            self.dtype = dtype
        return self

    def _need(self):
        if self._device.type != "cuda":
            raise RuntimeError("the VAE runs only on an MI355X (gfx950); call .to('cuda') first")

    def encoder_hip(self):
        self._need()
        if self._enc is None:
            from fdhip.vae import HipEncoder
            self._enc = HipEncoder(self._sd, "encoder.", with_out=True, device=self._device, dtype=self.dtype,
                                   quant_sd=self._sd)
        return self._enc

    def decoder_hip(self):
        self._need()
        if self._dec is None:
            from fdhip.vae import HipDecoder
            self._dec = HipDecoder(self._sd, device=self._device, dtype=self.dtype)
        return self._dec

    def encode_moments_nhwc(self, x, H, W):
        if self.use_tiling and (H > self.tile_sample_min_size or W > self.tile_sample_min_size):
            from fdhip.tiling import tiled_vae_encode
            return tiled_vae_encode(self, x, H, W, self.process_group)
        return self.encoder_hip().encode_graphed(x, 1, H, W)

    def decode_nhwc(self, z, h, w):
        tl = self.tile_latent_min_size
        if self.use_tiling and (h > tl or w > tl):
            from fdhip.tiling import tiled_vae_decode
            return tiled_vae_decode(self, z, h, w, self.process_group)
        return self.decoder_hip().decode_graphed(z, 1, h, w)

    def encode(self, x, return_dict=True):
        _, _, H, W = x.shape
        xn = torch.empty((H * W, 3), dtype=self.dtype, device=self._device)
        ops.nchw_to_nhwc(x.to(self._device).contiguous(), xn, 1, 3, H * W)
        m = self.encode_moments_nhwc(xn, H, W).clone()  # the latent_dist outlives the graph's output buffer
        d = _LatentDist(self, m, H // 8, W // 8)
        return SimpleNamespace(latent_dist=d) if return_dict else (d,)

    def decode(self, z, return_dict=True):
        _, _, h, w = z.shape
        zn = torch.empty((h * w, 4), dtype=self.dtype, device=self._device)
        ops.nchw_to_nhwc(z.to(self._device).contiguous(), zn, 1, 4, h * w)
        y = self.decode_nhwc(zn, h, w)
        out = torch.empty((1, 3, 8 * h, 8 * w), dtype=self.dtype, device=self._device)
        ops.nhwc_to_nchw(y, out, 1, 3, 64 * h * w)
        return SimpleNamespace(sample=out) if return_dict else (out,)
