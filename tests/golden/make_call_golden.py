"""Pin the denoise-loop orchestration: run the reference's own ``FaithDiffStableDiffusionXLPipeline.__call__``
(pipeline_FaithDiff_tlc.py:1187-1459) on CPU and record its outputs (tests/golden/call_golden.npz).

Run in the build container only (the reference is not on the GPU box):
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_call_golden.py

The reference's module is stub-imported as in make_golden.py (diffusers / cv2 / peft / torchvision absent).  What
the reference would take from diffusers is supplied here as restatements with diffusers 0.28's interface:
  * the Euler scheduler: diffusers EulerDiscreteScheduler semantics (scale_model_input / step with a step index
    that the reference saves and restores per tile, :1282,1331,1375), its timestep / sigma schedule computed by
    the product's host scheduler (FaithDiff/schedulers);
  * DDPMScheduler.add_noise (:1276), VaeImageProcessor pre/post-processing (identity on tensors here);
  * the UNet / VAE / denoise encoder: cheap deterministic stand-ins (tests/golden/_det.py) that depend on every
    input the loop hands them (CFG row order, tile position via add_time_ids, timestep, image latents);
  * encode_prompt returns fixed embeddings (the reference passes ``prompt`` to it, :1237-1243; its numerics are
    pinned against transformers' CLIP elsewhere);
  * the module's hard-coded ``torch.device('cuda')`` (:1223) and ``device=`` of _gaussian_weights (:228) map to
    the CPU through a proxy of the ``torch`` module installed in the reference module's globals only.
What is pinned: CFG concatenation order ([negative, positive]), add_time_ids = [orig, tile (i, j), target] per
tile, scale_model_input / Euler per tile with the per-tile scheduler state, CFG combine (+ rescale_noise_cfg),
the start_point 'lr' VAE sample and DDPM add_noise at t = 999 on noise * init_sigma, TLC grids / blend every step,
latents / scaling_factor into the decoder.  Only inputs and outputs are written; no reference source is copied.
"""
import importlib
import os
import sys
import types
from types import SimpleNamespace

import numpy as np
import torch

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
for p in (HERE, os.path.join(ROOT, "faithdiff-dev_amd")):
    sys.path.insert(0, p)
from _det import (call_cases, call_inputs, standin_decode, standin_eps, standin_features,  # noqa: E402
                  standin_moments)
# the product's host schedule math, imported before the reference's own ``FaithDiff`` package takes the name
from FaithDiff.schedulers import EulerDiscreteScheduler as _ProductEuler, _alphas_cumprod  # noqa: E402

for _m in [m for m in sys.modules if m == "FaithDiff" or m.startswith("FaithDiff.")]:
    del sys.modules[_m]
sys.path.remove(os.path.join(ROOT, "faithdiff-dev_amd"))


class _TorchOnCPU(types.ModuleType):
    """The reference module's ``torch`` global: real torch, except that 'cuda' devices resolve to the CPU."""

    def __init__(self):
        super().__init__("torch")

    def __getattr__(self, name):
        return getattr(torch, name)

    @staticmethod
    def device(*a, **k):
        return torch.device("cpu")

    @staticmethod
    def tensor(*a, **k):
        k.pop("device", None)
        return torch.tensor(*a, **k)


class EulerShim:
    """diffusers 0.28 EulerDiscreteScheduler semantics (s_churn 0, epsilon prediction), schedule from the product's
    host scheduler."""
    order = 1

    def __init__(self):
        self.config = SimpleNamespace(num_train_timesteps=1000)
        self.timesteps = self.sigmas = None
        self._step_index = None

    def set_timesteps(self, num_inference_steps, device=None):
        s = _ProductEuler()
        s.set_timesteps(num_inference_steps)
        self.timesteps = torch.from_numpy(np.asarray(s.timesteps, dtype=np.float32))
        self.sigmas = torch.from_numpy(np.asarray(s.sigmas, dtype=np.float32))
        self._init_sigma = float(s.init_noise_sigma)
        self._step_index = None

    @property
    def init_noise_sigma(self):
        return self._init_sigma

    def _init_step_index(self, t):
        idx = (self.timesteps == t).nonzero()
        self._step_index = int(idx[1 if len(idx) > 1 else 0].item())

    def scale_model_input(self, sample, t):
        if self._step_index is None:
            self._init_step_index(t)
        sigma = self.sigmas[self._step_index]
        return sample / ((sigma ** 2 + 1) ** 0.5)

    def step(self, model_output, timestep, sample, generator=None, return_dict=True):
        if self._step_index is None:
            self._init_step_index(timestep)
        sample = sample.to(torch.float32)
        sigma = self.sigmas[self._step_index]
        pred = sample - sigma * model_output
        derivative = (sample - pred) / sigma
        prev = (sample + derivative * (self.sigmas[self._step_index + 1] - sigma)).to(model_output.dtype)
        self._step_index += 1
        return (prev,)


class DDPMShim:
    def __init__(self):
        self.alphas_cumprod = torch.from_numpy(_alphas_cumprod())

    def add_noise(self, original, noise, timesteps):
        acp = self.alphas_cumprod.to(dtype=original.dtype)
        a = (acp[timesteps] ** 0.5).flatten().view(-1, 1, 1, 1)
        b = ((1 - acp[timesteps]) ** 0.5).flatten().view(-1, 1, 1, 1)
        return a * original + b * noise


class VAEShim:
    def __init__(self, post_eps, record):
        self.post_eps, self.record = post_eps, record
        self.config = SimpleNamespace(scaling_factor=0.13025, latent_channels=4, force_upcast=False,
                                      latents_mean=None, latents_std=None, block_out_channels=(128, 256, 512, 512))
        self.dtype = torch.float32

    def encode(self, x, return_dict=True):
        m = standin_moments(x)
        mean, logvar = m.chunk(2, dim=1)
        eps = self.post_eps
        dist = SimpleNamespace(sample=lambda generator=None: mean + torch.exp(0.5 * logvar.clamp(-30.0, 20.0)) * eps)
        return SimpleNamespace(latent_dist=dist)

    def decode(self, z, return_dict=True):
        self.record["z"] = z.clone()
        y = standin_decode(z)
        return (y,) if not return_dict else SimpleNamespace(sample=y)


class UNetShim:
    config = SimpleNamespace(time_cond_proj_dim=None, sample_size=128)
    dtype = torch.float32

    def __call__(self, sample, timestep, encoder_hidden_states=None, timestep_cond=None, cross_attention_kwargs=None,
                 input_embedding=None, add_sample=True, added_cond_kwargs=None, return_dict=True):
        eps = standin_eps(sample, timestep, encoder_hidden_states, added_cond_kwargs["text_embeds"],
                          added_cond_kwargs["time_ids"], input_embedding)
        return (eps,)


def reference_call(mod, case, seed):
    name, H, W, target, steps, g, rescale, start = case
    img, pe, npe, ppe, nppe, noise, post = call_inputs(H, W, seed)
    rec = {}
    Pipe = mod.FaithDiffStableDiffusionXLPipeline
    pipe = object.__new__(Pipe)
    pipe.vae = VAEShim(post, rec)
    pipe.unet = UNetShim()
    pipe.denoise_encoder = standin_features
    pipe.scheduler = EulerShim()
    pipe.DDPM_scheduler = DDPMShim()
    pipe.image_processor = SimpleNamespace(preprocess=lambda imgs, height=None, width=None: torch.cat(imgs, 0),
                                           postprocess=lambda image, output_type="pil": image)
    pipe.vae_scale_factor = 8
    pipe.default_sample_size = 128
    pipe.watermark = None
    pipe.progress_bar = lambda total=None: _NullBar()
    pipe.maybe_free_model_hooks = lambda: None
    pipe.encode_prompt = lambda *a, **k: (pe, npe, ppe, nppe)
    torch.manual_seed(0)  # the reference's global-RNG randint (:1274) has no numeric effect
    image = Pipe.__call__(pipe, lr_img=img, prompt="a photo", negative_prompt="", num_inference_steps=steps,
                          guidance_scale=g, guidance_rescale=rescale, start_point=start, height=H, width=W,
                          overlap=0.5, target_size=target, latents=noise.clone(), output_type="pt",
                          return_dict=False)[0]
    latents = rec["z"] * pipe.vae.config.scaling_factor
    return latents, image


class _NullBar:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False

    def update(self, *a):
        pass


def main():
    import make_golden
    sys.meta_path.insert(0, make_golden._Finder())
    sys.path.insert(0, REF)
    mod = importlib.import_module("FaithDiff.pipelines.pipeline_FaithDiff_tlc")
    assert os.path.realpath(mod.__file__).startswith(REF), mod.__file__
    mod.torch = _TorchOnCPU()
    out = {}
    for k, case in enumerate(call_cases()):
        lat, img = reference_call(mod, case, 500 + 10 * k)
        out[f"{case[0]}_latents"] = lat.numpy()
        out[f"{case[0]}_image"] = img.numpy()
        print(case[0], tuple(lat.shape), float(lat.std()), tuple(img.shape))
    path = os.path.join(HERE, "call_golden.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main()
