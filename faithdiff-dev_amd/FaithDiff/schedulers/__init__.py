"""EulerDiscreteScheduler / DDPMScheduler (diffusers 0.28 semantics).

Only the host-side schedule math lives here (timesteps, sigmas, coefficients: a few dozen scalars per
call, computed in numpy as diffusers does).  The per-element work -- scale_model_input, the Euler
update and DDPM add_noise -- runs fused in HIP kernels (fd_tlc_scale_input, fd_tlc_cfg_euler_step,
fd_vae_sample_add_noise).  Scheduler state is per call, so the reference's per-tile
``scheduler.__dict__`` save/restore (pipeline_FaithDiff_tlc.py:1282,1331,1375) has no equivalent:
every tile sees the same step index, which is all that bookkeeping achieved.
"""
import numpy as np


class _Config(dict):
    __getattr__ = dict.__getitem__


def _alphas_cumprod(n=1000, beta_start=0.00085, beta_end=0.012):
    # diffusers computes the 'scaled_linear' betas and their cumprod with torch (fp32 on CPU); numpy's
    # linspace/cumprod round differently in the last ulp, so follow torch exactly.
    import torch
    betas = torch.linspace(beta_start ** 0.5, beta_end ** 0.5, n, dtype=torch.float32) ** 2
    return torch.cumprod(1.0 - betas, dim=0).numpy()


class EulerDiscreteScheduler:
    order = 1

    def __init__(self, num_train_timesteps=1000, beta_start=0.00085, beta_end=0.012, steps_offset=1,
                 timestep_spacing="leading", prediction_type="epsilon"):
        if prediction_type != "epsilon":
            raise ValueError("only prediction_type='epsilon' is supported (SDXL)")
        self.config = _Config(num_train_timesteps=num_train_timesteps, beta_start=beta_start, beta_end=beta_end,
                              steps_offset=steps_offset, timestep_spacing=timestep_spacing,
                              prediction_type=prediction_type)
        self.alphas_cumprod = _alphas_cumprod(num_train_timesteps, beta_start, beta_end)
        self.timesteps = None
        self.sigmas = None
        self.num_inference_steps = None

    def set_timesteps(self, num_inference_steps=None, device=None, timesteps=None):
        n_train = self.config.num_train_timesteps
        if timesteps is not None:
            ts = np.array(timesteps, dtype=np.float32)
            num_inference_steps = len(ts)
        elif self.config.timestep_spacing == "leading":
            step_ratio = n_train // num_inference_steps
            ts = (np.arange(0, num_inference_steps) * step_ratio).round()[::-1].copy().astype(np.float32)
            ts += self.config.steps_offset
        elif self.config.timestep_spacing == "trailing":
            step_ratio = n_train / num_inference_steps
            ts = np.arange(n_train, 0, -step_ratio).round().copy().astype(np.float32) - 1
        elif self.config.timestep_spacing == "linspace":
            ts = np.linspace(0, n_train - 1, num_inference_steps, dtype=np.float64)[::-1].copy().astype(np.float32)
        else:
            raise ValueError(f"unknown timestep_spacing {self.config.timestep_spacing}")
        acp = self.alphas_cumprod
        sig = np.array(((1 - acp) / acp) ** 0.5)
        sig = np.interp(ts, np.arange(0, len(sig)), sig)
        self.sigmas = np.concatenate([sig, [0.0]]).astype(np.float32)
        self.timesteps = ts
        self.num_inference_steps = num_inference_steps

    @property
    def init_noise_sigma(self):
        mx = float(self.sigmas.max())
        if self.config.timestep_spacing in ("linspace", "trailing"):
            return mx
        return (mx ** 2 + 1) ** 0.5


class DDPMScheduler:
    def __init__(self, num_train_timesteps=1000, beta_start=0.00085, beta_end=0.012):
        self.config = _Config(num_train_timesteps=num_train_timesteps, beta_start=beta_start, beta_end=beta_end)
        self.alphas_cumprod = _alphas_cumprod(num_train_timesteps, beta_start, beta_end)

    def add_noise_coefficients(self, t):
        """add_noise(x0, n, t) = a * x0 + b * n  (pipeline:1276; applied on device by the fused kernel)."""
        a = float(self.alphas_cumprod[int(t)]) ** 0.5
        b = float(1.0 - self.alphas_cumprod[int(t)]) ** 0.5
        return a, b
