"""fp64/fp32 restatement of the diffusers 0.28 schedulers the hot path uses.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).  SURVEY Appendix B.3:
  * betas 'scaled_linear' 0.00085 -> 0.012 over 1000 train steps, acp = cumprod(1 - beta)
  * EulerDiscreteScheduler, timestep_spacing 'leading', steps_offset 1, final sigma 0,
    init_noise_sigma = sqrt(sigma_max^2 + 1); scale_model_input x / sqrt(sigma^2 + 1);
    step (s_churn = 0 => gamma = 0): x' = x + ((x - (x - sigma*eps)) / sigma) * (sigma_next - sigma), in fp32.
  * DDPMScheduler.add_noise(x0, n, t) = sqrt(acp[t]) x0 + sqrt(1 - acp[t]) n  (pipeline:1276).
"""
import numpy as np
import torch


def alphas_cumprod(n_train=1000, beta_start=0.00085, beta_end=0.012):
    betas = torch.linspace(beta_start ** 0.5, beta_end ** 0.5, n_train, dtype=torch.float32) ** 2
    return torch.cumprod(1.0 - betas, dim=0)


def euler_schedule(num_inference_steps, n_train=1000, steps_offset=1):
    """Returns (timesteps float32 [n], sigmas float32 [n+1], init_noise_sigma float)."""
    acp = alphas_cumprod(n_train).numpy()
    step_ratio = n_train // num_inference_steps
    ts = (np.arange(0, num_inference_steps) * step_ratio).round()[::-1].copy().astype(np.float32)
    ts += steps_offset
    sig = np.array(((1 - acp) / acp) ** 0.5)
    sig = np.interp(ts, np.arange(0, len(sig)), sig)
    sig = np.concatenate([sig, [0.0]]).astype(np.float32)
    init = float((sig.max() ** 2 + 1) ** 0.5)
    return torch.from_numpy(ts), torch.from_numpy(sig), init


def euler_scale(x, sigma):
    return x / ((sigma ** 2 + 1) ** 0.5)


def euler_step(eps, x, sigma, sigma_next):
    x = x.float()
    pred = x - sigma * eps.float()
    d = (x - pred) / sigma
    return x + d * (sigma_next - sigma)


def ddpm_add_noise(x0, noise, t):
    acp = alphas_cumprod()
    a = acp[t] ** 0.5
    b = (1 - acp[t]) ** 0.5
    return a * x0 + b * noise
