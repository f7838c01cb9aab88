"""fp32 CPU restatement of ``FaithDiffStableDiffusionXLPipeline.__call__`` (the TLC denoise loop).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).
Follows FaithDiff/pipelines/pipeline_FaithDiff_tlc.py:1008-1459 on explicit seeded inputs
(SURVEY 8(d)): the reference draws its noise from a CUDA generator / the global CUDA RNG
(:1261-1276), which no CPU run can reproduce, so the noise tensors are arguments here.

Per step i (:1324-1409): re-grid the blended latent (i>=1), then per tile: CFG duplicate,
scale_model_input, add_time_ids = [orig_h, orig_w, tile_i, tile_j, tgt_h, tgt_w] (latent-grid
offsets, App. A quirk 2), UNet, CFG combine (+ optional rescale_noise_cfg), Euler step; then the
gaussian-weighted fp32 blend (grids_inverse).  Finally latents / 0.13025 -> VAE decode.
"""
import torch

from . import schedulers as S
from .tlc import LocalAttention


def rescale_noise_cfg(noise_cfg, noise_pred_text, guidance_rescale=0.0):  # pipeline:286-305
    std_text = noise_pred_text.std(dim=list(range(1, noise_pred_text.ndim)), keepdim=True)
    std_cfg = noise_cfg.std(dim=list(range(1, noise_cfg.ndim)), keepdim=True)
    rescaled = noise_cfg * (std_text / std_cfg)
    return guidance_rescale * rescaled + (1 - guidance_rescale) * noise_cfg


@torch.no_grad()
def run_pipeline(unet, vae, denoise_encoder, lr_img, prompt_embeds, negative_prompt_embeds,
                 pooled_prompt_embeds, negative_pooled_prompt_embeds, noise, posterior_eps,
                 num_inference_steps=20, guidance_scale=5.0, overlap=0.5, target_size=None,
                 original_size=None, start_point="lr", guidance_rescale=0.0, add_sample=True,
                 decode=True, step_callback=None, eps_callback=None):
    """Returns dict(latents=final fp32 latent (1,4,h,w), image=decoded (1,3,H,W) or None).
    ``eps_callback(i, n, x, eps, eps_raw)`` sees every tile's step input ``x`` (before scale_model_input), the UNet's
    own noise prediction ``eps_raw`` (CFG rows [uncond, cond]) and the guided ``eps`` the Euler step consumes (the
    teacher-forced per-step pins)."""
    _, _, H, W = lr_img.shape
    original_size = original_size or (H, W)
    target_size = target_size or (H, W)
    tlc_lat = LocalAttention((target_size[0] // 8, target_size[1] // 8), overlap)
    tlc_img = LocalAttention((target_size[0] // 8, target_size[1] // 8), overlap)

    ts, sig, init_sigma = S.euler_schedule(num_inference_steps)
    image_latents = tlc_img.grids(denoise_encoder(lr_img))
    latents = noise * init_sigma
    if start_point == "lr":
        z = vae.encode_sample(lr_img, posterior_eps) * vae.scaling_factor
        latents = S.ddpm_add_noise(z[0:1], latents, 999)
    latents = tlc_lat.grids(latents)

    ctx = torch.cat([negative_prompt_embeds, prompt_embeds], 0)
    text = torch.cat([negative_pooled_prompt_embeds, pooled_prompt_embeds], 0)
    do_cfg = guidance_scale > 1
    for i, t in enumerate(ts):
        if i >= 1:
            latents = tlc_lat.grids(latents)
        sigma, sigma_next = float(sig[i]), float(sig[i + 1])
        outs = []
        for n in range(latents.shape[0]):
            x = latents[n:n + 1]
            c = image_latents[n:n + 1]
            xin = torch.cat([x] * 2) if do_cfg else x
            cin = torch.cat([c] * 2) if do_cfg else c
            xin = S.euler_scale(xin, sigma)
            pi, pj = tlc_lat.idxes[n]["i"], tlc_lat.idxes[n]["j"]
            tid = torch.tensor([[original_size[0], original_size[1], pi, pj, target_size[0], target_size[1]]],
                               dtype=torch.float32).repeat(xin.shape[0], 1)
            eps = unet(xin, t, ctx if do_cfg else ctx[1:], {"text_embeds": text if do_cfg else text[1:],
                                                              "time_ids": tid}, input_embedding=cin,
                       add_sample=add_sample)
            eps_raw = eps
            if do_cfg:
                u, c_ = eps.chunk(2)
                eps = u + guidance_scale * (c_ - u)
                if guidance_rescale > 0.0:
                    eps = rescale_noise_cfg(eps, c_, guidance_rescale)
            if eps_callback is not None:
                eps_callback(i, n, x, eps, eps_raw)
            outs.append(S.euler_step(eps, x, sigma, sigma_next))
        latents = tlc_lat.grids_inverse(torch.cat(outs, 0))
        if step_callback is not None:
            step_callback(i, latents)
    image = vae.decode(latents / vae.scaling_factor) if decode else None
    return {"latents": latents, "image": image}
