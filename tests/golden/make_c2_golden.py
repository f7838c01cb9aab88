"""Generate the C2 headline-parity golden (BASELINE.json configs[1]): the fp32 CPU oracle pipeline at
1024x1024, one TLC tile, 20 Euler steps, CFG 5, start_point 'lr', on the seeded random-init weights that
``FaithDiff_pipeline('random-init', ..., seed=0, init_device='cpu')`` builds, with explicit prompt
embeddings, initial noise and VAE posterior draw (tests/golden/_det.py:c2_inputs).

Follows pipeline_FaithDiff_tlc.py:1187-1459 through oracle/pipeline.py:run_pipeline.  Writes
tests/golden/c2/{c2_golden.npz, c2_image.png}: the latent after steps 1, 5, 10, 15 and 20 (fp32), the
final decoded uint8 image, and the sha256 of the uint8 input image (the GPU test re-creates the input
from the same seed and checks the hash first).  Also writes tests/golden/c2/c2_eps_golden.npz: the oracle's step
input latent, the UNet's noise prediction (both CFG rows) and the guided one (after CFG, the eps the Euler step
consumes) at steps 1, 10, 19 and 20 --
the teacher-forced per-step eps pins of SURVEY 8(d) (tests/test_pipeline_gpu.py::test_c2_teacher_forced_eps).
Run here (CPU, ~8 min on 8 cores):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_c2_golden.py
"""
import hashlib
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
for p in (ROOT, os.path.join(ROOT, "faithdiff-dev_amd"), HERE):
    if p not in sys.path:
        sys.path.insert(0, p)

from _det import c2_inputs  # noqa: E402

KEEP_STEPS = (0, 4, 9, 14, 19)
EPS_STEPS = (0, 9, 18, 19)  # steps 1, 10, 19, 20: t = 951, 501, 51, 1 (sigma 11.03, 1.62, 0.23, 0.04)


def oracle_models(seed=0):
    """The oracle UNet / VAE / denoise encoder loaded with exactly the weights the product factory draws."""
    from FaithDiff.models.unet_2d_condition_vae_extension import RANDOM_INIT, AutoencoderKL, UNet2DConditionModel
    from oracle.unet import UNet2DConditionModel as RefUNet
    from oracle.vae import AutoencoderKL as RefVAE, DenoiseEncoder as RefEnc
    unet = UNet2DConditionModel.from_pretrained(RANDOM_INIT, subfolder="unet", variant="fp16", seed=seed)
    unet.load_additional_layers(weight_path=RANDOM_INIT, dtype=torch.float16)
    vae = AutoencoderKL.from_pretrained(RANDOM_INIT, seed=seed)
    ru, rv, re_ = RefUNet(), RefVAE(), RefEnc()
    ru.load_state_dict(unet._sd)
    rv.load_state_dict(vae._sd)
    re_.load_state_dict(unet.denoise_encoder._sd)
    for m in (ru, rv, re_):
        m.eval()
    return ru, rv, re_


def main():
    from oracle.pipeline import run_pipeline
    torch.set_num_threads(int(os.environ.get("THREADS", os.cpu_count() or 8)))
    c = c2_inputs()
    img_u8 = np.asarray(c["img"], dtype=np.uint8)
    sha = hashlib.sha256(img_u8.tobytes()).hexdigest()
    x = torch.from_numpy(img_u8.astype(np.float32) / 255.0 * 2 - 1).permute(2, 0, 1)[None].contiguous()
    ru, rv, re_ = oracle_models(c["seed"])
    kept = {}

    def cb(i, lat):
        print(f"step {i + 1}/{c['steps']}  {time.strftime('%H:%M:%S')}", flush=True)
        if i in KEEP_STEPS:
            kept[f"lat_step{i + 1}"] = lat.float().numpy().copy()

    eps_kept = {}

    def ecb(i, n, x, eps, eps_raw):
        if i in EPS_STEPS:
            eps_kept[f"x_step{i + 1}"] = x.float().numpy().copy()
            eps_kept[f"eps_step{i + 1}"] = eps.float().numpy().copy()
            eps_kept[f"unet_eps_step{i + 1}"] = eps_raw.float().numpy().copy()

    t0 = time.time()
    ref = run_pipeline(ru, rv, re_, x, c["pe"], c["npe"], c["ppe"], c["nppe"], c["noise"], c["post"],
                       num_inference_steps=c["steps"], guidance_scale=c["guidance"], overlap=c["overlap"],
                       target_size=c["target"], original_size=(c["H"], c["W"]), start_point="lr",
                       step_callback=cb, eps_callback=ecb)
    img = ((ref["image"][0].permute(1, 2, 0) / 2 + 0.5).clamp(0, 1) * 255).round().to(torch.uint8).numpy()
    out = os.path.join(HERE, "c2")
    os.makedirs(out, exist_ok=True)
    np.savez_compressed(os.path.join(out, "c2_golden.npz"), final=ref["latents"].numpy(), input_sha256=np.array(sha),
                        **kept)
    np.savez_compressed(os.path.join(out, "c2_eps_golden.npz"), input_sha256=np.array(sha), **eps_kept)
    from PIL import Image
    Image.fromarray(img).save(os.path.join(out, "c2_image.png"))
    print(f"done in {time.time() - t0:.0f} s; input sha256 {sha}")


if __name__ == "__main__":
    main()
