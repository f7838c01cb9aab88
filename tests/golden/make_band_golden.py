"""Generate the band.png golden: the reference's own in-tree input (examples/band.png, copied as data to
tests/golden/band/band.png) through test_wo_llava.py's preprocessing (:65,78-82; upscale 1) and the fp32 CPU
oracle pipeline (oracle/pipeline.py:run_pipeline, following pipeline_FaithDiff_tlc.py:1187-1459): 1080x784 padded
input, 135x98 latent, two ragged 128x98 TLC tiles (target 1024), 4 Euler steps, CFG 5, start_point 'lr', on the
seeded random-init weights of ``FaithDiff_pipeline('random-init', ..., seed=0)``, with seeded prompt embeddings /
noise / posterior draw (tests/golden/_det.py:band_inputs; the LLaVA caption is OUT of scope).

Writes tests/golden/band/{band_golden.npz, band_image.png}: the latent after every step (fp32), the final decoded
uint8 image (1080x784, before the crop), the TLC tile count and the sha256 of the padded uint8 input (the GPU
test, tests/test_pipeline_gpu.py::test_band_matches_golden, re-creates the input and checks the hash first).
Run here (CPU, ~6 min on 8 cores):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_band_golden.py
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

from _det import band_inputs  # noqa: E402
from make_c2_golden import oracle_models  # noqa: E402


def main():
    from oracle.pipeline import run_pipeline
    from oracle.tlc import LocalAttention
    torch.set_num_threads(int(os.environ.get("THREADS", os.cpu_count() or 8)))
    c = band_inputs(1)
    img_u8 = np.asarray(c["img"], dtype=np.uint8)
    # check_image_size is cv2.copyMakeBorder(BORDER_REPLICATE) in the reference (utils/image_process.py:7-21)
    src = np.asarray(c["image"], dtype=np.uint8)
    want = np.pad(src, ((0, c["H"] - c["h0"]), (0, c["W"] - c["w0"]), (0, 0)), mode="edge")
    assert img_u8.shape == (784, 1080, 3) and np.array_equal(img_u8, want)
    sha = hashlib.sha256(img_u8.tobytes()).hexdigest()
    ntiles = LocalAttention((c["target"][0] // 8, c["target"][1] // 8), c["overlap"]).grids(
        torch.zeros(1, 1, c["H"] // 8, c["W"] // 8)).shape[0]
    x = torch.from_numpy(img_u8.astype(np.float32) / 255.0 * 2 - 1).permute(2, 0, 1)[None].contiguous()
    ru, rv, re_ = oracle_models(c["seed"])
    kept = {}

    def cb(i, lat):
        print(f"step {i + 1}/{c['steps']}  {time.strftime('%H:%M:%S')}", flush=True)
        kept[f"lat_step{i + 1}"] = lat.float().numpy().copy()

    t0 = time.time()
    ref = run_pipeline(ru, rv, re_, x, c["pe"], c["npe"], c["ppe"], c["nppe"], c["noise"], c["post"],
                       num_inference_steps=c["steps"], guidance_scale=c["guidance"], overlap=c["overlap"],
                       target_size=c["target"], original_size=(c["H"], c["W"]), start_point="lr",
                       step_callback=cb)
    img = ((ref["image"][0].permute(1, 2, 0) / 2 + 0.5).clamp(0, 1) * 255).round().to(torch.uint8).numpy()
    out = os.path.join(HERE, "band")
    os.makedirs(out, exist_ok=True)
    np.savez_compressed(os.path.join(out, "band_golden.npz"), final=ref["latents"].numpy(),
                        input_sha256=np.array(sha), ntiles=np.array(ntiles), **kept)
    from PIL import Image
    Image.fromarray(img).save(os.path.join(out, "band_image.png"))
    print(f"done in {time.time() - t0:.0f} s; {ntiles} tiles; input sha256 {sha}")


if __name__ == "__main__":
    main()
