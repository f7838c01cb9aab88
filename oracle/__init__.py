"""CPU fp32 oracle for the FaithDiff denoising hot path.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import anything under ``oracle/``; the
product path (``faithdiff-dev_amd/``) never does, and fails loudly when its HIP
library is missing instead of falling back here.

What it restates (reference = tpetkovich/FaithDiff-dev @ 2025-07-18):
  * ``unet.py``      SDXL ``UNet2DConditionModel`` + FaithDiff extras
                     (FaithDiff/models/unet_2d_condition_vae_extension.py:199-697)
                     and the diffusers 0.28 blocks it subclasses.
  * ``vae.py``       AutoencoderKL (sdxl-vae-fp16-fix) and the
                     FaithDiff ``Encoder`` (ext:39-196) incl. ``tiled_encode``.
  * ``schedulers.py`` EulerDiscreteScheduler / DDPMScheduler.add_noise (App. B.3).
  * ``tlc.py``       ``LocalAttention`` grids / gaussian weights / grids_inverse
                     (FaithDiff/pipelines/pipeline_FaithDiff_tlc.py:101-252).
  * ``pipeline.py``  the ``__call__`` denoise loop (pipeline:1008-1459) on
                     explicit, seeded inputs.

Pinning (see DESIGN.md "Parity"): the FaithDiff-owned pieces (TLC, the
information transformer, ControlNetConditioningEmbedding, rescale_noise_cfg,
colour fix) are pinned against golden vectors generated from the reference
itself (tests/golden/make_golden.py, stub-imported with diffusers absent).
The diffusers-owned blocks are pinned structurally only (exact parameter
counts and diffusers state-dict key names): **parity unpinned** for those
numerics, because diffusers 0.28 is absent from the image and the reference
has no tests.
"""
