"""Pin the oracle's UNet forward / Encoder trunk and the product's load_state_dict routing against the reference's
own UNet2DConditionModel.forward (ext:480-697), Encoder.encode (ext:122-148) and load_state_dict (ext:444-478), run
on the oracle's blocks by tests/golden/make_unet_golden.py (unet_golden.npz, unet_lsd_golden.json).

Bars: the oracle restatement vs the reference's own orchestration on the same fp32 blocks, rel-L2 <= 1e-5 (measured
0: the same arithmetic in the same order); load_state_dict: the product raises exactly where the reference raises,
and every key the reference loads is loaded with the same value."""
import json
import os

import numpy as np
import pytest
import torch

from _det import UNET_WEIGHT_SEED, det_tensor, lsd_cases, unet_golden_cases, unet_inputs

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def ugold():
    return np.load(os.path.join(HERE, "unet_golden.npz"))


def _extras():
    from fdhip import arch
    ext_shapes = {k: v for k, v in arch.unet_param_shapes(True).items()
                  if k.startswith(("information_transformer_layes.", "condition_embedding.", "spatial_ch_projs."))}
    den_shapes = arch.encoder_param_shapes("denoise_encoder.", with_out=False)
    return arch.random_init({**ext_shapes, **den_shapes}, seed=8), den_shapes


def _rel(a, b):
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def test_oracle_unet_forward_matches_reference_forward(ugold):
    """oracle/unet.py's forward (extras injection, skip bookkeeping, forward_upsample_size at 62x46, add_sample=False,
    no input_embedding) against the reference's forward on the same weights and inputs."""
    import parity
    from fdhip import arch
    from oracle.unet import UNet2DConditionModel
    ref = UNet2DConditionModel()
    ref.load_state_dict(arch.random_init(arch.unet_param_shapes(), seed=UNET_WEIGHT_SEED))
    ref.eval()
    with torch.no_grad():
        for name, h, w, ntiles, t, add_sample, with_emb in unet_golden_cases():
            B, x, cond, ctx, text, tids = unet_inputs(h, w, ntiles)
            outs = []
            for i in range(0, B, 2):
                s = slice(i, i + 2)
                outs.append(ref(x[s], t, ctx, {"text_embeds": text[s], "time_ids": tids[s]},
                                input_embedding=cond[s] if with_emb else None, add_sample=add_sample))
            got = torch.cat(outs, 0).numpy()
            rel = _rel(got, ugold[f"unet_{name}"])
            parity.record(f"oracle_vs_reference_forward_{name}", rel, 1e-5)
            assert rel <= 1e-5, (name, rel)


def test_oracle_encoder_trunk_matches_reference_encode(ugold):
    from oracle.vae import DenoiseEncoder
    extras, _ = _extras()
    den = DenoiseEncoder().eval()
    den.load_state_dict({k[len("denoise_encoder."):]: v for k, v in extras.items() if k.startswith("denoise_encoder.")})
    with torch.no_grad():
        got = den.encode(det_tensor((1, 3, 72, 56), 5101, 0.7)).numpy()
    assert _rel(got, ugold["encode_72x56"]) <= 1e-6


def test_product_load_state_dict_routing_matches_reference():
    """The product's UNet2DConditionModel.load_state_dict (FaithDiff/models/unet_2d_condition_vae_extension.py) on
    the reference's cases: core non-strict, each present extras group strict, agg_net (an empty ModuleList in the
    reference) refusing keys under strict, shape mismatches raising regardless of strict."""
    from FaithDiff.models.unet_2d_condition_vae_extension import UNet2DConditionModel
    with open(os.path.join(HERE, "unet_lsd_golden.json")) as f:
        gold = json.load(f)
    extras, _ = _extras()
    for name, sd, strict in lsd_cases(extras, "conv_in.weight", (320, 4, 3, 3)):
        g = gold[name]
        assert g["strict"] == strict and g["n_keys"] == len(sd)
        m = UNet2DConditionModel({}, seed=0)
        try:
            m.load_state_dict(sd, strict=strict)
            raised = None
        except RuntimeError as e:
            raised = type(e).__name__
        assert (raised is None) == (g["raised"] is None), (name, raised, g["raised"])
        if raised is None:
            held = dict(m._sd)
            if m.denoise_encoder is not None:
                held.update({"denoise_encoder." + k: v for k, v in m.denoise_encoder._sd.items()})
            for k in g["loaded"]:
                assert k in held and torch.equal(held[k], sd[k]), (name, k)
