"""Pin the FaithDiff-owned UNet code: run the reference's own ``UNet2DConditionModel.forward`` (ext:480-697),
``Encoder.encode`` (ext:122-148) and the prefix-split ``load_state_dict`` (ext:444-478) on CPU fp32 and record their
outputs (tests/golden/unet_golden.npz, tests/golden/unet_lsd_golden.json).

Run in the build container only (the reference is not on the GPU box):
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_unet_golden.py

The reference module is stub-imported as in make_golden.py (diffusers / cv2 / peft / torchvision absent).  Its methods
are called unbound on a probe object (a subclass of the reference's class, created without ``__init__``) whose
submodules are:
  * the extras built by the reference's OWN ``init_information_transformer_layes`` /
    ``init_ControlNetConditioningEmbedding`` / ``init_extra_weights`` (ext:389-403: ResidualAttentionBlock,
    ControlNetConditioningEmbedding, zero-init spatial_ch_projs, empty agg_net) and loaded by the reference's own
    ``load_state_dict``;
  * the diffusers-owned core (conv_in, down/mid/up blocks, conv_norm_out) from the oracle (oracle/unet.py), wrapped
    in adapters with diffusers 0.28's call signatures (``hidden_states=``, ``res_hidden_states_tuple=``,
    ``upsample_size=`` ...).  ``super().load_state_dict(core, strict=False)`` (ext:474) lands on the oracle core.
What is pinned: the time / aug embedding sum, conv_in, the extras injection (ext:571-579, add_sample), the skip
bookkeeping (ext:611-684), the forward_upsample_size path for latents not divisible by 4 (ext:522-529, 665-666), the
output head, the Encoder trunk order, and load_state_dict's routing (which prefixes go where, which cases raise).
The diffusers block internals stay the oracle's restatement (parity unpinned: diffusers is absent).
Only inputs and outputs are written; no reference source is copied.
"""
import importlib
import json
import os
import sys
import types
from types import SimpleNamespace

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
for p in (HERE, ROOT, os.path.join(ROOT, "faithdiff-dev_amd")):
    sys.path.insert(0, p)
from _det import UNET_WEIGHT_SEED, det_tensor, lsd_cases, unet_golden_cases, unet_inputs  # noqa: E402
from fdhip import arch  # noqa: E402  (host-side shapes / seeded init only)
from oracle import unet as O  # noqa: E402
from oracle.vae import DenoiseEncoder  # noqa: E402

# the reference's own ``FaithDiff`` package must win the name, not the product's
for _m in [m for m in sys.modules if m == "FaithDiff" or m.startswith("FaithDiff.")]:
    del sys.modules[_m]
sys.path.remove(os.path.join(ROOT, "faithdiff-dev_amd"))


# ---------------------------------------------------------------- diffusers-0.28 call-signature adapters (restated)
class _Down:
    """DownBlock2D / CrossAttnDownBlock2D: forward(hidden_states, temb, encoder_hidden_states, ...) ->
    (hidden_states, output_states) with one output per resnet (+ the downsampler's)."""

    def __init__(self, blk):
        self.blk = blk
        self.resnets = blk.resnets
        self.has_cross_attention = blk.attentions is not None

    def __call__(self, hidden_states, temb=None, encoder_hidden_states=None, attention_mask=None,
                 cross_attention_kwargs=None, encoder_attention_mask=None, additional_residuals=None):
        assert attention_mask is None and encoder_attention_mask is None and additional_residuals is None
        x, outs = self.blk(hidden_states, temb, encoder_hidden_states)
        return x, tuple(outs)


class _Mid:
    has_cross_attention = True

    def __init__(self, blk):
        self.blk = blk

    def __call__(self, hidden_states, temb=None, encoder_hidden_states=None, attention_mask=None,
                 cross_attention_kwargs=None, encoder_attention_mask=None):
        return self.blk(hidden_states, temb, encoder_hidden_states)


class _Up:
    """UpBlock2D / CrossAttnUpBlock2D: each resnet takes res_hidden_states_tuple[-1] (then drops it), concatenated
    on channels; the upsampler gets ``upsample_size`` (nearest to that size, else x2)."""

    def __init__(self, blk):
        self.blk = blk
        self.resnets = blk.resnets
        self.has_cross_attention = blk.attentions is not None

    def __call__(self, hidden_states, temb=None, res_hidden_states_tuple=None, encoder_hidden_states=None,
                 cross_attention_kwargs=None, upsample_size=None, attention_mask=None, encoder_attention_mask=None):
        x = hidden_states
        res = tuple(res_hidden_states_tuple)
        for i, r in enumerate(self.blk.resnets):
            x = torch.cat([x, res[-1]], dim=1)
            res = res[:-1]
            x = r(x, temb)
            if self.blk.attentions is not None:
                x = self.blk.attentions[i](x, encoder_hidden_states)
        if self.blk.upsamplers is not None:
            x = self.blk.upsamplers[0](x, upsample_size)
        return x


class _CoreLoader:
    """What ``super().load_state_dict(core_dict, strict=False)`` (ext:474) resolves to on the probe: the oracle core."""

    def load_state_dict(self, state_dict, strict=True):
        self.core_keys = sorted(state_dict)
        return self.core.load_state_dict(state_dict, strict=strict)


def _install_core(probe, core):
    """diffusers UNet2DConditionModel attributes the reference forward reads (ext:522-690), on the oracle core."""
    probe.core = core
    probe.num_upsamplers = 2
    probe.config = SimpleNamespace(center_input_sample=False, class_embeddings_concat=False,
                                   addition_embed_type="text_time")
    probe.conv_in = core.conv_in
    probe.time_embed_act = None
    probe.down_blocks = [_Down(b) for b in core.down_blocks]
    probe.mid_block = _Mid(core.mid_block)
    probe.up_blocks = [_Up(b) for b in core.up_blocks]
    probe.conv_norm_out = core.conv_norm_out
    probe.conv_act = nn.SiLU()
    probe.conv_out = core.conv_out

    def get_time_embed(sample, timestep):  # diffusers get_time_embed: scalar -> [B], Timesteps(320, flip, 0)
        t = timestep if torch.is_tensor(timestep) else torch.tensor([timestep], dtype=torch.float32)
        t = t.reshape(-1).expand(sample.shape[0])
        return O.timestep_embedding(t, 320).to(sample.dtype)

    def get_aug_embed(emb, encoder_hidden_states, added_cond_kwargs):  # addition_embed_type 'text_time'
        text = added_cond_kwargs["text_embeds"]
        te = O.timestep_embedding(added_cond_kwargs["time_ids"].flatten(), 256).reshape(text.shape[0], -1)
        return core.add_embedding(torch.cat([text, te], dim=-1).to(emb.dtype))

    probe.get_time_embed = get_time_embed
    probe.time_embedding = lambda t_emb, timestep_cond=None: core.time_embedding(t_emb)
    probe.get_class_embed = lambda sample, class_labels: None
    probe.get_aug_embed = get_aug_embed
    probe.process_encoder_hidden_states = lambda encoder_hidden_states, added_cond_kwargs: encoder_hidden_states


def make_probe(ext, core, with_encoder=True):
    Ref = ext.UNet2DConditionModel
    Probe = type("Probe", (Ref, _CoreLoader), {})
    probe = object.__new__(Probe)
    _install_core(probe, core)
    probe.denoise_encoder = DenoiseEncoder() if with_encoder else None
    probe.information_transformer_layes = probe.condition_embedding = probe.agg_net = probe.spatial_ch_projs = None
    Ref.init_information_transformer_layes(probe)  # ext:393-399
    Ref.init_ControlNetConditioningEmbedding(probe, 512)  # ext:400-401
    Ref.init_extra_weights(probe)  # ext:402-403
    return probe


def _group_state(probe):
    out = {}
    for name in ("denoise_encoder", "information_transformer_layes", "condition_embedding", "agg_net",
                 "spatial_ch_projs"):
        m = getattr(probe, name)
        if m is not None:
            for k, v in m.state_dict().items():
                out[f"{name}.{k}"] = v
    for k, v in probe.core.state_dict().items():
        out[k] = v
    return out


def main():
    import make_golden
    sys.meta_path.insert(0, make_golden._Finder())
    sys.path.insert(0, REF)
    ext = importlib.import_module("FaithDiff.models.unet_2d_condition_vae_extension")
    assert os.path.realpath(ext.__file__).startswith(REF), ext.__file__
    torch.set_grad_enabled(False)

    # ---- 1. load_state_dict routing (ext:444-478) on a tiny core stand-in (what is pinned is the prefix split)
    ext_shapes = {k: v for k, v in arch.unet_param_shapes(True).items()
                  if k.startswith(("information_transformer_layes.", "condition_embedding.", "spatial_ch_projs."))}
    den_shapes = arch.encoder_param_shapes("denoise_encoder.", with_out=False)
    extras = arch.random_init({**ext_shapes, **den_shapes}, seed=8)
    tiny = nn.Module()
    tiny.conv_in = nn.Conv2d(4, 320, 3, padding=1)
    lsd = {}
    for name, sd, strict in lsd_cases(extras, "conv_in.weight", (320, 4, 3, 3)):
        probe = object.__new__(type("Probe", (ext.UNet2DConditionModel, _CoreLoader), {}))
        probe.core = tiny
        for a in ("denoise_encoder", "information_transformer_layes", "condition_embedding", "agg_net",
                  "spatial_ch_projs"):
            setattr(probe, a, None)
        probe.denoise_encoder = DenoiseEncoder()
        ext.UNet2DConditionModel.init_information_transformer_layes(probe)
        ext.UNet2DConditionModel.init_ControlNetConditioningEmbedding(probe, 512)
        ext.UNet2DConditionModel.init_extra_weights(probe)
        with torch.no_grad():
            for m in (probe.denoise_encoder, probe.information_transformer_layes, probe.condition_embedding,
                      probe.spatial_ch_projs, tiny):
                for p in m.parameters():
                    p.fill_(-123.0)
        try:
            probe.load_state_dict(sd, strict=strict)
            raised = None
        except Exception as e:  # noqa: BLE001 -- the pinned outcome is "raises"
            raised = type(e).__name__
        state = _group_state(probe)
        loaded = sorted(k for k, v in sd.items() if k in state and state[k].shape == v.shape
                        and torch.equal(state[k], v.to(state[k].dtype)))
        lsd[name] = {"strict": strict, "raised": raised, "n_keys": len(sd), "loaded": loaded}
        print("lsd", name, strict, raised, len(loaded), "/", len(sd))
    with open(os.path.join(HERE, "unet_lsd_golden.json"), "w") as f:
        json.dump(lsd, f, indent=0, sort_keys=True)

    # ---- 2. Encoder.encode (ext:122-148) on the oracle trunk
    den = DenoiseEncoder().eval()
    den.load_state_dict({k[len("denoise_encoder."):]: v for k, v in extras.items() if k.startswith("denoise_encoder.")})
    ns = SimpleNamespace(conv_in=den.conv_in, down_blocks=den.down_blocks, mid_block=den.mid_block, training=False,
                         gradient_checkpointing=False)
    out = {}
    xe = det_tensor((1, 3, 72, 56), 5101, 0.7)
    out["encode_72x56"] = ext.Encoder.encode(ns, xe).numpy()
    print("encode", out["encode_72x56"].shape)

    # ---- 3. UNet forward (ext:480-697): the full SDXL architecture, the GPU parity tests' seeded weights
    sd = arch.random_init(arch.unet_param_shapes(), seed=UNET_WEIGHT_SEED)
    sd.update(arch.random_init(den_shapes, seed=UNET_WEIGHT_SEED + 1))
    core = O.UNet2DConditionModel(with_extras=False).eval()
    probe = make_probe(ext, core)
    probe.load_state_dict(sd, strict=True)  # the reference's own prefix split fills the core AND the extras
    for a in ("information_transformer_layes", "condition_embedding", "spatial_ch_projs"):
        getattr(probe, a).eval()
    del sd
    for name, h, w, ntiles, t, add_sample, with_emb in unet_golden_cases():
        B, x, cond, ctx, text, tids = unet_inputs(h, w, ntiles)
        outs = []
        for i in range(0, B, 2):  # one forward per tile (the information transformer attends over the CFG pair)
            s = slice(i, i + 2)
            outs.append(ext.UNet2DConditionModel.forward(
                probe, x[s], t, ctx, added_cond_kwargs={"text_embeds": text[s], "time_ids": tids[s]},
                input_embedding=cond[s] if with_emb else None, add_sample=add_sample, return_dict=False)[0])
        y = torch.cat(outs, 0)
        out[f"unet_{name}"] = y.numpy()
        print("unet", name, tuple(y.shape), float(y.std()))
    path = os.path.join(HERE, "unet_golden.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main()
