"""SDXL text encoders on HIP (fdhip.clip) vs transformers' own CLIPTextModel /
CLIPTextModelWithProjection (the implementation diffusers calls in encode_prompt, pipeline:485-717), fp32 on the
host, same seeded random weights of the real architectures, same token ids (BOS, random body, EOS, padding as
each SDXL tokenizer pads: 49407 for tokenizer, 0 for tokenizer_2).

Bars: hidden_states[-2] (what SDXL keeps) and last_hidden_state rel-L2 <= 2e-2, pooled / text_embeds rel-L2 <=
2e-2 -- bf16 activations through 12 / 32 pre-LN layers (the reference itself runs these encoders in fp16)."""
import pytest
import torch

import parity  # records every measured value (tests/golden/parity.py)

pytestmark = pytest.mark.gpu


def rel(a, b):
    return parity.rel_l2(a.float(), b.float())


def make_ids(pad, seed=0):
    g = torch.Generator().manual_seed(seed)
    rows = []
    for n in (5, 40):  # short prompt (mostly padding) and a long one
        body = torch.randint(256, 49406, (n,), generator=g).tolist()
        r = [49406] + body + [49407]
        rows.append(r + [pad] * (77 - len(r)))
    return torch.tensor(rows)


@pytest.mark.parametrize("which", ["L", "G"])
def test_clip_text_encoder_matches_transformers(which):
    from transformers import CLIPTextConfig, CLIPTextModel, CLIPTextModelWithProjection
    from fdhip import arch
    from fdhip.clip import HipCLIPTextModel, random_clip
    cfg = arch.CLIP_L if which == "L" else arch.CLIP_G
    sd = random_clip(cfg, seed=5)
    tcfg = CLIPTextConfig(vocab_size=cfg["vocab"], hidden_size=cfg["D"], intermediate_size=cfg["inter"],
                          num_hidden_layers=cfg["layers"], num_attention_heads=cfg["heads"],
                          max_position_embeddings=cfg["max_pos"],
                          hidden_act="quick_gelu" if cfg["act"] == "quickgelu" else "gelu",
                          layer_norm_eps=1e-5, projection_dim=cfg["proj"] or 768, eos_token_id=2,
                          attn_implementation="eager")
    ref = (CLIPTextModelWithProjection if cfg["proj"] else CLIPTextModel)(tcfg).eval()
    # our keys are the reference's (transformers 4.x: "text_model." prefix); newer releases drop the prefix
    tf_keys = set(ref.state_dict())
    tsd = {(k if k in tf_keys else k[len("text_model."):]): v for k, v in sd.items()}
    missing, unexpected = ref.load_state_dict(tsd, strict=False)
    assert not unexpected and all("position_ids" in k for k in missing), (missing, unexpected)
    ids = make_ids(49407 if which == "L" else 0)
    with torch.no_grad():
        want = ref(ids, output_hidden_states=True)
    hip = HipCLIPTextModel(sd, cfg, "cuda", torch.bfloat16)
    got = hip.forward(ids)
    torch.cuda.synchronize()
    assert len(got["hidden_states"]) == len(want.hidden_states) == cfg["layers"] + 1
    r2 = rel(got["hidden_states"][-2].cpu(), want.hidden_states[-2])
    rl = rel(got["last_hidden_state"].cpu(), want.last_hidden_state)
    if cfg["proj"]:
        rp = rel(got["text_embeds"].cpu(), want.text_embeds)
    else:
        rp = rel(got["pooled"].cpu(), want.pooler_output)
    print(f"clip {which}: hidden[-2] rel={r2:.3e} last rel={rl:.3e} pooled/proj rel={rp:.3e}")
    assert r2 < 2e-2 and rl < 2e-2 and rp < 2e-2


def test_encode_prompt_dropin_shapes_and_negative():
    """encode_prompt through the drop-in encoders: (1, 77, 2048) context, (1, 1280) pooled, the "" negative prompt
    encoded (not zeroed, :622), deterministic."""
    from FaithDiff.models.clip_text import CLIPTextModel, CLIPTextModelWithProjection, FallbackCLIPTokenizer
    from FaithDiff.pipelines.pipeline_FaithDiff_tlc import FaithDiffStableDiffusionXLPipeline
    from fdhip import arch
    from fdhip.clip import random_clip
    vae = type("V", (), {"config": type("C", (), {"block_out_channels": (128, 256, 512, 512)})()})()
    pipe = FaithDiffStableDiffusionXLPipeline(
        vae=vae, denoise_encoder=None, text_encoder=CLIPTextModel(random_clip(arch.CLIP_L, 1)).to("cuda"),
        text_encoder_2=CLIPTextModelWithProjection(random_clip(arch.CLIP_G, 2)).to("cuda"),
        tokenizer=FallbackCLIPTokenizer(49407), tokenizer_2=FallbackCLIPTokenizer(0))
    pe, npe, ppe, nppe = pipe.encode_prompt("a photo of a red car, highly detailed", negative_prompt="")
    assert pe.shape == (1, 77, 2048) and npe.shape == (1, 77, 2048)
    assert ppe.shape == (1, 1280) and nppe.shape == (1, 1280)
    assert npe.abs().sum() > 0 and not torch.equal(pe, npe)
    pe2, _, _, _ = pipe.encode_prompt("a photo of a red car, highly detailed", negative_prompt="")
    assert torch.equal(pe, pe2)


def test_clip_graph_replay_is_bitwise():
    """The text encoder runs as a hipGraph (fdhip/graphs.py, min_uses=1: the first call of a shape runs eagerly once,
    then captures and replays): replays with other token ids give bitwise what the eager forward gives (both
    references built with the graph cache off), the EOS row picked on the device included."""
    from fdhip import arch
    from fdhip.clip import HipCLIPTextModel, random_clip
    cfg = arch.CLIP_G  # with the projection (text_embeds)
    sd = random_clip(cfg, seed=9)
    hip = HipCLIPTextModel(sd, cfg, "cuda", torch.bfloat16)
    ids = make_ids(0, seed=3)
    a, b = ids[:1], ids[1:]  # B = 1, as encode_prompt calls it: a short and a long prompt

    def snap(o):
        return [t.clone() for t in o["hidden_states"]] + [o["last_hidden_state"].clone(), o["pooled"].clone(),
                                                           o["text_embeds"].clone()]
    hip.graphs.enabled = False
    ref_b = snap(hip.forward(b))  # eager
    ref_a = snap(hip.forward(a))  # eager
    hip.graphs.enabled = True
    got_a = snap(hip.forward(a))  # first use: eager sizing run, capture, replay
    got_b = snap(hip.forward(b))  # replay
    got_a2 = snap(hip.forward(a))  # replay
    assert len(hip.graphs) == 1
    for x, y in zip(got_a, ref_a):
        assert torch.equal(x, y)
    for x, y in zip(got_b, ref_b):
        assert torch.equal(x, y)
    for x, y in zip(got_a2, ref_a):
        assert torch.equal(x, y)
    assert not torch.equal(got_a[-1], got_b[-1])
    # the fp32 surface (CLIPTextModel.__call__): outputs packed in the graph, one private copy per call
    for _ in range(3):  # eager, capture + replay, replay
        fa = hip.forward_f32(a)
        fb = hip.forward_f32(b)
        fa_l = list(fa["hidden_states"]) + [fa["last_hidden_state"], fa["pooled"], fa["text_embeds"]]
        fb_l = list(fb["hidden_states"]) + [fb["last_hidden_state"], fb["pooled"], fb["text_embeds"]]
        for x, y in zip(fa_l, ref_a):
            assert x.dtype == torch.float32 and torch.equal(x, y.float())
        for x, y in zip(fb_l, ref_b):
            assert torch.equal(x, y.float())


def test_clip_row_groups_are_bitwise_solo_passes():
    """forward(ids of two prompts, groups=2) -- encode_prompt's batched prompt + negative pass -- gives each prompt's
    rows bitwise as its own B = 1 forward (every GEMM planned on the per-group row count, ops.tile_groups)."""
    from fdhip import arch
    from fdhip.clip import HipCLIPTextModel, random_clip
    for cfg, pad in ((arch.CLIP_L, 49407), (arch.CLIP_G, 0)):
        hip = HipCLIPTextModel(random_clip(cfg, seed=4), cfg, "cuda", torch.bfloat16)
        ids = make_ids(pad, seed=6)
        both = hip.forward_f32(ids, groups=2)
        solo = [hip.forward_f32(ids[i:i + 1]) for i in range(2)]
        keys = ["last_hidden_state", "pooled"] + (["text_embeds"] if cfg["proj"] else [])
        for i in range(2):
            for k in keys:
                assert torch.equal(both[k][i:i + 1], solo[i][k]), (cfg["D"], k, i)
            for x, y in zip(both["hidden_states"], solo[i]["hidden_states"]):
                assert torch.equal(x[i:i + 1], y)
