"""Full UNet forward (HIP bf16) vs the fp32 CPU oracle on identical seeded random-init weights.

Tolerance: bf16 storage of every activation through ~1000 fused ops gives a relative L2 error of a
few 1e-3 per layer that does not compound much (residual stream).  Measured rel-L2 8.3e-3 .. 8.7e-3 and
cosine 0.99996 (round 1); the bar is about 2x that: rel-L2 <= 1.5e-2 and cosine >= 0.9999 on eps, at C2's tile
shape (B=2, 128x128 latent), a small tile and a ragged two-tile batch.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

_CACHE = {}


def unet_pair():
    if "pair" not in _CACHE:
        from fdhip import arch
        from fdhip.unet import HipUNet
        from oracle.unet import UNet2DConditionModel
        sd = arch.random_init(arch.unet_param_shapes(), seed=1)
        ref = UNet2DConditionModel()
        ref.load_state_dict(sd)
        ref.eval()
        hip = HipUNet(sd, "cuda", torch.bfloat16)
        del sd
        _CACHE["pair"] = (ref, hip)
    return _CACHE["pair"]


def hip_fp16():
    """The same seeded UNet computing in fp16, the reference's own UNet dtype (reference create_FaithDiff_model.py:21-22)."""
    if "hip16" not in _CACHE:
        from fdhip import arch
        from fdhip.unet import HipUNet
        sd = arch.random_init(arch.unet_param_shapes(), seed=1)
        _CACHE["hip16"] = HipUNet(sd, "cuda", torch.float16)
        del sd
    return _CACHE["hip16"]


def make_inputs(h, w, ntiles=1, seed=0):
    from _det import unet_inputs
    return unet_inputs(h, w, ntiles, seed)


def run_hip(hip, B, x, cond, ctx, text, tids, t, h, w):
    dev = "cuda"
    hip.set_context(ctx)
    xn = x.permute(0, 2, 3, 1).reshape(B * h * w, 4).to(dev, torch.bfloat16).contiguous()
    cn = cond.permute(0, 2, 3, 1).reshape(B * h * w, 512).to(dev, torch.bfloat16).contiguous()
    tt = torch.full((B,), float(t), device=dev)
    eps = hip.forward(xn, tt, tids.to(dev), text.to(dev), cn, B, h, w)
    torch.cuda.synchronize()
    return eps.float().reshape(B, h, w, 4).permute(0, 3, 1, 2).cpu()


def run_ref(ref, B, x, cond, ctx, text, tids, t):
    """One oracle forward per tile (B = 2 CFG rows), as the reference's tile loop does (pipeline:1330):
    its information transformer attends over the whole batch axis, so tiles must not share a forward."""
    outs = []
    with torch.no_grad():
        for i in range(0, B, 2):
            s = slice(i, i + 2)
            outs.append(ref(x[s], t, ctx, {"text_embeds": text[s], "time_ids": tids[s]}, input_embedding=cond[s]))
    return torch.cat(outs, 0)


def metrics(a, b):
    import parity
    return parity.rel_l2(a, b), parity.cos(a, b)


@pytest.mark.parametrize("h,w,ntiles,t", [(32, 32, 1, 951.0), (40, 24, 2, 501.0), (128, 128, 1, 951.0),
                                           (62, 46, 1, 951.0)])
def test_unet_forward_matches_oracle(h, w, ntiles, t):
    """62x46 is not a multiple of 4: diffusers' forward_upsample_size path (ext:522-529, 665-666), 62 -> 31 -> 16 down
    and 16 -> 31 -> 62 up, as every test_wo_llava.py image whose padded latent is not a multiple of 4 runs."""
    ref, hip = unet_pair()
    B, x, cond, ctx, text, tids = make_inputs(h, w, ntiles)
    out = run_hip(hip, B, x, cond, ctx, text, tids, t, h, w)
    exp = run_ref(ref, B, x, cond, ctx, text, tids, t)
    rel, cos = metrics(out, exp)
    print(f"unet {h}x{w} tiles={ntiles}: rel_l2={rel:.3e} cos={cos:.6f} |eps|={exp.norm().item():.3e}")
    assert rel < 1.5e-2 and cos > 0.9999


@pytest.mark.parametrize("dtype", ["bf16", "fp16"])
@pytest.mark.parametrize("name", ["s32", "odd62x46", "noadd32", "noemb24"])
def test_unet_forward_matches_reference_golden(name, dtype):
    """HIP UNet directly against the reference's own forward (ext:480-697) run on the oracle's fp32 blocks
    (tests/golden/make_unet_golden.py): same weights (seed 1), same inputs; covers add_sample=False (ext:579) and
    no input_embedding (ext:572).  Same bar as against the oracle (bf16); fp16, the reference's own UNet dtype, the
    same kernels' fp16 instances: rel-L2 < 3e-3."""
    import os

    import numpy as np
    from _det import unet_golden_cases
    case = {c[0]: c for c in unet_golden_cases()}[name]
    _, h, w, ntiles, t, add_sample, with_emb = case
    hip = hip_fp16() if dtype == "fp16" else unet_pair()[1]
    dt = torch.float16 if dtype == "fp16" else torch.bfloat16
    B, x, cond, ctx, text, tids = make_inputs(h, w, ntiles)
    dev = "cuda"
    hip.set_context(ctx)
    xn = x.permute(0, 2, 3, 1).reshape(B * h * w, 4).to(dev, dt).contiguous()
    cn = cond.permute(0, 2, 3, 1).reshape(B * h * w, 512).to(dev, dt).contiguous() if with_emb else None
    eps = hip.forward(xn, torch.full((B,), float(t), device=dev), tids.to(dev), text.to(dev), cn, B, h, w,
                      add_sample=add_sample)
    torch.cuda.synchronize()
    out = eps.float().reshape(B, h, w, 4).permute(0, 3, 1, 2).cpu()
    gold = torch.from_numpy(np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden",
                                                 "unet_golden.npz"))[f"unet_{name}"])
    rel, cos = metrics(out, gold)
    print(f"unet {name} ({dtype}) vs reference-forward golden: rel_l2={rel:.3e} cos={cos:.6f}")
    assert rel < (3e-3 if dtype == "fp16" else 1.5e-2) and cos > 0.9999


def test_unet_cfg_rows_and_tile_batching_consistent():
    """Batching two tiles in one forward == two single-tile forwards (rows independent, bitwise)."""
    _, hip = unet_pair()
    h = w = 32
    B, x, cond, ctx, text, tids = make_inputs(h, w, 2, seed=5)
    both = run_hip(hip, B, x, cond, ctx, text, tids, 951.0, h, w)
    one = run_hip(hip, 2, x[:2], cond[:2], ctx, text[:2], tids[:2], 951.0, h, w)
    two = run_hip(hip, 2, x[2:], cond[2:], ctx, text[2:], tids[2:], 951.0, h, w)
    assert torch.equal(both[:2], one) and torch.equal(both[2:], two)


def test_unet_fp8_weights_match_oracle():
    """quantize_8bit / use_fp8 (utils/system.py:13-32): every UNet parameter rounded to unscaled
    float8_e4m3fn, compute at 16 bit.  The HIP UNet (bf16 compute on the e4m3 values) against the fp32 oracle
    on the same e4m3-rounded weights: same bar as the bf16 model (rel-L2 <= 1.5e-2, cos >= 0.9999; measured
    7.5e-3).  This is the default use_fp8 arithmetic (quantize_8bit without fp8_mfma).  The e4m3
    rounding itself (fp8 model vs bf16 model) is reported, not bounded: it is the reference's own choice."""
    from fdhip import arch
    from fdhip.unet import HipUNet
    from oracle.unet import UNet2DConditionModel
    sd = arch.quantize_e4m3(arch.random_init(arch.unet_param_shapes(), seed=1))
    ref = UNet2DConditionModel()
    ref.load_state_dict(sd)
    ref.eval()
    hip = HipUNet(sd, "cuda", torch.bfloat16)
    del sd
    h = w = 32
    B, x, cond, ctx, text, tids = make_inputs(h, w, 1, seed=3)
    out = run_hip(hip, B, x, cond, ctx, text, tids, 951.0, h, w)
    exp = run_ref(ref, B, x, cond, ctx, text, tids, 951.0)
    rel, cos = metrics(out, exp)
    _, hip16 = unet_pair()
    out16 = run_hip(hip16, B, x, cond, ctx, text, tids, 951.0, h, w)
    q_rel, _ = metrics(out, out16)
    print(f"unet fp8-weights {h}x{w}: rel_l2 vs oracle={rel:.3e} cos={cos:.6f}; e4m3 vs bf16 weights rel={q_rel:.3e}")
    assert rel < 1.5e-2 and cos > 0.9999


def test_graph_replay_follows_set_context():
    """HipUNet.run replays a captured hipGraph; a new prompt given to set_context (the prompt K/V projection
    is computed there, once per prompt) must reach the replayed graph: run() after set_context(ctx2) equals an
    eager forward under ctx2, bitwise, and differs from the ctx1 result."""
    _, hip = unet_pair()
    h = w = 32
    B, x, cond, ctx1, text, tids = make_inputs(h, w, 1, seed=3)
    ctx2 = torch.randn(2, 77, 2048, generator=torch.Generator().manual_seed(9))
    dev = "cuda"
    xn = x.permute(0, 2, 3, 1).reshape(B * h * w, 4).to(dev, torch.bfloat16).contiguous()
    cn = cond.permute(0, 2, 3, 1).reshape(B * h * w, 512).to(dev, torch.bfloat16).contiguous()
    tt = torch.full((B,), 951.0, device=dev)
    args = (xn, tt, tids.to(dev), text.to(dev), cn, B, h, w)
    hip.graphs.clear()
    hip.set_context(ctx1)
    for _ in range(3):  # eager, capture, replay
        r1 = hip.run(*args).clone()
    hip.set_context(ctx2)
    r2 = hip.run(*args).clone()
    e2 = hip.forward(*args).clone()
    hip.set_context(ctx1)
    e1 = hip.forward(*args).clone()
    assert len(hip.graphs) == 1
    assert torch.equal(r2, e2)
    assert torch.equal(r1, e1)
    assert not torch.equal(r1, r2)


def test_cond_embed_hoisted_is_bitwise():
    """HipUNet.cond_embed (the condition embedding computed once per tile, outside the loop) + forward(...,
    cond_embedded=True) gives the bits of forward(image latents) -- for a two-tile batch whose embedding is
    computed in one launch set as in the pipeline."""
    _, hip = unet_pair()
    h, w = 40, 24
    B, x, cond, ctx, text, tids = make_inputs(h, w, 2, seed=5)
    dev = "cuda"
    hip.set_context(ctx)
    xn = x.permute(0, 2, 3, 1).reshape(B * h * w, 4).to(dev, torch.bfloat16).contiguous()
    cn = cond.permute(0, 2, 3, 1).reshape(B * h * w, 512).to(dev, torch.bfloat16).contiguous()
    tt = torch.full((B,), 701.0, device=dev)
    full = hip.forward(xn, tt, tids.to(dev), text.to(dev), cn, B, h, w).clone()
    ie = hip.cond_embed(cn, B, h, w)
    hoisted = hip.forward(xn, tt, tids.to(dev), text.to(dev), ie, B, h, w, cond_embedded=True)
    assert torch.equal(full, hoisted)
    # per-tile embeddings (2 rows each) == the batched one
    ie1 = torch.cat([hip.cond_embed(cn[i * 2 * h * w:(i + 1) * 2 * h * w].contiguous(), 2, h, w) for i in range(2)])
    assert torch.equal(ie1, ie)
