"""Pin the CPU oracle against vectors generated from the reference itself (tests/golden/make_golden.py)."""
import numpy as np
import torch

from _det import det_tensor, fill_module
from oracle import tlc, pipeline as opipe
from oracle.unet import ResidualAttentionBlock, ControlNetConditioningEmbedding

SIZES = [(64, 64), (128, 128), (128, 192), (200, 136), (256, 256), (512, 512), (540, 960),
         (96, 300), (135, 240), (1024, 1024)]


def test_tlc_origins_match_reference(golden):
    for h, w in SIZES:
        idx, _ = tlc.tile_origins(h, w, (128, 128), 0.5)
        np.testing.assert_array_equal(np.array(idx, dtype=np.int64), golden[f"tlc_{h}x{w}_idx"])
    # tile counts quoted in SURVEY 8 (C3 4096^2 -> 49 tiles)
    assert int(golden["tlc_512x512_ntiles"]) == 49


def test_gaussian_weights_bitexact(golden):
    for kh, kw in [(128, 128), (64, 64), (128, 96)]:
        w = tlc.gaussian_weights(kw, kh)
        np.testing.assert_array_equal(w[0].numpy(), golden[f"gauss_{kh}x{kw}"])


def test_tlc_blend_matches_reference(golden):
    for h, w in SIZES:
        if h * w > 200 * 200:
            continue
        la = tlc.LocalAttention((128, 128), 0.5)
        x = det_tensor((1, 4, h, w), 1000 + h * 7 + w)
        tiles = la.grids(x)
        outs = tiles * (1.0 + 0.01 * torch.arange(tiles.shape[0]).view(-1, 1, 1, 1)) + 0.05
        np.testing.assert_array_equal(la.grids_inverse(outs).numpy(), golden[f"tlc_{h}x{w}_inv"])


def test_rescale_noise_cfg(golden):
    a = det_tensor((1, 4, 16, 16), 11)
    b = det_tensor((1, 4, 16, 16), 12, 0.5)
    np.testing.assert_allclose(opipe.rescale_noise_cfg(a, b, 0.7).numpy(), golden["rescale_cfg_out"], rtol=1e-6, atol=1e-6)


def test_information_transformer_block(golden):
    blk = fill_module(ResidualAttentionBlock(640, 8), 2000).eval()
    row = det_tensor((1, 64, 640), 21)
    with torch.no_grad():
        same = blk(torch.cat([row, row], 0)).numpy()
        diff = blk(torch.cat([row, det_tensor((1, 64, 640), 22)], 0)).numpy()
    np.testing.assert_allclose(same, golden["rab_same_out"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(diff, golden["rab_diff_out"], rtol=1e-5, atol=1e-5)


def test_information_transformer_identical_rows_reduce_pointwise():
    """SURVEY key finding 5: with identical CFG rows, MHA over the batch axis == out_proj(v_proj(x))."""
    blk = fill_module(ResidualAttentionBlock(640, 8), 2000).eval()
    row = det_tensor((1, 64, 640), 21)
    x = torch.cat([row, row], 0)
    with torch.no_grad():
        full = blk(x)
        h = blk.ln_1(x)
        wv = blk.attn.in_proj_weight[1280:]
        bv = blk.attn.in_proj_bias[1280:]
        y = x + blk.attn.out_proj(h @ wv.T + bv)
        y = y + blk.mlp(blk.ln_2(y))
    torch.testing.assert_close(full, y, rtol=1e-5, atol=1e-5)


def test_condition_embedding(golden):
    cne = fill_module(ControlNetConditioningEmbedding(320, 512), 3000).eval()
    with torch.no_grad():
        out = cne(det_tensor((1, 512, 8, 8), 31)).numpy()
    np.testing.assert_allclose(out, golden["cne_out"], rtol=1e-5, atol=1e-5)


class _OracleUNet:
    """oracle/pipeline.py's UNet call signature over the shared stand-in (tests/golden/_det.py)."""

    def __call__(self, x, t, ctx, added, input_embedding=None, add_sample=True):
        from _det import standin_eps
        return standin_eps(x, t, ctx, added["text_embeds"], added["time_ids"], input_embedding)


class _OracleVAE:
    scaling_factor = 0.13025

    def encode_sample(self, x, eps):
        from _det import standin_moments
        mean, logvar = standin_moments(x).chunk(2, dim=1)
        return mean + torch.exp(0.5 * logvar.clamp(-30.0, 20.0)) * eps

    def decode(self, z):
        from _det import standin_decode
        return standin_decode(z)


def test_pipeline_orchestration_matches_reference_call():
    """oracle/pipeline.py:run_pipeline against the reference's own FaithDiffStableDiffusionXLPipeline.__call__
    (pipeline_FaithDiff_tlc.py:1187-1459, run by tests/golden/make_call_golden.py) with the same stand-in models:
    CFG order, per-tile add_time_ids, per-tile scheduler state, rescale_noise_cfg, 'lr' / 'noise' start, TLC blend
    and decode scaling, at a multi-tile, a ragged and a clamped-tile size."""
    import os

    from _det import call_cases, call_inputs, standin_features
    from oracle.pipeline import run_pipeline
    gold = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "call_golden.npz"))
    for k, (name, H, W, target, steps, g, rescale, start) in enumerate(call_cases()):
        img, pe, npe, ppe, nppe, noise, post = call_inputs(H, W, 500 + 10 * k)
        res = run_pipeline(_OracleUNet(), _OracleVAE(), standin_features, img, pe, npe, ppe, nppe, noise, post,
                           num_inference_steps=steps, guidance_scale=g, overlap=0.5, target_size=target,
                           original_size=(H, W), start_point=start, guidance_rescale=rescale)
        np.testing.assert_allclose(res["latents"].numpy(), gold[f"{name}_latents"], rtol=2e-5, atol=2e-5,
                                   err_msg=name)
        np.testing.assert_allclose(res["image"].numpy(), gold[f"{name}_image"], rtol=2e-5, atol=2e-5, err_msg=name)


def test_denoise_encoder_tiling_matches_reference(golden):
    """oracle DenoiseEncoder.blend_v / blend_h / tiled_encode / forward against the reference's Encoder methods
    (ext:150-196), both run on the same stand-in trunk: tile grid, in-place blend order, crop."""
    import types

    from _det import standin_features
    from oracle.vae import DenoiseEncoder
    for name, (H, W, ts, ov) in {"a": (160, 136, 64, 0.25), "b": (200, 96, 96, 0.25)}.items():
        ns = types.SimpleNamespace(tile_sample_min_size=ts, tile_latent_min_size=ts // 8, tile_overlap_factor=ov,
                                   use_tiling=True, encode=standin_features, blend_v=DenoiseEncoder.blend_v,
                                   blend_h=DenoiseEncoder.blend_h)
        ns.tiled_encode = types.MethodType(DenoiseEncoder.tiled_encode, ns)
        x = det_tensor((1, 3, H, W), 4000 + H + W, 0.7)
        # the stand-in trunk's vectorised tanh differs by one fp32 ulp between host CPUs (the golden was written on
        # another container: 17 of 2720 values, 3e-8); a wrong tile grid / blend / crop moves values by ~1e-2
        np.testing.assert_allclose(DenoiseEncoder.forward(ns, x).numpy(), golden[f"enc_tiled_{name}"], rtol=1e-6,
                                   atol=1e-7)
    av, bv = det_tensor((1, 8, 12, 11), 4100), det_tensor((1, 8, 9, 11), 4101)
    np.testing.assert_array_equal(DenoiseEncoder.blend_v(av, bv.clone(), 5).numpy(), golden["enc_blend_v"])
    ah, bh = det_tensor((1, 8, 9, 10), 4102), det_tensor((1, 8, 9, 11), 4103)
    np.testing.assert_array_equal(DenoiseEncoder.blend_h(ah, bh.clone(), 4).numpy(), golden["enc_blend_h"])
