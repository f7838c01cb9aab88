"""CPU tests of the product's host-side logic against the reference's golden vectors and the oracle."""
import os

import numpy as np
import pytest
import torch
from PIL import Image

SIZES = [(64, 64), (128, 128), (128, 192), (200, 136), (256, 256), (512, 512), (540, 960),
         (96, 300), (135, 240), (1024, 1024)]


def test_tile_grid_matches_reference(golden):
    from FaithDiff.pipelines.tlc import TileGrid
    for h, w in SIZES:
        g = TileGrid(h, w, (128, 128), 0.5)
        idx = np.array([[d["i"], d["j"]] for d in g.idxes], dtype=np.int64)
        np.testing.assert_array_equal(idx, golden[f"tlc_{h}x{w}_idx"])
        assert g.ntiles == int(golden[f"tlc_{h}x{w}_ntiles"])
        for t in range(g.ntiles):
            assert g.origin(t) == tuple(idx[t])


def test_tile_weights_bitexact(golden):
    from FaithDiff.pipelines.tlc import TileGrid
    for kh, kw in [(128, 128), (64, 64), (128, 96)]:
        g = TileGrid(kh, kw, (kh, kw), 0.5)
        np.testing.assert_array_equal(g.weights(), golden[f"gauss_{kh}x{kw}"])


def test_tile_counts_for_survey_configs():
    from FaithDiff.pipelines.tlc import TileGrid
    assert TileGrid(512, 512, (128, 128), 0.5).ntiles == 49        # C3 4096^2
    assert TileGrid(540, 960, (128, 128), 0.5).ntiles == 112       # 8K output 7680x4320
    assert TileGrid(1024, 1024, (128, 128), 0.5).ntiles == 225     # 8192^2
    assert TileGrid(128, 128, (128, 128), 0.5).ntiles == 1         # C2


@pytest.mark.parametrize("count,tb", [(225, 13), (49, 13), (1947, 13), (13, 13), (5, 13), (1, 4), (112, 15)])
def test_tile_batches_cover_every_tile_once(count, tb):
    """The denoise loop's tile batches (full + remainder, or balanced): every tile once, in order, <= tb per forward;
    balanced sizes differ by at most one and use the same number of forwards."""
    from FaithDiff.pipelines.tlc import tile_batches
    plain, bal = tile_batches(count, tb), tile_batches(count, tb, True)
    for bs in (plain, bal):
        assert [c0 for c0, _ in bs] == list(np.cumsum([0] + [n for _, n in bs])[:-1])
        assert sum(n for _, n in bs) == count and all(0 < n <= tb for _, n in bs)
    assert len(bal) == len(plain) == -(-count // tb)
    assert max(n for _, n in bal) - min(n for _, n in bal) <= 1
    assert tile_batches(0, tb) == tile_batches(0, tb, True) == []


def test_max_tile_batch_keeps_32bit_offsets():
    """The tile-batch cap: 128^2 tiles with CFG fit 51 per forward (the default 25 is half of it); the widest
    activation of a capped forward stays inside 2^31 elements, one more tile would not."""
    from FaithDiff.pipelines.tlc import WIDEST_CHANNELS, max_tile_batch
    assert max_tile_batch(128, 128, 2) == 51
    for kh, kw, cfg in [(128, 128, 2), (128, 98, 2), (64, 64, 1), (128, 128, 1)]:
        tb = max_tile_batch(kh, kw, cfg)
        assert tb * cfg * kh * kw * WIDEST_CHANNELS < 2 ** 31 <= (tb + 1) * cfg * kh * kw * WIDEST_CHANNELS
    from fdhip import knobs
    assert knobs.default("FD_TILE_BATCH") <= max_tile_batch(128, 128, 2) // 2


@pytest.mark.parametrize("n", [4, 20, 50])
def test_euler_schedule_matches_oracle(n):
    from FaithDiff.schedulers import DDPMScheduler, EulerDiscreteScheduler
    from oracle import schedulers as S
    s = EulerDiscreteScheduler()
    s.set_timesteps(n)
    ts, sig, init = S.euler_schedule(n)
    np.testing.assert_array_equal(s.timesteps, ts.numpy())
    np.testing.assert_array_equal(s.sigmas, sig.numpy())
    assert abs(s.init_noise_sigma - init) < 1e-6
    a, b = DDPMScheduler().add_noise_coefficients(999)
    x0, nz = torch.ones(1), torch.ones(1)
    assert abs(float(S.ddpm_add_noise(x0, 0 * nz, 999)) - a) < 1e-6
    assert abs(float(S.ddpm_add_noise(0 * x0, nz, 999)) - b) < 1e-6


def test_survey_schedule_constants():
    from FaithDiff.schedulers import DDPMScheduler, EulerDiscreteScheduler
    s = EulerDiscreteScheduler()
    s.set_timesteps(20)
    assert list(s.timesteps[:3]) == [951.0, 901.0, 851.0] and s.timesteps[-1] == 1.0
    assert abs(s.sigmas[0] - 11.02834) < 1e-4 and abs(s.init_noise_sigma - 11.07358) < 1e-4
    a, b = DDPMScheduler().add_noise_coefficients(999)
    assert abs(a - 0.068265) < 1e-5 and abs(b - 0.997667) < 1e-5


def test_check_image_size_replicate_pad():
    from utils.image_process import check_image_size
    rng = np.random.default_rng(0)
    arr = rng.integers(0, 255, (37, 61, 3), dtype=np.uint8)
    out, w0, h0, w1, h1 = check_image_size(Image.fromarray(arr))
    assert (w0, h0, w1, h1) == (61, 37, 64, 40)
    o = np.asarray(out)
    np.testing.assert_array_equal(o[:37, :61], arr)
    np.testing.assert_array_equal(o[37:, :61], np.repeat(arr[36:37], 3, 0))   # BORDER_REPLICATE rows
    np.testing.assert_array_equal(o[:, 61:], np.repeat(o[:, 60:61], 3, 1))   # and columns


def test_color_fix_matches_reference(golden):
    from _det import det_tensor
    from utils.color_fix import adaptive_instance_normalization, wavelet_reconstruction
    tgt = det_tensor((1, 3, 40, 56), 41, 0.2, 0.5).clamp(0, 1)
    src = det_tensor((1, 3, 40, 56), 42, 0.25, 0.45).clamp(0, 1)
    np.testing.assert_allclose(adaptive_instance_normalization(tgt, src).numpy(), golden["cf_adain"], rtol=1e-6,
                               atol=1e-6)
    np.testing.assert_allclose(wavelet_reconstruction(tgt, src).numpy(), golden["cf_wavelet"], rtol=1e-6, atol=1e-6)


def test_color_fix_pil_roundtrip():
    from utils.color_fix import adain_color_fix, wavelet_color_fix
    rng = np.random.default_rng(1)
    a = Image.fromarray(rng.integers(0, 255, (33, 47, 3), dtype=np.uint8))
    b = Image.fromarray(rng.integers(0, 255, (33, 47, 3), dtype=np.uint8))
    assert adain_color_fix(a, b).size == a.size
    assert wavelet_color_fix(a, a).size == a.size
    # identical source and target: wavelet reconstruction is the identity (up to uint8 truncation)
    assert np.abs(np.asarray(wavelet_color_fix(a, a)).astype(int) - np.asarray(a).astype(int)).max() <= 1


def test_product_arch_matches_oracle_and_survey_counts():
    from fdhip import arch
    torch.set_default_device("meta")
    try:
        from oracle.unet import UNet2DConditionModel
        from oracle.vae import AutoencoderKL, DenoiseEncoder
        for spec, mod in [(arch.unet_param_shapes(), UNet2DConditionModel()), (arch.vae_param_shapes(), AutoencoderKL()),
                          (arch.encoder_param_shapes("", False), DenoiseEncoder())]:
            assert {k: tuple(v.shape) for k, v in mod.state_dict().items()} == spec
    finally:
        torch.set_default_device("cpu")
    assert arch.count(arch.unet_param_shapes(False)) == 2_567_463_684
    assert arch.count(arch.unet_param_shapes(True)) - arch.count(arch.unet_param_shapes(False)) == 10_608_512
    assert arch.count(arch.encoder_param_shapes("", False)) == 34_125_696
    assert arch.count(arch.vae_param_shapes()) == 83_653_863
    assert abs(arch.unet_flops(128, 128, 2) / 1e12 - 14.217) < 1e-3
    assert abs(arch.vae_decode_flops(128, 128) / 1e12 - 10.47) < 1e-2


def test_random_init_is_deterministic_and_order_free():
    from fdhip import arch
    shapes = {k: v for k, v in list(arch.unet_param_shapes().items())[:20]}
    a = arch.random_init(shapes, seed=3)
    b = arch.random_init(dict(reversed(list(shapes.items()))), seed=3)
    for k in shapes:
        assert torch.equal(a[k], b[k])
    c = arch.random_init(shapes, seed=4)
    assert not torch.equal(a["conv_in.weight"], c["conv_in.weight"])


def test_pipeline_check_inputs_errors():
    from FaithDiff.pipelines.pipeline_FaithDiff_tlc import FaithDiffStableDiffusionXLPipeline
    from types import SimpleNamespace
    vae = SimpleNamespace(config=SimpleNamespace(block_out_channels=(128, 256, 512, 512)))
    p = FaithDiffStableDiffusionXLPipeline(vae=vae, denoise_encoder=None, unet=None)
    img = Image.new("RGB", (64, 64))
    with pytest.raises(ValueError):
        p.check_inputs(None, "a", None, 64, 64, None)
    with pytest.raises(ValueError):
        p.check_inputs(img, "a", None, 60, 64, None)
    with pytest.raises(ValueError):
        p.check_inputs(img, None, None, 64, 64, None)
    with pytest.raises(ValueError):
        p.check_inputs(img, "a", None, 64, 64, None, prompt_embeds=torch.zeros(1))
    with pytest.raises(ValueError):
        p.check_inputs(img, None, None, 64, 64, None, prompt_embeds=torch.zeros(1, 77, 2048))
    p.check_inputs(img, "a", None, 64, 64, None)


def test_synthetic_text_encoder_deterministic():
    from FaithDiff.pipelines.pipeline_FaithDiff_tlc import SyntheticTextEncoder
    te = SyntheticTextEncoder()
    a, pa = te("a cat")
    b, pb = te("a cat")
    c, _ = te("")
    assert a.shape == (1, 77, 2048) and pa.shape == (1, 1280)
    assert torch.equal(a, b) and torch.equal(pa, pb) and not torch.equal(a, c)
    assert c.abs().sum() > 0  # "" is encoded, not zeroed (pipeline:622-675)


@pytest.mark.parametrize("which", ["L", "G"])
def test_clip_param_shapes_match_transformers(which):
    """The HIP text encoders' state-dict keys and shapes are transformers' (real SDXL text_encoder* weights load
    strictly); built on the meta device, no memory."""
    from transformers import CLIPTextConfig, CLIPTextModel, CLIPTextModelWithProjection
    from fdhip import arch
    cfg = arch.CLIP_L if which == "L" else arch.CLIP_G
    tcfg = CLIPTextConfig(vocab_size=cfg["vocab"], hidden_size=cfg["D"], intermediate_size=cfg["inter"],
                          num_hidden_layers=cfg["layers"], num_attention_heads=cfg["heads"],
                          max_position_embeddings=cfg["max_pos"], projection_dim=cfg["proj"] or 768)
    with torch.device("meta"):
        m = (CLIPTextModelWithProjection if cfg["proj"] else CLIPTextModel)(tcfg)
    # transformers 4.x (the reference's pin, and the saved SDXL files) prefixes the text tower with
    # "text_model."; newer releases drop the prefix in the module tree (and remap old files on load)
    want = {(k if k.startswith(("text_model.", "text_projection")) else "text_model." + k): tuple(v.shape)
            for k, v in m.state_dict().items() if "position_ids" not in k}
    assert want == {k: tuple(v) for k, v in arch.clip_param_shapes(cfg).items()}
    n = sum(int(np.prod(s)) for s in want.values())
    assert n == (123060480 if which == "L" else 694659840)  # CLIP ViT-L/14 text, OpenCLIP bigG/14 text + proj


def test_fallback_tokenizer_framing():
    """Stand-in tokenizer (no vocab files offline): CLIP framing -- BOS, <= 75 ids, EOS, pad to 77 with the
    tokenizer's pad id; deterministic; truncation keeps the EOS."""
    from FaithDiff.models.clip_text import FallbackCLIPTokenizer
    t1, t2 = FallbackCLIPTokenizer(49407), FallbackCLIPTokenizer(0)
    a = t1("A photo of a cat.", padding="max_length", max_length=77, truncation=True).input_ids
    b = t2("A photo of a cat.", padding="max_length", max_length=77, truncation=True).input_ids
    assert a.shape == (1, 77) and a[0, 0] == 49406
    n = int((a[0] != 49407).sum())  # BOS + 5 words + '.' = 7 non-pad ids before the EOS
    assert n == 7 and a[0, n] == 49407 and (a[0, n:] == 49407).all()
    assert torch.equal(a[0, :n + 1], b[0, :n + 1]) and (b[0, n + 1:] == 0).all()
    assert int(a[0].argmax()) == n and int(b[0].argmax()) == n  # pooled row = first EOS for both encoders
    long = t1(" ".join(["word"] * 200), max_length=77).input_ids
    assert long.shape == (1, 77) and long[0, -1] == 49407
    assert torch.equal(t1("x y", max_length=77).input_ids, t1("x y", max_length=77).input_ids)


def test_quantize_e4m3_semantics():
    """a18: quantize_8bit = torch's float8_e4m3fn cast of every UNet parameter (RNE, no scale, NaN past 448),
    widened exactly; integers untouched.  The drop-in's use_fp8 flag routes the UNet through it."""
    import torch
    from fdhip import arch
    x = torch.tensor([0.1, 447.9, 1000.0, 1e-4, -3.3, 2.0 ** -9, 0.0])
    q = arch.quantize_e4m3({"w": x, "i": torch.tensor([3])})
    assert torch.equal(q["i"], torch.tensor([3]))
    exp = x.to(torch.float8_e4m3fn).to(torch.float32)
    assert torch.equal(torch.nan_to_num(q["w"], nan=-1.0), torch.nan_to_num(exp, nan=-1.0))
    assert torch.isnan(q["w"][2]) and q["w"][3] == 0 and q["w"][5] == 2.0 ** -9
    # every e4m3 value is exact in bf16 (the HIP UNet stores them without a second rounding)
    allv = torch.arange(256, dtype=torch.uint8).view(torch.float8_e4m3fn).to(torch.float32)
    fin = allv[torch.isfinite(allv)]
    assert torch.equal(fin.to(torch.bfloat16).to(torch.float32), fin)
    from FaithDiff.models.unet_2d_condition_vae_extension import UNet2DConditionModel
    u = UNet2DConditionModel({})
    u.quantize_8bit()
    assert u._fp8


def test_upsample_conv_phase_packing_is_the_same_function():
    """pack_conv3x3_up2: Upsample2D (nearest x2, then conv3x3 pad 1; diffusers Upsample2D, called by the VAE decoder
    and the UNet up blocks, unet_2d_condition_vae_extension.py:665-666) as four 2x2 convs of the low-resolution
    input, each phase's weights the fp32 sums of the taps that land on one source pixel -- equal in fp64 to the
    upsample-then-conv, borders included (odd sizes too)."""
    import torch.nn.functional as F
    from fdhip import ops
    g = torch.Generator().manual_seed(5)
    for (n, ci, co, H, W) in [(2, 8, 6, 5, 7), (1, 4, 4, 1, 1), (1, 3, 5, 6, 4)]:
        x = torch.randn(n, ci, H, W, generator=g, dtype=torch.float64)
        w = torch.randn(co, ci, 3, 3, generator=g, dtype=torch.float64)
        ref = F.conv2d(F.interpolate(x, scale_factor=2, mode="nearest"), w, padding=1)
        wph = ops.pack_conv3x3_up2(w).double().reshape(4, co, 2, 2, ci).permute(0, 1, 4, 2, 3)
        xp = F.pad(x, (1, 1, 1, 1))
        out = torch.empty_like(ref)
        for a in range(2):
            for b in range(2):
                out[:, :, a::2, b::2] = F.conv2d(xp[:, :, a:a + H + 1, b:b + W + 1], wph[2 * a + b])
        torch.testing.assert_close(out, ref, rtol=1e-5, atol=1e-5)


def test_band_fixture_preprocessing_and_tile_grid():
    """The reference's examples/band.png (tests/golden/band/band.png) through test_wo_llava.py:65,78-82 on the host
    (convert('RGB'), x1 LANCZOS, check_image_size): the padded input is the one the band golden was generated from
    (sha256), 1080x784 with edge-replicated padding, and the product's TLC grid cuts its 135x98 latent into the same
    two ragged 128x98 tiles as the oracle (tests/golden/make_band_golden.py)."""
    import hashlib

    import numpy as np
    from _det import band_inputs
    from FaithDiff.pipelines.tlc import TileGrid
    gold = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "band", "band_golden.npz"))
    c = band_inputs(1)
    u8 = np.asarray(c["img"], dtype=np.uint8)
    assert (c["W"], c["H"], c["w0"], c["h0"]) == (1080, 784, 1079, 778)
    assert hashlib.sha256(u8.tobytes()).hexdigest() == str(gold["input_sha256"])
    src = np.asarray(c["image"], dtype=np.uint8)
    assert np.array_equal(u8[:778, :1079], src) and np.array_equal(u8[778:, :1079], np.repeat(src[-1:], 6, 0))
    g = TileGrid(c["H"] // 8, c["W"] // 8, (128, 128), 0.5)
    assert (g.kh, g.kw, g.ntiles) == (98, 128, int(gold["ntiles"])) == (98, 128, 2)
    assert gold["final"].shape == (1, 4, 98, 135) and np.isfinite(gold["final"]).all()
