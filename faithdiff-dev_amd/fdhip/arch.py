"""Architecture spec of the FaithDiff/SDXL UNet, the sdxl-vae-fp16-fix AutoencoderKL and the FaithDiff
denoise encoder: parameter names (diffusers 0.28 state-dict keys) and shapes, plus a seeded random init.

The reference loads real checkpoints by HF name (create_FaithDiff_model.py:13-16, CKPT_PTH.py:3-5); none
exist offline, so the ``random-init`` path (BASELINE.json north star) draws every tensor from a per-key
seeded generator: results do not depend on iteration order, and the same (key, seed) gives the same
values on every host.  Zero-initialised modules of the reference (condition_embedding.conv_out,
spatial_ch_projs, ext:209,399) are NOT zero here, so that the conditioning path is exercised.
"""
import zlib

import torch

UNET_CH = (320, 640, 1280)
UNET_LAYERS = (0, 2, 10)
UNET_HEADS = (5, 10, 20)
VAE_CH = (128, 256, 512, 512)


def _lin(d, name, n, k, bias=True):
    d[name + ".weight"] = (n, k)
    if bias:
        d[name + ".bias"] = (n,)


def _conv(d, name, co, ci, k=3, bias=True):
    d[name + ".weight"] = (co, ci, k, k)
    if bias:
        d[name + ".bias"] = (co,)


def _norm(d, name, c):
    d[name + ".weight"] = (c,)
    d[name + ".bias"] = (c,)


def _resnet(d, p, cin, cout, temb=True):
    _norm(d, p + ".norm1", cin)
    _conv(d, p + ".conv1", cout, cin)
    if temb:
        _lin(d, p + ".time_emb_proj", cout, 1280)
    _norm(d, p + ".norm2", cout)
    _conv(d, p + ".conv2", cout, cout)
    if cin != cout:
        _conv(d, p + ".conv_shortcut", cout, cin, 1)


def _t2d(d, p, c, layers):
    _norm(d, p + ".norm", c)
    _lin(d, p + ".proj_in", c, c)
    for i in range(layers):
        b = f"{p}.transformer_blocks.{i}"
        _norm(d, b + ".norm1", c)
        for n in ("to_q", "to_k", "to_v"):
            _lin(d, f"{b}.attn1.{n}", c, c, bias=False)
        _lin(d, b + ".attn1.to_out.0", c, c)
        _norm(d, b + ".norm2", c)
        _lin(d, b + ".attn2.to_q", c, c, bias=False)
        _lin(d, b + ".attn2.to_k", c, 2048, bias=False)
        _lin(d, b + ".attn2.to_v", c, 2048, bias=False)
        _lin(d, b + ".attn2.to_out.0", c, c)
        _norm(d, b + ".norm3", c)
        _lin(d, b + ".ff.net.0.proj", 8 * c, c)
        _lin(d, b + ".ff.net.2", c, 4 * c)
    _lin(d, p + ".proj_out", c, c)


def up_skip_channels():
    C = UNET_CH
    return [[C[2], C[2], C[1]], [C[1], C[1], C[0]], [C[0], C[0], C[0]]]


def unet_param_shapes(with_extras=True):
    """diffusers key -> shape for the SDXL UNet (+ FaithDiff extras, ext:389-403)."""
    d = {}
    C, Lr = UNET_CH, UNET_LAYERS
    _conv(d, "conv_in", C[0], 4)
    _lin(d, "time_embedding.linear_1", 1280, 320)
    _lin(d, "time_embedding.linear_2", 1280, 1280)
    _lin(d, "add_embedding.linear_1", 1280, 2816)
    _lin(d, "add_embedding.linear_2", 1280, 1280)
    prev = C[0]
    for i in range(3):
        for j in range(2):
            _resnet(d, f"down_blocks.{i}.resnets.{j}", prev if j == 0 else C[i], C[i])
            if Lr[i]:
                _t2d(d, f"down_blocks.{i}.attentions.{j}", C[i], Lr[i])
        if i < 2:
            _conv(d, f"down_blocks.{i}.downsamplers.0.conv", C[i], C[i])
        prev = C[i]
    _resnet(d, "mid_block.resnets.0", C[2], C[2])
    _t2d(d, "mid_block.attentions.0", C[2], Lr[2])
    _resnet(d, "mid_block.resnets.1", C[2], C[2])
    skips = up_skip_channels()
    prev = C[2]
    for i in range(3):
        lvl = 2 - i
        co = C[lvl]
        for j in range(3):
            cin = (prev if j == 0 else co) + skips[i][j]
            _resnet(d, f"up_blocks.{i}.resnets.{j}", cin, co)
            if Lr[lvl]:
                _t2d(d, f"up_blocks.{i}.attentions.{j}", co, Lr[lvl])
        if i < 2:
            _conv(d, f"up_blocks.{i}.upsamplers.0.conv", co, co)
        prev = co
    _norm(d, "conv_norm_out", C[0])
    _conv(d, "conv_out", 4, C[0])
    if with_extras:
        for i in range(2):
            p = f"information_transformer_layes.{i}"
            d[p + ".attn.in_proj_weight"] = (1920, 640)
            d[p + ".attn.in_proj_bias"] = (1920,)
            _lin(d, p + ".attn.out_proj", 640, 640)
            _norm(d, p + ".ln_1", 640)
            _lin(d, p + ".mlp.c_fc", 1280, 640)
            _lin(d, p + ".mlp.c_proj", 640, 1280)
            _norm(d, p + ".ln_2", 640)
        _lin(d, "spatial_ch_projs", 320, 640)
        _conv(d, "condition_embedding.conv_in", 512, 512)
        _norm(d, "condition_embedding.norm_in", 512)
        _conv(d, "condition_embedding.conv_out", 320, 512)
    return d


def _vae_attn(d, p, c):
    _norm(d, p + ".group_norm", c)
    for n in ("to_q", "to_k", "to_v", "to_out.0"):
        _lin(d, f"{p}.{n}", c, c)


def encoder_param_shapes(prefix="", with_out=True):
    """VAE encoder trunk (diffusers Encoder); with_out=False is the FaithDiff denoise encoder (ext:39-196)."""
    d = {}
    ch = VAE_CH
    _conv(d, prefix + "conv_in", ch[0], 3)
    prev = ch[0]
    for i, c in enumerate(ch):
        for j in range(2):
            _resnet(d, f"{prefix}down_blocks.{i}.resnets.{j}", prev if j == 0 else c, c, temb=False)
        if i < 3:
            _conv(d, f"{prefix}down_blocks.{i}.downsamplers.0.conv", c, c)
        prev = c
    _resnet(d, prefix + "mid_block.resnets.0", ch[-1], ch[-1], temb=False)
    _vae_attn(d, prefix + "mid_block.attentions.0", ch[-1])
    _resnet(d, prefix + "mid_block.resnets.1", ch[-1], ch[-1], temb=False)
    if with_out:
        _norm(d, prefix + "conv_norm_out", ch[-1])
        _conv(d, prefix + "conv_out", 8, ch[-1])
    return d


def vae_param_shapes():
    d = encoder_param_shapes("encoder.", True)
    rch = tuple(reversed(VAE_CH))
    _conv(d, "decoder.conv_in", rch[0], 4)
    _resnet(d, "decoder.mid_block.resnets.0", rch[0], rch[0], temb=False)
    _vae_attn(d, "decoder.mid_block.attentions.0", rch[0])
    _resnet(d, "decoder.mid_block.resnets.1", rch[0], rch[0], temb=False)
    prev = rch[0]
    for i, c in enumerate(rch):
        for j in range(3):
            _resnet(d, f"decoder.up_blocks.{i}.resnets.{j}", prev if j == 0 else c, c, temb=False)
        if i < 3:
            _conv(d, f"decoder.up_blocks.{i}.upsamplers.0.conv", c, c)
        prev = c
    _norm(d, "decoder.conv_norm_out", rch[-1])
    _conv(d, "decoder.conv_out", 3, rch[-1])
    _conv(d, "quant_conv", 8, 8, 1)
    _conv(d, "post_quant_conv", 4, 4, 1)
    return d


def random_init(shapes, seed=0, device="cpu", dtype=torch.float32, gain=1.0):
    """Seeded per-key init: weights U(-1,1)*gain/sqrt(fan_in); biases U(-1,1)*0.05;
    norm weights 1 + 0.1*U(-1,1); norm biases 0.05*U(-1,1)."""
    sd = {}
    for name, shape in shapes.items():
        g = torch.Generator(device=device).manual_seed((zlib.crc32(name.encode()) ^ (seed * 0x9E3779B1)) & 0x7FFFFFFF)
        u = torch.rand(shape, generator=g, device=device, dtype=torch.float32) * 2 - 1
        is_norm = (".norm" in name or ".ln_" in name or name.startswith("conv_norm_out") or "group_norm" in name
                   or "norm_in" in name or "conv_norm_out" in name or "layer_norm" in name)
        if len(shape) == 1:
            if is_norm and name.endswith("weight"):
                t = 1.0 + 0.1 * u
            else:
                t = 0.05 * u
        else:
            fan_in = 1
            for s in shape[1:]:
                fan_in *= s
            t = u * (gain / fan_in ** 0.5)
        sd[name] = t.to(dtype)
    return sd


# SDXL text encoders (diffusers StableDiffusionXLPipeline: text_encoder = CLIPTextModel ViT-L/14,
# text_encoder_2 = CLIPTextModelWithProjection OpenCLIP ViT-bigG/14), transformers config fields.
CLIP_L = dict(vocab=49408, D=768, layers=12, heads=12, inter=3072, act="quickgelu", proj=None, max_pos=77)
CLIP_G = dict(vocab=49408, D=1280, layers=32, heads=20, inter=5120, act="gelu", proj=1280, max_pos=77)


def clip_param_shapes(cfg):
    """transformers CLIPTextModel / CLIPTextModelWithProjection state-dict keys (real weights load as-is)."""
    D, I = cfg["D"], cfg["inter"]
    d = {"text_model.embeddings.token_embedding.weight": (cfg["vocab"], D),
         "text_model.embeddings.position_embedding.weight": (cfg["max_pos"], D)}
    for i in range(cfg["layers"]):
        p = f"text_model.encoder.layers.{i}"
        for n in ("q_proj", "k_proj", "v_proj", "out_proj"):
            d[f"{p}.self_attn.{n}.weight"] = (D, D)
            d[f"{p}.self_attn.{n}.bias"] = (D,)
        for n in ("layer_norm1", "layer_norm2"):
            d[f"{p}.{n}.weight"] = (D,)
            d[f"{p}.{n}.bias"] = (D,)
        d[f"{p}.mlp.fc1.weight"] = (I, D)
        d[f"{p}.mlp.fc1.bias"] = (I,)
        d[f"{p}.mlp.fc2.weight"] = (D, I)
        d[f"{p}.mlp.fc2.bias"] = (D,)
    d["text_model.final_layer_norm.weight"] = (D,)
    d["text_model.final_layer_norm.bias"] = (D,)
    if cfg["proj"]:
        d["text_projection.weight"] = (cfg["proj"], D)
    return d


def quantize_e4m3(sd):
    """utils/system.py:13-32 (quantize_8bit) semantics: ``unet.to(torch.float8_e4m3fn)`` casts EVERY floating
    parameter of the UNet -- core, FaithDiff extras, norm weights and biases -- to OCP e4m3 with no scale
    (round to nearest even; |x| > 448 is not representable and becomes NaN, as in torch); the pipeline then
    computes at 16 bit under autocast, i.e. on the e4m3 values widened exactly.  Returns those widened
    values in fp32 (e4m3 is a subset of bf16, so the HIP UNet stores them without a second rounding).
    The denoise encoder is not part of ``sd`` here; the reference keeps it fp16 (:24-26)."""
    return {k: (v.to(torch.float8_e4m3fn).to(torch.float32) if v.is_floating_point() else v) for k, v in sd.items()}


def count(shapes):
    n = 0
    for s in shapes.values():
        k = 1
        for x in s:
            k *= x
        n += k
    return n


def unet_flops(h, w, B=2, with_extras=True, Lk=77, prompt_kv=True, cond_embed=True):
    """Algorithmic FLOPs (2 per MAC) of one UNet forward on B rows of an h x w latent: every conv / Linear
    GEMM plus attention QK^T and PV (4*Lq*Lk*d per head); norms/elementwise are bytes, not FLOPs
    (SURVEY 8(d)).  C2 (B=2, 128x128) = 14.217 TFLOP.  prompt_kv=False leaves out the attn2 to_k / to_v
    projections of the prompt (0.105 TFLOP at C2), which HipUNet computes once per prompt (set_context);
    cond_embed=False the condition embedding of the image latents (0.251 TFLOP), computed once per tile
    (HipUNet.cond_embed)."""
    C, Lr, Hd = UNET_CH, UNET_LAYERS, UNET_HEADS
    f = 0.0

    def conv(M, ci, co, k=3):
        return 2.0 * M * co * k * k * ci

    def lin(M, k, n):
        return 2.0 * M * k * n

    def resnet(M, ci, co):
        x = conv(M, ci, co) + conv(M, co, co)
        if ci != co:
            x += lin(M, ci, co)
        return x

    def t2d(M, T, c, layers):
        x = 2 * lin(M, c, c)
        for _ in range(layers):
            x += lin(M, c, 3 * c) + lin(M, c, c) + 4.0 * B * T * T * c        # attn1
            x += lin(M, c, c) + (lin(B * Lk, 2048, 2 * c) if prompt_kv else 0.0) + lin(M, c, c) \
                + 4.0 * B * T * Lk * c  # attn2
            x += lin(M, c, 8 * c) + lin(M, 4 * c, c)                          # GEGLU FF
        return x

    sizes = [(h, w)]
    for _ in range(2):
        sizes.append(((sizes[-1][0] + 1) // 2, (sizes[-1][1] + 1) // 2))
    M = [B * a * b for a, b in sizes]
    T = [a * b for a, b in sizes]
    f += conv(M[0], 4, C[0])
    if with_extras:
        if cond_embed:
            f += conv(M[0], 512, 512) + conv(M[0], 512, 320)
        f += 2 * (lin(M[0], 640, 1920) + lin(M[0], 640, 640) + 4.0 * M[0] * B * 640 + lin(M[0], 640, 1280)
                  + lin(M[0], 1280, 640))
        f += lin(M[0], 640, 320)
    prev = C[0]
    for i in range(3):
        for j in range(2):
            f += resnet(M[i], prev if j == 0 else C[i], C[i])
            if Lr[i]:
                f += t2d(M[i], T[i], C[i], Lr[i])
        if i < 2:
            f += conv(M[i + 1], C[i], C[i])
        prev = C[i]
    f += 2 * resnet(M[2], C[2], C[2]) + t2d(M[2], T[2], C[2], Lr[2])
    skips = up_skip_channels()
    prev = C[2]
    for i in range(3):
        lvl = 2 - i
        for j in range(3):
            f += resnet(M[lvl], (prev if j == 0 else C[lvl]) + skips[i][j], C[lvl])
            if Lr[lvl]:
                f += t2d(M[lvl], T[lvl], C[lvl], Lr[lvl])
        if i < 2:
            f += conv(M[lvl - 1], C[lvl], C[lvl])
        prev = C[lvl]
    f += conv(M[0], C[0], 4)
    return f


def vae_decode_flops(h, w):
    """AutoencoderKL.decode on an h x w latent (10.47 TFLOP at 128x128)."""
    rch = tuple(reversed(VAE_CH))
    f = 2.0 * h * w * 4 * 4 + 2.0 * h * w * rch[0] * 9 * 4

    def resnet(M, ci, co):
        x = 2.0 * M * co * 9 * ci + 2.0 * M * co * 9 * co
        return x + (2.0 * M * ci * co if ci != co else 0.0)

    T = h * w
    f += 2 * resnet(T, 512, 512) + 4 * 2.0 * T * 512 * 512 + 4.0 * T * T * 512
    hh, ww, prev = h, w, rch[0]
    for i, c in enumerate(rch):
        for j in range(3):
            f += resnet(hh * ww, prev if j == 0 else c, c)
        if i < 3:
            hh, ww = hh * 2, ww * 2
            f += 2.0 * hh * ww * c * 9 * c
        prev = c
    f += 2.0 * hh * ww * 3 * 9 * rch[-1]
    return f


# BSRNet pre-pass (FaithDiff/models/bsrnet_arch.py:77-98, RRDBNet(in_nc=3, out_nc=3, nf=64, nb=23, gc=32, sf=4)):
# the reference's state-dict keys and shapes.
def bsrnet_param_shapes(nb=23, nf=64, gc=32, in_nc=3, out_nc=3):
    d = {}

    def conv(name, cin, cout):
        d[name + ".weight"] = (cout, cin, 3, 3)
        d[name + ".bias"] = (cout,)
    conv("conv_first", in_nc, nf)
    for i in range(nb):
        for j in (1, 2, 3):
            for k in range(1, 6):
                conv(f"RRDB_trunk.{i}.RDB{j}.conv{k}", nf + (k - 1) * gc, gc if k < 5 else nf)
    for n in ("trunk_conv", "upconv1", "upconv2", "HRconv"):
        conv(n, nf, nf)
    conv("conv_last", nf, out_nc)
    return d
