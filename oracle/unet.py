"""fp32 CPU restatement of the SDXL UNet + FaithDiff conditioning extras.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Module/parameter names are exactly diffusers 0.28's so that a diffusers state
dict (and ``FaithDiff.bin``) loads unchanged.  Forward semantics follow:
  * FaithDiff forward order ............ unet_2d_condition_vae_extension.py:480-697
  * ControlNetConditioningEmbedding ... ext:199-219 (norm -> conv_in -> SiLU -> conv_out)
  * QuickGELU / LayerNorm / ResidualAttentionBlock ... ext:222-260
    (nn.MultiheadAttention with batch_first=False: attends over the *batch* axis)
  * extras construction ................ ext:389-403
  * diffusers blocks (ResnetBlock2D, Transformer2DModel, BasicTransformerBlock,
    Down/Up/Mid blocks, Timesteps/TimestepEmbedding) per SURVEY Appendix B.1.
"""
import math
from collections import OrderedDict

import torch
import torch.nn as nn
import torch.nn.functional as F


# ----------------------------------------------------------------------------- embeddings
def timestep_embedding(t, dim, flip_sin_to_cos=True, shift=0.0, max_period=10000):
    """diffusers.models.embeddings.get_timestep_embedding (SDXL: flip=True, shift=0)."""
    half = dim // 2
    exponent = -math.log(max_period) * torch.arange(half, dtype=torch.float32) / (half - shift)
    emb = t.float()[:, None] * torch.exp(exponent)[None, :]
    emb = torch.cat([torch.sin(emb), torch.cos(emb)], dim=-1)
    if flip_sin_to_cos:
        emb = torch.cat([emb[:, half:], emb[:, :half]], dim=-1)
    return emb


class TimestepEmbedding(nn.Module):
    def __init__(self, cin, dim):
        super().__init__()
        self.linear_1 = nn.Linear(cin, dim)
        self.linear_2 = nn.Linear(dim, dim)

    def forward(self, x):
        return self.linear_2(F.silu(self.linear_1(x)))


# ----------------------------------------------------------------------------- resnet / attention
class ResnetBlock2D(nn.Module):
    """diffusers ResnetBlock2D, resnet_time_scale_shift='default', output_scale_factor=1."""

    def __init__(self, cin, cout, temb_channels=1280, eps=1e-5, groups=32):
        super().__init__()
        self.norm1 = nn.GroupNorm(groups, cin, eps=eps)
        self.conv1 = nn.Conv2d(cin, cout, 3, padding=1)
        self.time_emb_proj = nn.Linear(temb_channels, cout) if temb_channels else None
        self.norm2 = nn.GroupNorm(groups, cout, eps=eps)
        self.conv2 = nn.Conv2d(cout, cout, 3, padding=1)
        self.conv_shortcut = nn.Conv2d(cin, cout, 1) if cin != cout else None

    def forward(self, x, temb=None):
        h = self.conv1(F.silu(self.norm1(x)))
        if temb is not None and self.time_emb_proj is not None:
            h = h + self.time_emb_proj(F.silu(temb))[:, :, None, None]
        h = self.conv2(F.silu(self.norm2(h)))
        if self.conv_shortcut is not None:
            x = self.conv_shortcut(x)
        return x + h


class Attention(nn.Module):
    """diffusers Attention + AttnProcessor2_0 (SDPA, scale = dim_head**-0.5)."""

    def __init__(self, query_dim, heads, dim_head, cross_dim=None, bias=False, out_bias=True,
                 group_norm_groups=None, eps=1e-6):
        super().__init__()
        inner = heads * dim_head
        self.heads = heads
        self.group_norm = nn.GroupNorm(group_norm_groups, query_dim, eps=eps) if group_norm_groups else None
        self.to_q = nn.Linear(query_dim, inner, bias=bias)
        self.to_k = nn.Linear(cross_dim or query_dim, inner, bias=bias)
        self.to_v = nn.Linear(cross_dim or query_dim, inner, bias=bias)
        self.to_out = nn.ModuleList([nn.Linear(inner, query_dim, bias=out_bias), nn.Dropout(0.0)])

    def forward(self, x, ctx=None):  # x: (B, T, C)
        B, T, _ = x.shape
        ctx = x if ctx is None else ctx
        q, k, v = self.to_q(x), self.to_k(ctx), self.to_v(ctx)
        hd = q.shape[-1] // self.heads
        q = q.view(B, -1, self.heads, hd).transpose(1, 2)
        k = k.view(B, -1, self.heads, hd).transpose(1, 2)
        v = v.view(B, -1, self.heads, hd).transpose(1, 2)
        o = F.scaled_dot_product_attention(q, k, v)
        o = o.transpose(1, 2).reshape(B, T, -1)
        return self.to_out[0](o)


class GEGLU(nn.Module):
    def __init__(self, dim, inner):
        super().__init__()
        self.proj = nn.Linear(dim, inner * 2)

    def forward(self, x):
        h, g = self.proj(x).chunk(2, dim=-1)
        return h * F.gelu(g)  # exact erf GELU


class FeedForward(nn.Module):
    def __init__(self, dim, mult=4):
        super().__init__()
        self.net = nn.ModuleList([GEGLU(dim, dim * mult), nn.Dropout(0.0), nn.Linear(dim * mult, dim)])

    def forward(self, x):
        return self.net[2](self.net[0](x))


class BasicTransformerBlock(nn.Module):
    def __init__(self, dim, heads, cross_dim=2048):
        super().__init__()
        self.norm1 = nn.LayerNorm(dim, eps=1e-5)
        self.attn1 = Attention(dim, heads, 64)
        self.norm2 = nn.LayerNorm(dim, eps=1e-5)
        self.attn2 = Attention(dim, heads, 64, cross_dim=cross_dim)
        self.norm3 = nn.LayerNorm(dim, eps=1e-5)
        self.ff = FeedForward(dim)

    def forward(self, x, ctx):
        x = self.attn1(self.norm1(x)) + x
        x = self.attn2(self.norm2(x), ctx) + x
        x = self.ff(self.norm3(x)) + x
        return x


class Transformer2DModel(nn.Module):
    """use_linear_projection=True, GN(32, eps 1e-6)."""

    def __init__(self, dim, heads, layers, cross_dim=2048):
        super().__init__()
        self.norm = nn.GroupNorm(32, dim, eps=1e-6)
        self.proj_in = nn.Linear(dim, dim)
        self.transformer_blocks = nn.ModuleList([BasicTransformerBlock(dim, heads, cross_dim) for _ in range(layers)])
        self.proj_out = nn.Linear(dim, dim)

    def forward(self, x, ctx):
        B, C, H, W = x.shape
        res = x
        h = self.norm(x).permute(0, 2, 3, 1).reshape(B, H * W, C)
        h = self.proj_in(h)
        for blk in self.transformer_blocks:
            h = blk(h, ctx)
        h = self.proj_out(h)
        return h.reshape(B, H, W, C).permute(0, 3, 1, 2) + res


class Downsample2D(nn.Module):
    def __init__(self, ch, padding=1):
        super().__init__()
        self.padding = padding
        self.conv = nn.Conv2d(ch, ch, 3, stride=2, padding=padding)

    def forward(self, x):
        if self.padding == 0:  # VAE encoder form: pad (0,1,0,1) with zeros
            x = F.pad(x, (0, 1, 0, 1), mode="constant", value=0.0)
        return self.conv(x)


class Upsample2D(nn.Module):
    def __init__(self, ch):
        super().__init__()
        self.conv = nn.Conv2d(ch, ch, 3, padding=1)

    def forward(self, x, size=None):
        # diffusers Upsample2D: x2, or `upsample_size` (the next skip's size) when the latent is not a
        # multiple of 4 (forward_upsample_size, ext:522-529,665-666)
        if size is None:
            return self.conv(F.interpolate(x, scale_factor=2.0, mode="nearest"))
        return self.conv(F.interpolate(x, size=size, mode="nearest"))


# ----------------------------------------------------------------------------- UNet blocks
class DownBlock(nn.Module):
    def __init__(self, cin, cout, n_attn_layers, heads, add_downsample):
        super().__init__()
        self.resnets = nn.ModuleList([ResnetBlock2D(cin if i == 0 else cout, cout) for i in range(2)])
        if n_attn_layers:
            self.attentions = nn.ModuleList([Transformer2DModel(cout, heads, n_attn_layers) for _ in range(2)])
        else:
            self.attentions = None
        self.downsamplers = nn.ModuleList([Downsample2D(cout)]) if add_downsample else None

    def forward(self, x, temb, ctx):
        outs = []
        for i, r in enumerate(self.resnets):
            x = r(x, temb)
            if self.attentions is not None:
                x = self.attentions[i](x, ctx)
            outs.append(x)
        if self.downsamplers is not None:
            x = self.downsamplers[0](x)
            outs.append(x)
        return x, outs


class UpBlock(nn.Module):
    def __init__(self, cin_prev, cout, skip_chs, n_attn_layers, heads, add_upsample):
        super().__init__()
        rs = []
        for i in range(3):
            rin = (cin_prev if i == 0 else cout) + skip_chs[i]
            rs.append(ResnetBlock2D(rin, cout))
        self.resnets = nn.ModuleList(rs)
        if n_attn_layers:
            self.attentions = nn.ModuleList([Transformer2DModel(cout, heads, n_attn_layers) for _ in range(3)])
        else:
            self.attentions = None
        self.upsamplers = nn.ModuleList([Upsample2D(cout)]) if add_upsample else None

    def forward(self, x, skips, temb, ctx):
        for i, r in enumerate(self.resnets):
            x = torch.cat([x, skips.pop()], dim=1)
            x = r(x, temb)
            if self.attentions is not None:
                x = self.attentions[i](x, ctx)
        if self.upsamplers is not None:
            fwd_size = any(d % 4 for d in self._latent_hw) if hasattr(self, "_latent_hw") else False
            x = self.upsamplers[0](x, skips[-1].shape[2:] if (skips and fwd_size) else None)
        return x


class MidBlock(nn.Module):
    def __init__(self, ch, heads, layers):
        super().__init__()
        self.resnets = nn.ModuleList([ResnetBlock2D(ch, ch), ResnetBlock2D(ch, ch)])
        self.attentions = nn.ModuleList([Transformer2DModel(ch, heads, layers)])

    def forward(self, x, temb, ctx):
        x = self.resnets[0](x, temb)
        x = self.attentions[0](x, ctx)
        return self.resnets[1](x, temb)


# ----------------------------------------------------------------------------- FaithDiff extras
class ControlNetConditioningEmbedding(nn.Module):
    """ext:199-219 -- GN(32, eps 1e-6) -> conv_in -> SiLU -> conv_out (zero-init in the reference)."""

    def __init__(self, out_ch=320, ch=512):
        super().__init__()
        self.conv_in = nn.Conv2d(ch, ch, 3, padding=1)
        self.norm_in = nn.GroupNorm(num_channels=ch, num_groups=32, eps=1e-6)
        self.conv_out = nn.Conv2d(ch, out_ch, 3, padding=1)

    def forward(self, c):
        c = self.norm_in(c)
        e = F.silu(self.conv_in(c))
        return self.conv_out(e)


class QuickGELU(nn.Module):  # ext:222-226
    def forward(self, x):
        return x * torch.sigmoid(1.702 * x)


class ResidualAttentionBlock(nn.Module):
    """ext:238-260.  nn.MultiheadAttention(d, n) with batch_first=False, fed (B, HW, C):
    the *sequence* axis is B and the batch axis is HW (SURVEY key finding 5)."""

    def __init__(self, d_model=640, n_head=8):
        super().__init__()
        self.attn = nn.MultiheadAttention(d_model, n_head)
        self.ln_1 = nn.LayerNorm(d_model)
        self.mlp = nn.Sequential(OrderedDict([
            ("c_fc", nn.Linear(d_model, d_model * 2)), ("gelu", QuickGELU()),
            ("c_proj", nn.Linear(d_model * 2, d_model))]))
        self.ln_2 = nn.LayerNorm(d_model)

    def forward(self, x):
        h = self.ln_1(x)
        x = x + self.attn(h, h, h, need_weights=False)[0]
        x = x + self.mlp(self.ln_2(x))
        return x


# ----------------------------------------------------------------------------- the UNet
SDXL_UNET_CONFIG = dict(
    block_out_channels=(320, 640, 1280), transformer_layers=(0, 2, 10), heads=(5, 10, 20),
    cross_attention_dim=2048, addition_time_embed_dim=256, projection_class_embeddings_input_dim=2816,
    sample_size=128, in_channels=4, out_channels=4, time_cond_proj_dim=None,
)


class UNet2DConditionModel(nn.Module):
    """SDXL UNet (diffusers key names) + FaithDiff extras (ext:389-403)."""

    def __init__(self, with_extras=True):
        super().__init__()
        C = SDXL_UNET_CONFIG["block_out_channels"]
        L = SDXL_UNET_CONFIG["transformer_layers"]
        Hd = SDXL_UNET_CONFIG["heads"]
        self.conv_in = nn.Conv2d(4, C[0], 3, padding=1)
        self.time_embedding = TimestepEmbedding(C[0], 1280)
        self.add_embedding = TimestepEmbedding(2816, 1280)
        self.down_blocks = nn.ModuleList([
            DownBlock(C[0], C[0], 0, 0, True),
            DownBlock(C[0], C[1], L[1], Hd[1], True),
            DownBlock(C[1], C[2], L[2], Hd[2], False),
        ])
        self.mid_block = MidBlock(C[2], Hd[2], L[2])
        # skip channels consumed by each up resnet (popped from the end of the down-res list)
        self.up_blocks = nn.ModuleList([
            UpBlock(C[2], C[2], [C[2], C[2], C[1]], L[2], Hd[2], True),
            UpBlock(C[2], C[1], [C[1], C[1], C[0]], L[1], Hd[1], True),
            UpBlock(C[1], C[0], [C[0], C[0], C[0]], 0, 0, False),
        ])
        self.conv_norm_out = nn.GroupNorm(32, C[0], eps=1e-5)
        self.conv_out = nn.Conv2d(C[0], 4, 3, padding=1)
        if with_extras:
            self.information_transformer_layes = nn.Sequential(*[ResidualAttentionBlock(640, 8) for _ in range(2)])
            self.spatial_ch_projs = nn.Linear(640, 320)
            self.condition_embedding = ControlNetConditioningEmbedding(320, 512)
        else:
            self.information_transformer_layes = None
            self.spatial_ch_projs = None
            self.condition_embedding = None

    def core_parameters(self):
        extras = ("information_transformer_layes.", "spatial_ch_projs.", "condition_embedding.")
        return [p for n, p in self.named_parameters() if not n.startswith(extras)]

    def forward(self, sample, timestep, encoder_hidden_states, added_cond_kwargs, input_embedding=None,
                add_sample=True):
        B = sample.shape[0]
        t = torch.as_tensor(timestep, dtype=torch.float32).reshape(-1).expand(B)
        emb = self.time_embedding(timestep_embedding(t, 320))
        tid = added_cond_kwargs["time_ids"].float()
        te = timestep_embedding(tid.flatten(), 256).reshape(B, -1)
        aug = self.add_embedding(torch.cat([added_cond_kwargs["text_embeds"].float(), te], dim=-1))
        emb = emb + aug
        ctx = encoder_hidden_states

        x = self.conv_in(sample)
        if input_embedding is not None and self.condition_embedding is not None:
            ie = self.condition_embedding(input_embedding)
            b, c, h, w = ie.shape
            feat = torch.cat([x, ie], dim=1).view(b, 2 * c, h * w).transpose(1, 2)
            feat = self.information_transformer_layes(feat)
            alpha = self.spatial_ch_projs(feat).transpose(1, 2).reshape(b, c, h, w)
            x = x + alpha if add_sample else alpha

        skips = [x]
        for blk in self.down_blocks:
            x, outs = blk(x, emb, ctx)
            skips.extend(outs)
        x = self.mid_block(x, emb, ctx)
        for blk in self.up_blocks:
            blk._latent_hw = tuple(sample.shape[-2:])
            x = blk(x, skips, emb, ctx)
        x = F.silu(self.conv_norm_out(x))
        return self.conv_out(x)


def count_params(module):
    return sum(p.numel() for p in module.parameters())
