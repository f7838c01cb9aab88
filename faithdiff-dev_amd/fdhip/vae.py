"""fp16 AutoencoderKL (sdxl-vae-fp16-fix) encoder/decoder and the FaithDiff denoise encoder on HIP, NHWC.

Semantics per SURVEY Appendix B.2 and FaithDiff/models/unet_2d_condition_vae_extension.py:39-196:
resnets without temb (GN eps 1e-6), VAE Downsample2D = zero pad (0,1,0,1) + conv s2 p0 (folded into the
implicit-GEMM gather as pad=0 with a bottom/right zero fringe), Upsample2D = nearest x2 folded into the
next conv's gather, mid-block single-head d=512 attention with residual.

The d=512 mid-block attention runs as one flash kernel (fd_flash_attn_d512: online softmax in fp32, QK^T and PV on
the MFMA, K / V tiles staged through LDS), so no [T, T] score / probability buffer (1.5 GB at T = 16384) exists.
"""
import torch

from . import arch, knobs
from . import lib as L
from . import ops
from .graphs import GraphCache


def _dev(t, device, dtype):
    return t.to(device=device, dtype=dtype).contiguous()


class _Trunk:
    """Shared resnet / attention helpers (weights keyed by diffusers names under `prefix`)."""

    def __init__(self, sd, prefix, device, dtype):
        self.sd, self.prefix, self.device, self.dtype = sd, prefix, torch.device(device), dtype

    def f32(self, k):
        return _dev(self.sd[self.prefix + k], self.device, torch.float32)

    def w(self, k):
        return _dev(self.sd[self.prefix + k], self.device, self.dtype)

    def conv(self, k):
        return (_dev(ops.pack_conv3x3(self.sd[self.prefix + k + ".weight"]), self.device, self.dtype),
                self.f32(k + ".bias"))

    def direct(self, k):
        return (self.f32(k + ".weight").permute(0, 2, 3, 1).contiguous(), self.f32(k + ".bias"))

    def resnet(self, p, cin, cout):
        r = dict(cin=cin, cout=cout, n1=(self.f32(p + ".norm1.weight"), self.f32(p + ".norm1.bias")),
                 c1=self.conv(p + ".conv1"), n2=(self.f32(p + ".norm2.weight"), self.f32(p + ".norm2.bias")),
                 c2=self.conv(p + ".conv2"))
        if cin != cout:
            r["sc"] = (self.w(p + ".conv_shortcut.weight").reshape(cout, cin).contiguous(),
                       self.f32(p + ".conv_shortcut.bias"))
        return r

    def attn(self, p):
        wq = torch.cat([self.sd[self.prefix + f"{p}.to_{n}.weight"] for n in "qkv"], 0)
        bq = torch.cat([self.sd[self.prefix + f"{p}.to_{n}.bias"] for n in "qkv"], 0)
        return dict(gn=(self.f32(p + ".group_norm.weight"), self.f32(p + ".group_norm.bias")),
                    qkv=(_dev(wq, self.device, self.dtype), _dev(bq, self.device, torch.float32)),
                    out=(self.w(p + ".to_out.0.weight"), self.f32(p + ".to_out.0.bias")))


def run_resnet(r, x, n, H, W, dtype, device, stats=None):
    """ResnetBlock2D.  stats: GroupNorm statistics of x written by its producer (ops.GnStats), None = computed by
    the GroupNorm.  Returns (out, GnStats of out from conv2's epilogue, for the next GroupNorm)."""
    HW = H * W
    # norm -> SiLU -> conv pairs: the GroupNorm folded into the halo-staged conv's staging pass where it applies
    # (ops.gn_conv3x3), else its own pass
    s1 = ops.GnStats(n, HW, 32, x.device)
    h = ops.gn_conv3x3(x, *r["n1"], *r["c1"], n, H, W, 1e-6, silu=True, stats=stats, gn=s1)
    sc = ops.gemm(x, r["sc"][0], bias=r["sc"][1]) if "sc" in r else x
    s2 = ops.GnStats(n, HW, 32, x.device)
    return ops.gn_conv3x3(h, *r["n2"], *r["c2"], n, H, W, 1e-6, silu=True, stats=s1, residual=sc, gn=s2), s2


def run_attn(a, x, n, H, W, stats=None):
    """Single-head d=C attention with residual (diffusers Attention, AttnProcessor2_0): GroupNorm -> fused QKV
    projection -> fd_flash_attn_d512 (no [T, T] buffers) -> out projection + residual.  stats / returns: as
    run_resnet."""
    C = a["out"][0].shape[0]
    T = H * W
    h = ops.group_norm(x, *a["gn"], n, T, C, 32, 1e-6, silu=False, stats=stats)
    qkv = ops.gemm(h, a["qkv"][0], bias=a["qkv"][1])  # [n*T, 3C]
    out = torch.empty((n * T, C), dtype=x.dtype, device=x.device)
    if C == 512:
        ops.flash_attn_d512(qkv, out, n, T, C ** -0.5)
    else:  # materialised fallback for other head widths (not used by the SDXL VAE)
        Tp = (T + 63) // 64 * 64  # the P.V GEMM contracts over T: pad K to the kernel's 64 granule with zeros
        S = torch.empty((T, T), dtype=torch.float32, device=x.device)
        P = torch.zeros((T, Tp), dtype=x.dtype, device=x.device)
        Vt = torch.zeros((C, Tp), dtype=x.dtype, device=x.device)
        for i in range(n):
            q = qkv[i * T:(i + 1) * T]
            ops.gemm(q, q[:, C:], out=S, M=T, N=T, K=C, lda=3 * C, ldw=3 * C, alpha=C ** -0.5,
                     out_dtype=torch.float32)
            ops.softmax_rows(S, P, T, T, 1.0, ldp=Tp)
            ops.transpose(q[:, 2 * C:], 3 * C, Vt, Tp, T, C)
            ops.gemm(P, Vt, out=out[i * T:(i + 1) * T], K=Tp)
    so = ops.GnStats(n, T, 32, x.device)
    return ops.gemm(out, a["out"][0], bias=a["out"][1], residual=x, gn=so), so


class HipEncoder:
    """VAE encoder trunk (with_out=True: + conv_norm_out/conv_out/quant_conv -> moments [HW, 8]) or the
    FaithDiff denoise encoder (with_out=False -> mid-block features [HW, 512], ext:145-148)."""

    def __init__(self, sd, prefix="", with_out=True, device="cuda", dtype=torch.float16, quant_sd=None):
        L.require_device()
        t = _Trunk(sd, prefix, device, dtype)
        self.device, self.dtype = t.device, dtype
        ch = arch.VAE_CH
        self.conv_in = t.direct("conv_in")
        self.blocks = []
        prev = ch[0]
        for i, c in enumerate(ch):
            rs = [t.resnet(f"down_blocks.{i}.resnets.{j}", prev if j == 0 else c, c) for j in range(2)]
            ds = t.conv(f"down_blocks.{i}.downsamplers.0.conv") if i < 3 else None
            self.blocks.append((rs, ds))
            prev = c
        self.mid = (t.resnet("mid_block.resnets.0", 512, 512), t.attn("mid_block.attentions.0"),
                    t.resnet("mid_block.resnets.1", 512, 512))
        self.with_out = with_out
        if with_out:
            self.norm_out = (t.f32("conv_norm_out.weight"), t.f32("conv_norm_out.bias"))
            self.conv_out = t.conv("conv_out")
            q = quant_sd
            self.quant = (_dev(q["quant_conv.weight"], self.device, torch.float32).permute(0, 2, 3, 1).contiguous(),
                          _dev(q["quant_conv.bias"], self.device, torch.float32))
        # FaithDiff Encoder tiling knobs (ext:70-73); set via set_encoder_tile_settings / enable_tiling
        self.tile_sample_min_size = 1024
        self.tile_latent_min_size = int(self.tile_sample_min_size / 8)
        self.tile_overlap_factor = 0.25
        self.use_tiling = False
        self.graphs = GraphCache()

    def encode_graphed(self, x, n, H, W):
        """encode() through the graph cache (fdhip/graphs.py); returns the graph's static output."""
        return self.graphs.run(("enc", n, H, W, x.dtype), lambda x_: self.encode(x_, n, H, W), [x])

    def encode(self, x, n, H, W):
        """x: NHWC [n*H*W, 3] (dtype) in [-1, 1].  Returns NHWC [n*(H/8)*(W/8), 8 or 512]."""
        h = ops.conv_direct(x, *self.conv_in, n, H, W, 3, 3, 1, 1, out_dtype=self.dtype)
        hh, ww = H, W
        st = None  # GroupNorm statistics of h from its producer (ops.GnStats)
        for rs, ds in self.blocks:
            for r in rs:
                h, st = run_resnet(r, h, n, hh, ww, self.dtype, self.device, st)
            if ds is not None:
                st = ops.GnStats(n, (hh // 2) * (ww // 2), 32, h.device)
                h = ops.conv3x3(h, *ds, n, hh, ww, stride=2, pad=0, gn=st)
                hh, ww = hh // 2, ww // 2
        h, st = run_resnet(self.mid[0], h, n, hh, ww, self.dtype, self.device, st)
        h, st = run_attn(self.mid[1], h, n, hh, ww, st)
        h, st = run_resnet(self.mid[2], h, n, hh, ww, self.dtype, self.device, st)
        if self.with_out:
            h = ops.group_norm(h, *self.norm_out, n, hh * ww, 512, 32, 1e-6, silu=True, stats=st)
            h = ops.conv3x3(h, *self.conv_out, n, hh, ww)
            h = ops.conv_direct(h, *self.quant, n, hh, ww, 8, 1, 1, 0, out_dtype=self.dtype)
        return h


class HipDecoder:
    def __init__(self, sd, device="cuda", dtype=torch.float16):
        L.require_device()
        t = _Trunk(sd, "", device, dtype)
        self.device, self.dtype = t.device, dtype
        self.post_quant = t.direct("post_quant_conv")
        self.conv_in = t.direct("decoder.conv_in")
        self.mid = (t.resnet("decoder.mid_block.resnets.0", 512, 512), t.attn("decoder.mid_block.attentions.0"),
                    t.resnet("decoder.mid_block.resnets.1", 512, 512))
        rch = tuple(reversed(arch.VAE_CH))
        self.blocks = []
        prev = rch[0]
        for i, c in enumerate(rch):
            rs = [t.resnet(f"decoder.up_blocks.{i}.resnets.{j}", prev if j == 0 else c, c) for j in range(3)]
            us = None
            if i < 3:  # Upsample2D: the 3x3 form and the four-phase form (ops.pack_conv3x3_up2)
                k = f"decoder.up_blocks.{i}.upsamplers.0.conv"
                us = t.conv(k) + (_dev(ops.pack_conv3x3_up2(t.sd[t.prefix + k + ".weight"]), self.device, dtype),)
            self.blocks.append((rs, us))
            prev = c
        self.norm_out = (t.f32("decoder.conv_norm_out.weight"), t.f32("decoder.conv_norm_out.bias"))
        self.conv_out = t.conv("decoder.conv_out")
        # conv_out (128 -> 3): FD_VAE_NARROW=1 runs it on the direct narrow-N kernel (fd_conv3x3_narrow_gn, fp32
        # weights, 16-row strips) with conv_norm_out + SiLU applied in its staging; 0: GroupNorm pass + implicit GEMM
        self.conv_out32 = (ops.pack_conv3x3(t.sd[t.prefix + "decoder.conv_out.weight"]).float().to(self.device),
                           self.conv_out[1])
        self.graphs = GraphCache()

    def decode_graphed(self, z, n, h, w):
        """decode() through the graph cache (fdhip/graphs.py); returns the graph's static output."""
        return self.graphs.run(("dec", n, h, w, z.dtype), lambda z_: self.decode(z_, n, h, w), [z])

    def decode(self, z, n, h, w):
        """z: NHWC [n*h*w, 4] (already divided by scaling_factor).  Returns NHWC [n*8h*8w, 3] (dtype)."""
        x = ops.conv_direct(z, *self.post_quant, n, h, w, 4, 1, 1, 0, out_dtype=self.dtype)
        x = ops.conv_direct(x, *self.conv_in, n, h, w, 4, 3, 1, 1, out_dtype=self.dtype)
        x, st = run_resnet(self.mid[0], x, n, h, w, self.dtype, self.device)
        x, st = run_attn(self.mid[1], x, n, h, w, st)
        x, st = run_resnet(self.mid[2], x, n, h, w, self.dtype, self.device, st)
        hh, ww = h, w
        for rs, us in self.blocks:
            for r in rs:
                x, st = run_resnet(r, x, n, hh, ww, self.dtype, self.device, st)
            if us is not None:
                st = ops.GnStats(n, 4 * hh * ww, 32, x.device)
                if knobs.get("FD_UP2_PHASE") and ops.up2_phase_ok(x, us[2], n, hh, ww):
                    x = ops.conv3x3_up2(x, us[2], us[1], n, hh, ww, gn=st)
                else:
                    x = ops.conv3x3(x, us[0], us[1], n, hh, ww, upsample=True, gn=st)
                hh, ww = hh * 2, ww * 2
        if knobs.get("FD_VAE_NARROW"):  # conv_norm_out + SiLU folded into the narrow conv_out's staging
            aff = ops.group_norm_affine(x, *self.norm_out, n, hh * ww, 128, 32, 1e-6, stats=st)
            return ops.conv3x3_narrow(x, *self.conv_out32, n, hh, ww, gn_in=(aff, True))
        x = ops.group_norm(x, *self.norm_out, n, hh * ww, 128, 32, 1e-6, silu=True, stats=st)
        return ops.conv3x3(x, *self.conv_out, n, hh, ww)
