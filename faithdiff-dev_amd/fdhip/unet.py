"""SDXL UNet + FaithDiff conditioning extras on the HIP kernel library (bf16, NHWC).

Forward order follows FaithDiff/models/unet_2d_condition_vae_extension.py:480-697:
time/aug embedding (:543-561) -> conv_in (:571) -> condition_embedding + information transformer +
spatial_ch_projs (:572-579) -> down blocks (:611-630) -> mid (:641-655) -> up blocks (:660-684) ->
GN + SiLU + conv_out (:686-690).  The diffusers blocks follow SURVEY Appendix B.1.

MI355X-specific structure (not a translation of the reference's module graph):
  * activations stay NHWC bf16 [M = B*H*W, C]; every Linear and 3x3/1x1 conv is one fd_gemm launch with
    its bias / time-embedding add / residual / GEGLU fused into the MFMA epilogue;
  * the 22 ResnetBlock2D time_emb_proj Linears are one GEMM (SiLU(emb) x [sum C_out, 1280]^T);
  * attn1 uses one fused QKV projection; attn2's K/V projections of the prompt embeddings for all 70
    transformer blocks are ONE GEMM per forward ([ncfg*77, 2048] x [166400, 2048]^T), and one K/V pair
    [neg, pos] serves every tile of a batched forward (kv_mod = CFG width);
  * the up-block skip concat is folded into the conv1 gather (two-source implicit GEMM) after the
    GroupNorm reads the materialised concat;
  * the transformer blocks' LayerNorms (norm1/2/3) are folded into the GEMM pair around them: the
    residual-stream GEMM (proj_in, attn out-projections, ff out) also writes per-row (sum, sumsq)
    partials, and the next projection runs on the raw stream with W * gamma, finishing
    rstd * (acc - mean * rowsum(W * gamma)) + W . beta + b in its epilogue (no LayerNorm launches; FD_LN_FOLD=0
    restores them).
Rows are [tile0 uncond, tile0 cond, tile1 uncond, ...]: several TLC tiles can share one forward.
"""
import torch

from . import arch, knobs
from . import lib as L
from . import ops
from .graphs import GraphCache


def _dev(t, device, dtype):
    return t.to(device=device, dtype=dtype).contiguous()


class HipUNet:
    def __init__(self, sd, device="cuda", dtype=torch.bfloat16, fp8_mfma=False):
        """fp8_mfma: the transformer Linears (proj_in/out, QKV, attention out-projections, GEGLU, ff out) run
        on the e4m3 MFMA (fd_gemm_e4m3) with the weights as e4m3 bytes and activations quantized per row --
        the use_fp8 / quantize_8bit model.  Meant for weights already rounded by
        arch.quantize_e4m3 (then the byte packing is exact); convolutions stay on the 16-bit MFMA, and the
        separate LayerNorm path is used (the fold needs W * gamma, which is not an e4m3 weight)."""
        L.require_device()
        self.fp8_mfma = bool(fp8_mfma)
        # (MX e4m3 activations everywhere -- LayerNorm / flash attention writing OCP MX, FD_FP8_MX -- measured slower
        # than per-row scales (C2 21.00 vs 20.88 ms, C4 69.5 vs 71.3 tile-steps/s: profiles/r03_fp8_ab_*.json,
        # r05af_c4_mx_ab.txt) and was removed in round 6; MX stays where it is free, below)
        # MX output straight from the GEGLU epilogue (forces 256 x 128 tiles; profiles/r03_f8_tiles_mx.jsonl: 48.1 vs
        # 39.7 + a 2048 x 5120 quantization for the 256 x 160 bf16 form); FD_FP8_MX_GEGLU=1 turns it on (A/B)
        self.fp8_mx_geglu = knobs.get("FD_FP8_MX_GEGLU") == 1
        # per-row form with MX only where it is free: flash attention writes its output as MX and the out-projections
        # (K = C: the MX GEMM's speed, profiles/r03_f8_tiles_mx.jsonl) read it, removing the two activation
        # quantization launches per block.  C2 step on one box, alternated: 20.57 / 20.57 ms vs 20.65 / 20.67 per-row
        # everywhere vs 20.84 / 20.89 MX everywhere (profiles/r03_fp8_mxattn_ab_*.json).  FD_FP8_MX_ATTN=0: per-row
        self.fp8_mx_attn = self.fp8_mfma and knobs.get("FD_FP8_MX_ATTN") != 0
        self.device, self.dtype = torch.device(device), dtype
        f32 = torch.float32
        W = lambda k: _dev(sd[k], self.device, dtype)  # noqa: E731
        Fp = lambda k: _dev(sd[k], self.device, f32)  # noqa: E731
        self.W, self.Fp = W, Fp

        # time / add embeddings
        self.te = [(W("time_embedding.linear_1.weight"), Fp("time_embedding.linear_1.bias")),
                   (W("time_embedding.linear_2.weight"), Fp("time_embedding.linear_2.bias"))]
        self.ae = [(W("add_embedding.linear_1.weight"), Fp("add_embedding.linear_1.bias")),
                   (W("add_embedding.linear_2.weight"), Fp("add_embedding.linear_2.bias"))]
        self.conv_in = (Fp("conv_in.weight").permute(0, 2, 3, 1).contiguous(), Fp("conv_in.bias"))

        # all resnet time_emb_proj in one matrix
        temb_w, temb_b = [], []
        self._temb_off = 0

        def resnet(p, cin, cout):
            r = dict(cin=cin, cout=cout,
                     n1=(Fp(p + ".norm1.weight"), Fp(p + ".norm1.bias")),
                     c1=(_dev(ops.pack_conv3x3(sd[p + ".conv1.weight"]), self.device, dtype), Fp(p + ".conv1.bias")),
                     n2=(Fp(p + ".norm2.weight"), Fp(p + ".norm2.bias")),
                     c2=(_dev(ops.pack_conv3x3(sd[p + ".conv2.weight"]), self.device, dtype), Fp(p + ".conv2.bias")),
                     toff=self._temb_off)
            temb_w.append(sd[p + ".time_emb_proj.weight"])
            temb_b.append(sd[p + ".time_emb_proj.bias"])
            self._temb_off += cout
            if cin != cout:
                r["sc"] = (_dev(sd[p + ".conv_shortcut.weight"].reshape(cout, cin), self.device, dtype),
                           Fp(p + ".conv_shortcut.bias"))
            return r

        self.ln_fold = knobs.get("FD_LN_FOLD") != 0 and not self.fp8_mfma
        # attn2 as two GEMMs against per-prompt products (scores with the softmax in the epilogue, then P . (V W_o)):
        # the folded 16-bit model only (FD_XATTN_GEMM=0: Q projection + flash attention + out-projection)
        self.xattn = self.ln_fold and knobs.get("FD_XATTN_GEMM") != 0
        self._pbuf = {}

        # GroupNorm statistics from the producing conv / GEMM epilogue (256-row tiles; FD_UNET_GN_EPI=0: off)
        self.gn_epi = knobs.get("FD_UNET_GN_EPI") != 0
        self.cat_gn = self.gn_epi and knobs.get("FD_UNET_CAT_GN") != 0
        self._gn_src = None
        # transformer Linear weights: e4m3 bytes for the fp8 MFMA, else the compute dtype
        LW = (lambda t: ops.pack_e4m3(t.to(self.device))) if self.fp8_mfma else \
            (lambda t: _dev(t, self.device, dtype))  # noqa: E731

        def fold(w, n, bias=None):  # (W * gamma, rowsum, W . beta + b) on the device
            dev = lambda t: t.to(self.device)  # noqa: E731
            return ops.fold_layer_norm(dev(w), dev(sd[n + ".weight"]), dev(sd[n + ".bias"]),
                                       None if bias is None else dev(bias), dtype)

        def t2d(p, c, layers):
            blocks = []
            for i in range(layers):
                b = f"{p}.transformer_blocks.{i}"
                ffw, ffb = ops.pack_geglu(sd[b + ".ff.net.0.proj.weight"], sd[b + ".ff.net.0.proj.bias"])
                if self.ln_fold:
                    q2_f = fold(sd[b + ".attn2.to_q.weight"], b + ".norm2")
                    blocks.append(dict(
                        qkv_f=fold(torch.cat([sd[f"{b}.attn1.to_{n}.weight"] for n in "qkv"], 0), b + ".norm1"),
                        o1=(W(b + ".attn1.to_out.0.weight"), Fp(b + ".attn1.to_out.0.bias")),
                        q2_f=q2_f,
                        # cross-attention as two GEMMs (set_context / _t2d_folded): W_q'^T for the per-prompt score
                        # matrix, W_q . beta for its bias
                        q2_t=q2_f[0].t().contiguous() if self.xattn else None, q2_d=q2_f[2],
                        kv2=_dev(torch.cat([sd[b + ".attn2.to_k.weight"], sd[b + ".attn2.to_v.weight"]], 0),
                                 self.device, dtype),
                        o2=(W(b + ".attn2.to_out.0.weight"), Fp(b + ".attn2.to_out.0.bias")),
                        ff1_f=fold(ffw, b + ".norm3", ffb),
                        ff2=(W(b + ".ff.net.2.weight"), Fp(b + ".ff.net.2.bias")),
                    ))
                    continue
                blocks.append(dict(
                    n1=(Fp(b + ".norm1.weight"), Fp(b + ".norm1.bias")),
                    qkv=LW(torch.cat([sd[f"{b}.attn1.to_{n}.weight"] for n in "qkv"], 0)),
                    o1=(LW(sd[b + ".attn1.to_out.0.weight"]), Fp(b + ".attn1.to_out.0.bias")),
                    n2=(Fp(b + ".norm2.weight"), Fp(b + ".norm2.bias")),
                    q2=LW(sd[b + ".attn2.to_q.weight"]),
                    kv2=_dev(torch.cat([sd[b + ".attn2.to_k.weight"], sd[b + ".attn2.to_v.weight"]], 0), self.device,
                             dtype),
                    o2=(LW(sd[b + ".attn2.to_out.0.weight"]), Fp(b + ".attn2.to_out.0.bias")),
                    n3=(Fp(b + ".norm3.weight"), Fp(b + ".norm3.bias")),
                    ff1=(LW(ffw), _dev(ffb, self.device, f32)),
                    ff2=(LW(sd[b + ".ff.net.2.weight"]), Fp(b + ".ff.net.2.bias")),
                ))
            return dict(c=c, heads=c // 64, norm=(Fp(p + ".norm.weight"), Fp(p + ".norm.bias")),
                        pin=(LW(sd[p + ".proj_in.weight"]), Fp(p + ".proj_in.bias")),
                        pout=(LW(sd[p + ".proj_out.weight"]), Fp(p + ".proj_out.bias")), blocks=blocks)

        C, Lr = arch.UNET_CH, arch.UNET_LAYERS
        self.down = []
        prev = C[0]
        for i in range(3):
            blk = dict(resnets=[], attns=[], ds=None)
            for j in range(2):
                blk["resnets"].append(resnet(f"down_blocks.{i}.resnets.{j}", prev if j == 0 else C[i], C[i]))
                if Lr[i]:
                    blk["attns"].append(t2d(f"down_blocks.{i}.attentions.{j}", C[i], Lr[i]))
            if i < 2:
                p = f"down_blocks.{i}.downsamplers.0.conv"
                blk["ds"] = (_dev(ops.pack_conv3x3(sd[p + ".weight"]), self.device, dtype), Fp(p + ".bias"))
            self.down.append(blk)
            prev = C[i]
        self.mid = dict(r0=resnet("mid_block.resnets.0", C[2], C[2]), attn=t2d("mid_block.attentions.0", C[2], Lr[2]),
                        r1=resnet("mid_block.resnets.1", C[2], C[2]))
        skips = arch.up_skip_channels()
        self.up = []
        prev = C[2]
        for i in range(3):
            lvl = 2 - i
            co = C[lvl]
            blk = dict(resnets=[], attns=[], us=None)
            for j in range(3):
                blk["resnets"].append(resnet(f"up_blocks.{i}.resnets.{j}", (prev if j == 0 else co) + skips[i][j], co))
                if Lr[lvl]:
                    blk["attns"].append(t2d(f"up_blocks.{i}.attentions.{j}", co, Lr[lvl]))
            if i < 2:
                p = f"up_blocks.{i}.upsamplers.0.conv"
                blk["us"] = (_dev(ops.pack_conv3x3(sd[p + ".weight"]), self.device, dtype), Fp(p + ".bias"),
                             _dev(ops.pack_conv3x3_up2(sd[p + ".weight"]), self.device, dtype))
            self.up.append(blk)
            prev = co
        self.norm_out = (Fp("conv_norm_out.weight"), Fp("conv_norm_out.bias"))
        self.conv_out = (_dev(ops.pack_conv3x3(sd["conv_out.weight"]), self.device, dtype), Fp("conv_out.bias"))
        self.temb_w = _dev(torch.cat(temb_w, 0), self.device, dtype)
        self.temb_b = _dev(torch.cat(temb_b, 0), self.device, f32)
        self.temb_total = self._temb_off

        # FaithDiff extras
        self.has_extras = "spatial_ch_projs.weight" in sd
        if self.has_extras:
            self.cne = dict(norm=(Fp("condition_embedding.norm_in.weight"), Fp("condition_embedding.norm_in.bias")),
                            cin=(_dev(ops.pack_conv3x3(sd["condition_embedding.conv_in.weight"]), self.device, dtype),
                                 Fp("condition_embedding.conv_in.bias")),
                            cout=(_dev(ops.pack_conv3x3(sd["condition_embedding.conv_out.weight"]), self.device,
                                       dtype), Fp("condition_embedding.conv_out.bias")))
            self.itl = []
            for i in range(2):
                p = f"information_transformer_layes.{i}"
                self.itl.append(dict(
                    ln1=(Fp(p + ".ln_1.weight"), Fp(p + ".ln_1.bias")),
                    inp=(W(p + ".attn.in_proj_weight"), Fp(p + ".attn.in_proj_bias")),
                    outp=(W(p + ".attn.out_proj.weight"), Fp(p + ".attn.out_proj.bias")),
                    ln2=(Fp(p + ".ln_2.weight"), Fp(p + ".ln_2.bias")),
                    fc=(W(p + ".mlp.c_fc.weight"), Fp(p + ".mlp.c_fc.bias")),
                    proj=(W(p + ".mlp.c_proj.weight"), Fp(p + ".mlp.c_proj.bias"))))
                if self.ln_fold:  # ln_1 / ln_2 folded into in_proj / c_fc (partials from out_proj / c_proj epilogues)
                    self.itl[-1]["inp_f"] = fold(sd[p + ".attn.in_proj_weight"], p + ".ln_1", sd[p + ".attn.in_proj_bias"])
                    self.itl[-1]["fc_f"] = fold(sd[p + ".mlp.c_fc.weight"], p + ".ln_2", sd[p + ".mlp.c_fc.bias"])
            self.scp = (W("spatial_ch_projs.weight"), Fp("spatial_ch_projs.bias"))
        # all 70 attn2 K/V projections of the prompt as ONE [sum 2C, 2048] weight: one GEMM per forward
        kv_ws, off = [], 0
        for t in self._all_t2d():
            for b in t["blocks"]:
                b["kv_off"] = off
                off += b["kv2"].shape[0]
                kv_ws.append(b.pop("kv2"))
        self.kv_w = torch.cat(kv_ws, 0).contiguous()
        self.kv_total = off
        self.ctx = None
        self.ncfg = None
        self.npairs = 1
        self._kv = None
        self.graphs = GraphCache()

    # ------------------------------------------------------------------------------------------ context
    def _all_t2d(self):
        for blk in self.down:
            yield from blk["attns"]
        yield self.mid["attn"]
        for blk in self.up:
            yield from blk["attns"]

    def set_context(self, ctx, ncfg=None):
        """ctx: [npairs * ncfg, 77, 2048] prompt embeddings ([neg, pos] under CFG; ncfg defaults to all rows, one
        prompt pair).  Projects them through all 70 attn2 to_k/to_v at once into ``self._kv`` [rows*77, sum 2C] --
        once per prompt, not per forward: the reference recomputes attn2's K/V of the same prompt in every UNet call
        of the loop (pipeline:1350, 20 steps x every tile); the product is identical, the GEMM (105 GFLOP per pair,
        ~0.23 ms) runs once.
        One pair (npairs = 1): every CFG pair of a forward (the TLC tiles of one image) attends to it (kv_mod =
        ncfg).  Several pairs (images batched, one tile each): CFG pair j of a forward attends to prompt pair
        kv_pair0 + j (see forward), i.e. K/V block = row block (kv_mod = 0).
        The device buffers keep their addresses across calls with the same shape (new prompts are copied in),
        so the hipGraphs captured by run() stay valid; a new shape drops them."""
        c = ctx.to(device=self.device, dtype=self.dtype).reshape(-1, ctx.shape[-1])
        ncfg = ctx.shape[0] if ncfg is None else int(ncfg)
        if ctx.shape[0] % ncfg:
            raise ValueError(f"set_context: {ctx.shape[0]} prompt rows are not whole CFG groups of {ncfg}")
        if self.ctx is not None and self.ctx.shape == c.shape and self.ncfg == ncfg:
            self.ctx.copy_(c)
        else:
            self.ctx = c.contiguous().clone()
            self._kv = torch.empty((c.shape[0], self.kv_total), dtype=self.dtype, device=self.device)
            self.graphs.clear()
        new_shape = self.ncfg != ncfg or getattr(self, "Lk", None) != ctx.shape[1]
        self.ncfg, self.Lk = ncfg, ctx.shape[1]
        self.npairs = ctx.shape[0] // ncfg
        ops.gemm(self.ctx, self.kv_w, out=self._kv)  # [rows*77, sum 2C]: every attn2 K/V
        if self.xattn and self.Lk <= self.XSLOT:
            self._xattn_prep(ctx.shape[0], new_shape)

    XSLOT = ops.XSLOT

    def _xattn_prep(self, R, realloc):
        """Cross-attention as two GEMMs (ops.XAttnMats / xattn_prepare): per prompt row and attn2 block, the score
        matrix 0.125 K W_q' with its LayerNorm-fold constants and V W_o -- the prompt-only products of the reference's
        attn2 (diffusers Attention: to_q, SDPA, to_out, recomputed every UNet call at pipeline:1350) taken out of the
        denoise loop; each forward then runs two launches per block instead of three."""
        Lk, kv, ldkv = self.Lk, self._kv, self.kv_total
        for t in self._all_t2d():
            for b in t["blocks"]:
                if realloc or b.get("xm") is None or b["xm"].R != R:
                    b["xm"] = ops.XAttnMats(R, t["c"], t["heads"], self.dtype, self.device)
                off = b["kv_off"]
                ops.xattn_prepare(b["xm"], kv[:, off:], kv[:, off + t["c"]:], ldkv, Lk, b["q2_t"], b["q2_d"],
                                  b["o2"][0])

    # ------------------------------------------------------------------------------------------ blocks
    def _resnet(self, r, x, B, H, Wd, temb, x2=None, C1=None):
        """x: [M, cin] (or concat(x [M,C1], x2) when x2 is given)."""
        HW = H * Wd
        if x2 is not None:
            cat = torch.empty((B * HW, r["cin"]), dtype=self.dtype, device=self.device)
            s0 = self._gn_new(B, HW) if self.cat_gn else None  # the concat also writes norm1's statistics
            ops.concat_channels(x, C1, x2, r["cin"] - C1, cat, B * HW, gn=s0)
            x = cat
            self._gn_src = (cat, s0) if s0 is not None and s0.done else None
        # norm1 -> SiLU -> conv1 (+ time embedding), norm2 -> SiLU -> conv2 (+ shortcut): each GroupNorm folded into
        # the halo-staged conv's staging pass where that kernel takes the conv (ops.gn_conv3x3), else its own pass
        s1 = self._gn_new(B, HW)
        h = ops.gn_conv3x3(x, *r["n1"], *r["c1"], B, H, Wd, 1e-5, silu=True, stats=self._gn_stats_of(x),
                           rowbias=temb[:, r["toff"]:r["toff"] + r["cout"]], gn=s1)
        sc = ops.gemm(x, r["sc"][0], bias=r["sc"][1]) if "sc" in r else x
        s2 = self._gn_new(B, HW)
        out = ops.gn_conv3x3(h, *r["n2"], *r["c2"], B, H, Wd, 1e-5, silu=True, stats=s1, residual=sc, gn=s2)
        self._gn_src = (out, s2) if s2 is not None else None
        return out

    def _gn_new(self, B, HW):
        """GroupNorm statistics asked of the next conv / GEMM's epilogue (ops.GnStats; None when FD_UNET_GN_EPI=0)."""
        return ops.GnStats(B, HW, 32, self.device) if self.gn_epi else None

    def _gn_stats_of(self, x):
        """The statistics the producer of x wrote in its epilogue (resnet conv2 / transformer proj_out), if x is
        that output; consumed once."""
        src, self._gn_src = self._gn_src, None
        return src[1] if src is not None and src[0] is x else None

    def _t2d(self, t, x, B, H, Wd):
        C, heads, HW = t["c"], t["heads"], H * Wd
        M = B * HW
        h = ops.group_norm(x, *t["norm"], B, HW, C, 32, 1e-6, silu=False, stats=self._gn_stats_of(x))
        if self.ln_fold:
            return self._t2d_folded(t, x, h, B, H, Wd)
        lin = self._lin
        h = lin(h, t["pin"][0], bias=t["pin"][1])
        qkv = torch.empty((M, 3 * C), dtype=self.dtype, device=self.device)
        att = torch.empty((M, C), dtype=self.dtype, device=self.device)
        att8 = ops.MX(M, C, self.device) if self.fp8_mx_attn else None
        if self.fp8_mfma:  # LayerNorm writes e4m3 rows + scales straight into the fp8 GEMM's A operand
            q8 = torch.empty((M, C), dtype=torch.uint8, device=self.device)
            s8 = torch.empty((M,), dtype=torch.float32, device=self.device)

            def ln_lin(norm, w, bias=None, out=None, act="none"):
                ops.layer_norm_e4m3(h, *norm, 1e-5, q=q8, scale=s8)
                return ops.gemm_e4m3(q8, s8, w, out=out, bias=bias, act=act, out_dtype=self.dtype)
        else:
            n = torch.empty((M, C), dtype=self.dtype, device=self.device)

            def ln_lin(norm, w, bias=None, out=None, act="none"):
                ops.layer_norm(h, *norm, 1e-5, out=n)
                return lin(n, w, bias=bias, out=out, act=act)
        for b in t["blocks"]:
            ln_lin(b["n1"], b["qkv"], out=qkv)
            kv = self._kv[self._kv_row0:, b["kv_off"]:]  # [ncfg*77, ...] view; K at +0, V at +C, row stride kv_total
            Lk, ldkv = self.Lk, self.kv_total
            if att8 is not None:  # attention output as MX e4m3 -> MX out-projection GEMM (no quantization launch)
                ops.flash_attn_mx(qkv, qkv[:, C:], qkv[:, 2 * C:], att8, B, heads, HW, HW, 3 * C, 3 * C, 3 * C,
                                  HW * 3 * C, HW * 3 * C, HW * 3 * C, kv_mod=0, scale=0.125)
                ops.gemm_mx(att8, b["o1"][0], bias=b["o1"][1], residual=h, out=h)
                ln_lin(b["n2"], b["q2"], out=qkv[:, :C])
                ops.flash_attn_mx(qkv, kv, kv[:, C:], att8, B, heads, HW, Lk, 3 * C, ldkv, ldkv,
                                  HW * 3 * C, Lk * ldkv, Lk * ldkv, kv_mod=self._kv_mod, scale=0.125)
                ops.gemm_mx(att8, b["o2"][0], bias=b["o2"][1], residual=h, out=h)
                ff = ln_lin(b["n3"], b["ff1"][0], bias=b["ff1"][1], act="geglu")
                lin(ff, b["ff2"][0], bias=b["ff2"][1], residual=h, out=h)
                continue
            ops.flash_attn(qkv, qkv[:, C:], qkv[:, 2 * C:], att, B, heads, HW, HW, 3 * C, 3 * C, 3 * C, C,
                           HW * 3 * C, HW * 3 * C, HW * 3 * C, HW * C, kv_mod=0, scale=0.125)
            lin(att, b["o1"][0], bias=b["o1"][1], residual=h, out=h)
            ln_lin(b["n2"], b["q2"], out=qkv[:, :C])  # row stride 3C (the view's)
            ops.flash_attn(qkv, kv, kv[:, C:], att, B, heads, HW, Lk, 3 * C, ldkv, ldkv, C,
                           HW * 3 * C, Lk * ldkv, Lk * ldkv, HW * C, kv_mod=self._kv_mod, scale=0.125)
            lin(att, b["o2"][0], bias=b["o2"][1], residual=h, out=h)
            ff = ln_lin(b["n3"], b["ff1"][0], bias=b["ff1"][1], act="geglu")
            lin(ff, b["ff2"][0], bias=b["ff2"][1], residual=h, out=h)
        return self._proj_out(t, h, x, B, HW)

    def _proj_out(self, t, h, x, B, HW):
        """proj_out + residual; its epilogue also writes the next GroupNorm's statistics (16-bit GEMM)."""
        if self.fp8_mfma:
            return ops.linear_e4m3(h, t["pout"][0], bias=t["pout"][1], residual=x)
        s = self._gn_new(B, HW)
        out = ops.gemm(h, t["pout"][0], bias=t["pout"][1], residual=x, gn=s)
        self._gn_src = (out, s) if s is not None else None
        return out

    def _lin(self, x, w, bias=None, residual=None, out=None, act="none"):
        """A transformer Linear: fd_gemm (16-bit MFMA) or, for the fp8 model, fd_quant_rows_e4m3 + fd_gemm_e4m3."""
        if self.fp8_mfma:
            return ops.linear_e4m3(x, w, bias=bias, residual=residual, act=act, out=out)
        return ops.gemm(x, w, bias=bias, residual=residual, out=out, act=act,
                        ldc=None if out is None else out.stride(0))

    def _t2d_folded(self, t, x, hn, B, H, Wd):
        """_t2d with norm1/2/3 folded into the GEMMs (fd_gemm_params.ln_out / ln_in): `st` holds the
        per-row (sum, sumsq) partials of the current residual stream h, per 160 columns."""
        C, heads, HW = t["c"], t["heads"], H * Wd
        M = B * HW
        st = torch.empty((M, C // 160, 2), dtype=torch.float32, device=self.device)
        h = ops.gemm(hn, t["pin"][0], bias=t["pin"][1], ln_out=st)
        # the two-GEMM cross-attention needs its matrices (Lk <= 80) and whole 256-row groups per image
        xa = self.xattn and self.Lk <= self.XSLOT and HW % 256 == 0 and t["blocks"][0].get("xm") is not None
        qkv = torch.empty((M, 3 * C), dtype=self.dtype, device=self.device)
        att = torch.empty((M, C), dtype=self.dtype, device=self.device)
        nb = len(t["blocks"])
        for i, b in enumerate(t["blocks"]):
            w, c, d = b["qkv_f"]
            ops.gemm(h, w, bias=d, out=qkv, ln_in=st, ln_c=c)
            ops.flash_attn(qkv, qkv[:, C:], qkv[:, 2 * C:], att, B, heads, HW, HW, 3 * C, 3 * C, 3 * C, C,
                           HW * 3 * C, HW * 3 * C, HW * 3 * C, HW * C, kv_mod=0, scale=0.125)
            ops.gemm(att, b["o1"][0], bias=b["o1"][1], residual=h, out=h, ln_out=st)
            if xa:  # scores with the softmax in the epilogue, then P . V W_o + b_o + h (ops.xattn_attend)
                xm = b["xm"]
                ops.xattn_attend(h, st, xm, self._pbuf_get(M, xm.KP), HW, self._kv_mod, self._kv_row0 // self.Lk,
                                 self.Lk, b["o2"][1], st_out=st)
            else:
                w, c, d = b["q2_f"]
                ops.gemm(h, w, bias=d, out=qkv[:, :C], ldc=3 * C, ln_in=st, ln_c=c)
                kv = self._kv[self._kv_row0:, b["kv_off"]:]
                Lk, ldkv = self.Lk, self.kv_total
                ops.flash_attn(qkv, kv, kv[:, C:], att, B, heads, HW, Lk, 3 * C, ldkv, ldkv, C,
                               HW * 3 * C, Lk * ldkv, Lk * ldkv, HW * C, kv_mod=self._kv_mod, scale=0.125)
                ops.gemm(att, b["o2"][0], bias=b["o2"][1], residual=h, out=h, ln_out=st)
            w, c, d = b["ff1_f"]
            ff = ops.gemm(h, w, bias=d, act="geglu", ln_in=st, ln_c=c)
            ops.gemm(ff, b["ff2"][0], bias=b["ff2"][1], residual=h, out=h, ln_out=st if i + 1 < nb else None)
        return self._proj_out(t, h, x, B, HW)

    def _pbuf_get(self, M, KP):
        """The probability buffer of the two-GEMM cross-attention [M, KP]: persistent per shape (hipGraph replays
        reuse it) and zeroed once -- the score GEMM writes H*80 columns, the pad up to KP stays 0."""
        key = (M, KP)
        if key not in self._pbuf:
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError("two-GEMM cross-attention buffer first needed inside graph capture")
            self._pbuf[key] = torch.zeros((M, KP), dtype=self.dtype, device=self.device)
        return self._pbuf[key]

    def _cond_embed(self, cond, B, H, Wd, out=None):
        """condition_embedding (ext:528-534, the CNE: GroupNorm -> conv 512->512 + SiLU -> conv 512->320) of the
        image latents: [B*H*W, 512] -> [B*H*W, 320]."""
        HW = H * Wd
        c = ops.group_norm(cond, *self.cne["norm"], B, HW, 512, 32, 1e-6, silu=False)
        c = ops.conv3x3(c, *self.cne["cin"], B, H, Wd, act="silu")
        return ops.conv3x3(c, *self.cne["cout"], B, H, Wd, out=out)

    def cond_embed(self, cond, B, H, Wd, out=None):
        """The CNE of B rows of image-latent tiles, for forward(..., cond_embedded=True).  It depends only on
        the image latents, which are fixed for the whole denoise loop, so the pipeline computes it once per
        tile instead of in every step's forward (the reference recomputes it per UNet call, pipeline:1350).
        Run under the same per-tile grouping as forward, so the result is bitwise what forward computes."""
        assert self.has_extras and self.ncfg is not None
        with ops.tile_groups(B // self.ncfg):
            return self._cond_embed(cond, B, H, Wd, out=out)

    def _extras(self, x0, cond, B, H, Wd, embedded=False):
        HW = H * Wd
        M = B * HW
        ie = cond if embedded else self._cond_embed(cond, B, H, Wd)
        feat = torch.empty((M, 640), dtype=self.dtype, device=self.device)
        ops.concat_channels(x0, 320, ie, 320, feat, M)
        n = torch.empty_like(feat)
        att = torch.empty_like(feat)
        # FD_ITL_FOLD (with FD_LN_FOLD): ln_2 of each layer and ln_1 of the second folded into the next GEMM
        # (fd_gemm_params.ln_in), the per-row partials written by the out_proj / c_proj epilogues (ln_out); ln_1 of
        # the first layer (input: the concat) stays a pass
        fold = self.ln_fold and knobs.get("FD_ITL_FOLD") != 0 and "fc_f" in self.itl[0]
        st = torch.empty((M, 640 // 160, 2), dtype=torch.float32, device=self.device) if fold else None
        for li, lay in enumerate(self.itl):
            if fold and li > 0:
                w, c, d = lay["inp_f"]
                qkv = ops.gemm(feat, w, bias=d, ln_in=st, ln_c=c)
            else:
                ops.layer_norm(feat, *lay["ln1"], 1e-5, out=n)
                qkv = ops.gemm(n, lay["inp"][0], bias=lay["inp"][1])
            ops.mha_seq_axis(qkv, att, self.ncfg, B // self.ncfg, HW, 640, 8)
            ops.gemm(att, lay["outp"][0], bias=lay["outp"][1], residual=feat, out=feat, ln_out=st)
            if fold:
                w, c, d = lay["fc_f"]
                m = ops.gemm(feat, w, bias=d, act="quickgelu", ln_in=st, ln_c=c)
            else:
                ops.layer_norm(feat, *lay["ln2"], 1e-5, out=n)
                m = ops.gemm(n, lay["fc"][0], bias=lay["fc"][1], act="quickgelu")
            ops.gemm(m, lay["proj"][0], bias=lay["proj"][1], residual=feat, out=feat,
                     ln_out=st if fold and li + 1 < len(self.itl) else None)
        return feat

    # ------------------------------------------------------------------------------------------ forward
    def embeddings(self, t, time_ids, text_embeds, B):
        tf = torch.empty((B, 320), dtype=self.dtype, device=self.device)
        af = torch.empty((B, 2816), dtype=self.dtype, device=self.device)
        ops.time_features(t, time_ids, text_embeds, tf, af, B)
        h = ops.gemm(tf, self.te[0][0], bias=self.te[0][1], act="silu")
        emb = ops.gemm(h, self.te[1][0], bias=self.te[1][1], out_dtype=torch.float32)
        h = ops.gemm(af, self.ae[0][0], bias=self.ae[0][1], act="silu")
        emb = ops.gemm(h, self.ae[1][0], bias=self.ae[1][1], residual=emb, out_dtype=torch.float32)
        semb = torch.empty((B, 1280), dtype=self.dtype, device=self.device)
        ops.unary(emb, semb, "silu")
        return ops.gemm(semb, self.temb_w, bias=self.temb_b, out_dtype=torch.float32)  # [B, sum C_out]

    def run(self, x, t, time_ids, text_embeds, cond, B, H, Wd, add_sample=True, cond_embedded=False, kv_pair0=0):
        """forward() through the graph cache (fdhip/graphs.py): eager on the first call of a shape, captured on
        the second, one hipGraph replay after that.  The result is the graph's static output buffer (valid
        until the next run() of the same shape).  This is what the pipeline's denoise loop and bench.py call."""
        key = self._graph_key(B, H, Wd, add_sample, cond is None, cond_embedded, x.dtype, kv_pair0)
        return self.graphs.run(key, lambda *a: self.forward(*a, B, H, Wd, add_sample=add_sample,
                                                            cond_embedded=cond_embedded, kv_pair0=kv_pair0),
                               [x, t, time_ids, text_embeds, cond])

    def _graph_key(self, B, H, Wd, add_sample, no_cond, cond_embedded, dtype, kv_pair0):
        return ("unet", B, H, Wd, bool(add_sample), bool(no_cond), bool(cond_embedded), dtype, self.npairs > 1,
                kv_pair0)

    def graph_inputs(self, B, H, Wd, add_sample=True, cond_embedded=False, kv_pair0=0, has_cond=True):
        """The static input buffers [x, t, time_ids, text_embeds, cond] of run()'s captured graph for this call
        shape, or None before the capture.  The denoise loop writes the step's latent tile and timestep straight
        into them (fd_tlc_scale_input_t), so a replay needs no input copies."""
        return self.graphs.static_inputs(self._graph_key(B, H, Wd, add_sample, not has_cond, cond_embedded,
                                                         self.dtype, kv_pair0))

    def forward(self, x, t, time_ids, text_embeds, cond, B, H, Wd, add_sample=True, cond_embedded=False, kv_pair0=0):
        """x: NHWC [B*H*W, 4] (dtype); t: fp32 [B]; time_ids fp32 [B, 6]; text_embeds fp32 [B, 1280];
        cond: NHWC [B*H*W, 512] image latents (dtype) or None -- or, with cond_embedded=True, their
        condition embedding from cond_embed() [B*H*W, 320].  Returns eps NHWC [B*H*W, 4] (dtype).
        With one prompt pair in the context every CFG pair of the forward uses it; with several (images batched,
        set_context(ctx, ncfg)), CFG pair j uses prompt pair kv_pair0 + j."""
        assert self.ctx is not None, "call set_context(prompt_embeds) first"
        assert B % self.ncfg == 0
        if self.npairs > 1:
            if kv_pair0 + B // self.ncfg > self.npairs:
                raise ValueError(f"forward: pairs {kv_pair0}..{kv_pair0 + B // self.ncfg} past the "
                                 f"{self.npairs} prompt pairs of the context")
            self._kv_mod, self._kv_row0 = 0, kv_pair0 * self.ncfg * self.Lk
        else:
            self._kv_mod, self._kv_row0 = self.ncfg, 0
        with ops.tile_groups(B // self.ncfg):
            return self._forward(x, t, time_ids, text_embeds, cond, B, H, Wd, add_sample, cond_embedded)

    def _forward(self, x, t, time_ids, text_embeds, cond, B, H, Wd, add_sample, cond_embedded=False):
        # (the time / add embeddings on a second stream inside the graph measured 0.39 ms/step slower at C2 and
        # were removed in round 6: FD_SIDE_STREAM, git history)
        self._gn_src = None
        temb = self.embeddings(t, time_ids, text_embeds, B)
        x0 = ops.conv_direct(x, *self.conv_in, B, H, Wd, 4, 3, 1, 1, out_dtype=self.dtype)
        if cond is not None and self.has_extras:
            feat = self._extras(x0, cond, B, H, Wd, embedded=cond_embedded)
            if add_sample:
                x0 = ops.gemm(feat, self.scp[0], bias=self.scp[1], residual=x0)
            else:
                x0 = ops.gemm(feat, self.scp[0], bias=self.scp[1])
        skips = [(x0, 320, H, Wd)]
        h, hh, ww = x0, H, Wd
        for i, blk in enumerate(self.down):
            for j, r in enumerate(blk["resnets"]):
                h = self._resnet(r, h, B, hh, ww, temb)
                if blk["attns"]:
                    h = self._t2d(blk["attns"][j], h, B, hh, ww)
                skips.append((h, r["cout"], hh, ww))
            if blk["ds"] is not None:
                h = ops.conv3x3(h, *blk["ds"], B, hh, ww, stride=2, pad=1)
                hh, ww = (hh + 1) // 2, (ww + 1) // 2
                skips.append((h, r["cout"], hh, ww))
        h = self._resnet(self.mid["r0"], h, B, hh, ww, temb)
        h = self._t2d(self.mid["attn"], h, B, hh, ww)
        h = self._resnet(self.mid["r1"], h, B, hh, ww, temb)
        for i, blk in enumerate(self.up):
            for j, r in enumerate(blk["resnets"]):
                s, cs, _, _ = skips.pop()
                h = self._resnet(r, h, B, hh, ww, temb, x2=s, C1=r["cin"] - cs)
                if blk["attns"]:
                    h = self._t2d(blk["attns"][j], h, B, hh, ww)
            if blk["us"] is not None:
                # Upsample2D to the next skip's size (x2, or diffusers' forward_upsample_size path, ext:665-666)
                th, tw = skips[-1][2], skips[-1][3]
                us = blk["us"]
                if (th, tw) == (2 * hh, 2 * ww) and knobs.get("FD_UP2_PHASE") and ops.up2_phase_ok(h, us[2], B, hh, ww):
                    h = ops.conv3x3_up2(h, us[2], us[1], B, hh, ww)  # the four 2x2 phase convs (pack_conv3x3_up2)
                else:
                    h = ops.conv3x3(h, us[0], us[1], B, hh, ww, upsample=True, upsample_size=(th, tw))
                hh, ww = th, tw
        h = ops.group_norm(h, *self.norm_out, B, hh * ww, 320, 32, 1e-5, silu=True, stats=self._gn_stats_of(h))
        return ops.conv3x3(h, *self.conv_out, B, hh, ww)
