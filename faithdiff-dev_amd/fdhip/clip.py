"""SDXL's two CLIP text encoders on the HIP kernel library.

encode_prompt (pipeline_FaithDiff_tlc.py:485-717) runs CLIP ViT-L/14 (CLIPTextModel) and OpenCLIP ViT-bigG/14
(CLIPTextModelWithProjection) on 77 token ids and keeps hidden_states[-2] of each (concat -> 2048 channels)
plus the projected pooled output of the second (:608-613).  The algorithm is transformers' CLIPTextTransformer
(transformers==4.46.1, reference requirements.txt:3): token + position embedding; per layer a pre-LN causal
self-attention (q/k/v/out with bias, head dim 64, scale 1/8) and a pre-LN MLP fc1 -> act (quick_gelu for L,
gelu for bigG) -> fc2, both residual; final LayerNorm; pooled = final-LN row at argmax(input_ids) (the
legacy eos_token_id == 2 path of both SDXL configs; EOS 49407 is the largest id, so this is the first EOS);
text_projection without bias.  Each Linear is one fd_gemm (bias / activation / residual in the epilogue), the
attention one causal fd_flash_attn, the embeddings one fd_embed_tokens; activations bf16 (the reference: fp16).

The forward (~220 launches for bigG) is replayed as one hipGraph per (batch, length, row groups)
(fdhip/graphs.py, GraphCache(min_uses=1): the first call of a shape runs eagerly once to size the workspaces, then
captures and replays in that same call): eager ctypes launches made encode_prompt ~8 ms of a 1024^2 pipe() call.
The EOS row is picked on the device (argmax of the ids), so nothing in the forward needs the host.

Batching: encode_prompt sends the prompt and the negative prompt through each encoder as ONE batch of ``groups``
row groups (the reference makes one pass per prompt).  The forward runs under ops.tile_groups(groups), so every
fd_gemm sees the per-group row count (m_ref) and picks the kernel, tile family and split-K a solo pass of one
group would pick: each group's rows are bitwise what encoding it alone gives (GPU test).
"""
import torch

from . import arch
from . import lib as L
from . import ops
from .graphs import GraphCache


class HipCLIPTextModel:
    def __init__(self, sd, cfg, device="cuda", dtype=torch.bfloat16):
        L.require_device()
        self.cfg, self.device, self.dtype = dict(cfg), torch.device(device), dtype
        W = lambda k: sd[k].to(device=self.device, dtype=dtype).contiguous()  # noqa: E731
        Fp = lambda k: sd[k].to(device=self.device, dtype=torch.float32).contiguous()  # noqa: E731
        self.tok = W("text_model.embeddings.token_embedding.weight")
        self.pos = W("text_model.embeddings.position_embedding.weight")
        self.layers = []
        for i in range(cfg["layers"]):
            q = f"text_model.encoder.layers.{i}"
            p = f"{q}.self_attn"
            self.layers.append(dict(
                ln1=(Fp(f"{q}.layer_norm1.weight"), Fp(f"{q}.layer_norm1.bias")),
                qkv=torch.cat([sd[f"{p}.{n}_proj.weight"] for n in "qkv"], 0).to(self.device, dtype).contiguous(),
                qkv_b=torch.cat([sd[f"{p}.{n}_proj.bias"] for n in "qkv"], 0).to(self.device,
                                                                                 torch.float32).contiguous(),
                out=(W(f"{p}.out_proj.weight"), Fp(f"{p}.out_proj.bias")),
                ln2=(Fp(f"{q}.layer_norm2.weight"), Fp(f"{q}.layer_norm2.bias")),
                fc1=(W(f"{q}.mlp.fc1.weight"), Fp(f"{q}.mlp.fc1.bias")),
                fc2=(W(f"{q}.mlp.fc2.weight"), Fp(f"{q}.mlp.fc2.bias"))))
        self.fln = (Fp("text_model.final_layer_norm.weight"), Fp("text_model.final_layer_norm.bias"))
        self.proj = W("text_projection.weight") if cfg.get("proj") else None
        self.graphs = GraphCache(max_graphs=4, min_uses=1)  # one call per encoder per image: capture at once

    @torch.no_grad()
    def forward(self, input_ids, groups=1):
        """input_ids [B, T] (any int dtype, host or device); groups: the B rows are that many independent batches
        of B / groups rows each (bitwise what each group gives alone).  Returns a dict: hidden_states (list of
        [B, T, D] in the compute dtype: the embeddings, then each layer's output, as transformers'
        output_hidden_states), last_hidden_state, pooled ([B, D], final-LN EOS row), text_embeds ([B, proj] with a
        projection).  The tensors are the graph's static outputs: valid until the next call of the same shape
        (CLIPTextModel.__call__ uses forward_f32, which copies them out straight away)."""
        ids = torch.as_tensor(input_ids)
        B, T = ids.shape
        groups = self._check_groups(B, groups)
        ids_d = ids.to(device=self.device, dtype=torch.int32).contiguous().reshape(-1)
        outs = self.graphs.run(("clip", B, T, groups), lambda i: self._forward_dev(i, B, T, groups), [ids_d])
        nl = self.cfg["layers"]
        out = dict(hidden_states=list(outs[:nl + 1]), last_hidden_state=outs[nl + 1], pooled=outs[nl + 2])
        if self.proj is not None:
            out["text_embeds"] = outs[nl + 3]
        return out

    @torch.no_grad()
    def forward_f32(self, input_ids, groups=1):
        """forward() with every output as fp32 (what the transformers surface returns), all of them packed into one
        buffer inside the graph and copied out of its static memory by a single clone -- instead of ~50 separate
        conversions per call.  The returned tensors are views of that private copy."""
        ids = torch.as_tensor(input_ids)
        B, T = ids.shape
        groups = self._check_groups(B, groups)
        ids_d = ids.to(device=self.device, dtype=torch.int32).contiguous().reshape(-1)
        shapes = []

        def packed(i):
            outs = self._forward_dev(i, B, T, groups)
            flat = torch.empty(sum(o.numel() for o in outs), dtype=torch.float32, device=self.device)
            off = 0
            for o in outs:
                flat[off:off + o.numel()].view(o.shape).copy_(o)
                off += o.numel()
            return flat
        for o in self._out_shapes(B, T):
            shapes.append(o)
        flat = self.graphs.run(("clip32", B, T, groups), packed, [ids_d]).clone()
        views, off = [], 0
        for shp in shapes:
            n = 1
            for d in shp:
                n *= d
            views.append(flat[off:off + n].view(shp))
            off += n
        nl = self.cfg["layers"]
        out = dict(hidden_states=views[:nl + 1], last_hidden_state=views[nl + 1], pooled=views[nl + 2])
        if self.proj is not None:
            out["text_embeds"] = views[nl + 3]
        return out

    @staticmethod
    def _check_groups(B, groups):
        groups = max(int(groups), 1)
        if B % groups:
            raise ValueError(f"{B} rows do not split into {groups} equal groups")
        return groups

    def _out_shapes(self, B, T):
        D = self.cfg["D"]
        shp = [(B, T, D)] * (self.cfg["layers"] + 1) + [(B, T, D), (B, D)]
        if self.proj is not None:
            shp.append((B, self.proj.shape[0]))
        return shp

    def _forward_dev(self, ids_d, B, T, groups=1):
        """Device-only body of forward (capturable): a tuple (hidden states..., last, pooled[, text_embeds]).  Every
        launch sees the per-group row count (ops.tile_groups), so a batch of `groups` groups is bitwise each group's
        solo forward."""
        with ops.tile_groups(groups):
            return self._forward_body(ids_d, B, T)

    def _forward_body(self, ids_d, B, T):
        D = self.cfg["D"]
        H = D // 64
        M = B * T
        h = torch.empty((M, D), dtype=self.dtype, device=self.device)
        ops.embed_tokens(ids_d, self.tok, self.pos, h, B, T)
        hidden = [h.reshape(B, T, D)]
        n = torch.empty_like(h)
        qkv = torch.empty((M, 3 * D), dtype=self.dtype, device=self.device)
        att = torch.empty_like(h)
        act = "quickgelu" if self.cfg["act"] == "quickgelu" else "gelu"
        for lay in self.layers:
            h = h.clone()  # every layer's output is kept (hidden_states)
            ops.layer_norm(h, *lay["ln1"], 1e-5, out=n)
            ops.gemm(n, lay["qkv"], bias=lay["qkv_b"], out=qkv)
            ops.flash_attn(qkv, qkv[:, D:], qkv[:, 2 * D:], att, B, H, T, T, 3 * D, 3 * D, 3 * D, D,
                           T * 3 * D, T * 3 * D, T * 3 * D, T * D, kv_mod=0, scale=0.125, causal=True)
            ops.gemm(att, lay["out"][0], bias=lay["out"][1], residual=h, out=h)
            ops.layer_norm(h, *lay["ln2"], 1e-5, out=n)
            m = ops.gemm(n, lay["fc1"][0], bias=lay["fc1"][1], act=act)
            ops.gemm(m, lay["fc2"][0], bias=lay["fc2"][1], residual=h, out=h)
            hidden.append(h.reshape(B, T, D))
        last = torch.empty_like(h)
        ops.layer_norm(h, *self.fln, 1e-5, out=last)
        # pooled = the final-LN row at argmax(input_ids) (first EOS), selected on the device
        eos = ids_d.view(B, T).argmax(dim=-1).to(torch.int64)
        rows = torch.arange(B, device=self.device, dtype=torch.int64) * T + eos
        pooled = last.index_select(0, rows).contiguous()
        outs = hidden + [last.reshape(B, T, D), pooled]
        if self.proj is not None:
            outs.append(ops.gemm(pooled, self.proj))
        return tuple(outs)


def random_clip(cfg, seed, device="cpu"):
    """Seeded random-init state dict of the real architecture (no weights offline)."""
    return arch.random_init(arch.clip_param_shapes(cfg), seed=seed, device=device)
