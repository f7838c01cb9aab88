"""Drop-in text encoders and tokenizers for SDXL's encode_prompt (pipeline_FaithDiff_tlc.py:485-717).

The reference loads ``tokenizer``/``tokenizer_2`` (transformers CLIPTokenizer) and ``text_encoder``
(CLIPTextModel, ViT-L/14) / ``text_encoder_2`` (CLIPTextModelWithProjection, OpenCLIP ViT-bigG/14) from the SDXL
directory through diffusers.  Here the encoders run on the HIP library (fdhip.clip) behind the same call
surface the pipeline uses: ``encoder(input_ids, output_hidden_states=True)`` -> an output whose ``[0]`` is
``last_hidden_state`` (CLIPTextModel) or ``text_embeds`` (WithProjection) and whose ``.hidden_states`` holds
the embeddings and every layer's output.  Weights: a local diffusers ``text_encoder*/`` directory
(safetensors or a weights-only torch file, no pickle execution) or, for the 'random-init' sentinel, seeded
random weights of the real architecture.

Tokenizers: transformers' CLIPTokenizer when the directory holds ``vocab.json`` + ``merges.txt``; otherwise
(nothing can be downloaded here) a deterministic stand-in with CLIP's framing -- BOS 49406, up to 75 word ids,
EOS 49407, padding to 77 with the tokenizer's pad id (49407 for tokenizer, 0 = "!" for tokenizer_2) -- whose
word ids are crc32-hashed, i.e. NOT CLIP's BPE vocabulary (real text needs the real files).
"""
import os
import re
import zlib
from types import SimpleNamespace

import torch

from fdhip import arch

BOS, EOS = 49406, 49407


class FallbackCLIPTokenizer:
    model_max_length = 77

    def __init__(self, pad_token_id=EOS):
        self.pad_token_id = pad_token_id
        self.bos_token_id, self.eos_token_id = BOS, EOS

    def _ids(self, text):
        words = re.findall(r"[a-z0-9]+|[^\sa-z0-9]", text.lower())
        return [256 + zlib.crc32(w.encode("utf-8")) % (BOS - 256) for w in words]

    def __call__(self, prompt, padding="max_length", max_length=None, truncation=True, return_tensors="pt"):
        prompts = [prompt] if isinstance(prompt, str) else list(prompt)
        L = max_length or self.model_max_length
        rows = []
        for p in prompts:
            body = self._ids(p)
            if truncation:
                body = body[:L - 2]
            rows.append([BOS] + body + [EOS])
        if padding == "longest":
            L = max(len(r) for r in rows)
        ids = [r + [self.pad_token_id] * (L - len(r)) for r in rows]
        return SimpleNamespace(input_ids=torch.tensor(ids, dtype=torch.long))

    def batch_decode(self, ids):
        return ["<hashed tokens>"] * len(ids)


def load_tokenizer(path, subfolder, pad_token_id):
    d = os.path.join(str(path), subfolder)
    if os.path.isfile(os.path.join(d, "vocab.json")) and os.path.isfile(os.path.join(d, "merges.txt")):
        from transformers import CLIPTokenizer
        return CLIPTokenizer.from_pretrained(d, local_files_only=True)
    return FallbackCLIPTokenizer(pad_token_id)


def _load_weights(path, subfolder, cfg, seed):
    from .unet_2d_condition_vae_extension import RANDOM_INIT, RECEIVE, _check_keys, _empty, _load_file
    shapes = arch.clip_param_shapes(cfg)
    if path == RANDOM_INIT:
        return arch.random_init(shapes, seed=seed)
    if path == RECEIVE:
        return _empty(shapes)
    d = os.path.join(str(path), subfolder)
    for n in ("model.fp16.safetensors", "model.safetensors", "pytorch_model.fp16.bin", "pytorch_model.bin"):
        if os.path.exists(os.path.join(d, n)):
            sd = _load_file(os.path.join(d, n))
            sd = {k: v for k, v in sd.items() if k != "text_model.embeddings.position_ids"}
            _check_keys(sd, shapes, True, subfolder)
            return sd
    raise FileNotFoundError(f"no text-encoder weights under {d}")


class _Output(list):
    """Tuple-like model output: index 0 is the first field; named fields are attributes."""


class CLIPTextModel:
    """HIP-backed transformers.CLIPTextModel surface (ViT-L/14 config)."""
    cfg = arch.CLIP_L

    def __init__(self, sd, cfg=None):
        if cfg is not None:
            self.cfg = dict(cfg)
        self._sd = sd
        self._hip = None
        self._device = torch.device("cpu")
        self._dtype = torch.float16  # the reference's torch_dtype; compute here is bf16

    @classmethod
    def from_pretrained(cls, path, subfolder="text_encoder", seed=0, **kwargs):
        return cls(_load_weights(path, subfolder, cls.cfg, seed))

    @property
    def dtype(self):
        return self._dtype

    @property
    def device(self):
        return self._device

    def to(self, device=None, dtype=None, **kwargs):
        if isinstance(device, torch.dtype):
            device, dtype = None, device
        if dtype is not None:
            self._dtype = dtype
        if device is not None:
            self._device = torch.device(device)
            if self._device.type == "cuda" and self._device.index is None:
                self._device = torch.device("cuda", torch.cuda.current_device())
        return self

    def hip(self):
        if self._hip is None:
            if self._device.type != "cuda":
                raise RuntimeError("the text encoders run only on an MI355X (gfx950); call .to('cuda') first")
            from fdhip.clip import HipCLIPTextModel
            self._hip = HipCLIPTextModel(self._sd, self.cfg, self._device, torch.bfloat16)
        return self._hip

    def _first(self, out):
        return out["last_hidden_state"]

    @torch.no_grad()
    def __call__(self, input_ids, output_hidden_states=False, row_groups=1, **kwargs):
        """transformers' call surface.  row_groups (this build's addition, used by encode_prompt): the rows are
        that many independent prompt batches, each computed bitwise as if encoded alone."""
        out = self.hip().forward_f32(input_ids, groups=row_groups)  # fp32, one private copy per call
        o = _Output([self._first(out)])
        o.hidden_states = tuple(out["hidden_states"]) if output_hidden_states else None
        o.last_hidden_state = out["last_hidden_state"]
        o.pooler_output = out["pooled"]
        o.text_embeds = out.get("text_embeds")
        return o


class CLIPTextModelWithProjection(CLIPTextModel):
    """HIP-backed transformers.CLIPTextModelWithProjection surface (OpenCLIP ViT-bigG/14 config)."""
    cfg = arch.CLIP_G

    @classmethod
    def from_pretrained(cls, path, subfolder="text_encoder_2", seed=0, **kwargs):
        return cls(_load_weights(path, subfolder, cls.cfg, seed))

    def _first(self, out):
        return out["text_embeds"]
