"""t2i conditioning producer — API of libs/clip.py (`FrozenCLIPEmbedder`, 13-38).

The reference wraps transformers' CLIPTextModel (openai/clip-vit-large-patch14) and returns
`last_hidden_state` [B, 77, 768] for a list of prompts, the `context` of libs/uvit_t2i.py:378
(sample_t2i_discrete.py:49-53, train_t2i_discrete.py:343).  Here the text transformer runs on the HIP
encoder of libpdm (csrc/clip.hip, `pdm_clip_*` in include/pdm.h): the block Linears on the bf16 MFMA GEMM
with LayerNorm folded into qkv / fc1 and quick GELU fused into fc1's epilogue, a causal attention kernel,
fp32 residual stream.

Weights: `load_state_dict` takes a CLIPTextModel state_dict (the "transformer.text_model." / "text_model."
prefixes of the reference's module tree and of older transformers checkpoints are stripped), e.g. loaded
from a local copy of the checkpoint with safetensors or `torch.load(..., weights_only=True)`.  Nothing is
downloaded: `FrozenCLIPEmbedder(version=...)` accepts a local directory for the tokenizer and weights, and
`forward(text)` needs a tokenizer (transformers CLIPTokenizer from local files, or any callable returning
`input_ids`).  `encode_tokens(input_ids)` runs the encoder on ids directly.
"""
import ctypes
import os

import torch
import torch.nn as nn

from .. import _lib

# openai/clip-vit-large-patch14 text tower (the reference's default `version`)
VIT_L14_TEXT = dict(vocab_size=49408, hidden_size=768, intermediate_size=3072, num_hidden_layers=12,
                    num_attention_heads=12, max_position_embeddings=77, layer_norm_eps=1e-5)


class _Attn(nn.Module):
    def __init__(self, d):
        super().__init__()
        self.k_proj, self.v_proj, self.q_proj, self.out_proj = (nn.Linear(d, d) for _ in range(4))


class _Mlp(nn.Module):
    def __init__(self, d, f):
        super().__init__()
        self.fc1, self.fc2 = nn.Linear(d, f), nn.Linear(f, d)


class _Layer(nn.Module):
    def __init__(self, d, f):
        super().__init__()
        self.self_attn = _Attn(d)
        self.layer_norm1 = nn.LayerNorm(d)
        self.mlp = _Mlp(d, f)
        self.layer_norm2 = nn.LayerNorm(d)


class _Embeddings(nn.Module):
    def __init__(self, v, d, p):
        super().__init__()
        self.token_embedding = nn.Embedding(v, d)
        self.position_embedding = nn.Embedding(p, d)


class _Encoder(nn.Module):
    def __init__(self, d, f, n):
        super().__init__()
        self.layers = nn.ModuleList(_Layer(d, f) for _ in range(n))


class _ClipHandle:
    """pdm_clip handle + the packed device copies of the weights it points at."""

    def __init__(self, m, device):
        lib = _lib.load()
        cfg = _lib.PdmClipCfg(m.vocab_size, m.hidden_size, m.num_hidden_layers, m.num_attention_heads,
                              m.intermediate_size, m.max_position_embeddings, m.layer_norm_eps)
        h = ctypes.c_void_p()
        _lib.check(lib.pdm_clip_create(ctypes.byref(cfg), ctypes.byref(h)), "pdm_clip_create")
        self.lib, self.h, self.device = lib, h, device
        self.packed = {}
        self.ws = None
        sd = {k: v.detach() for k, v in m.state_dict().items()}
        buf = ctypes.create_string_buffer(256)
        for i in range(lib.pdm_clip_param_count(h)):
            dt, numel = ctypes.c_int(), ctypes.c_longlong()
            _lib.check(lib.pdm_clip_param_info(h, i, buf, 256, ctypes.byref(dt), ctypes.byref(numel)))
            name = buf.value.decode()
            t = self._pack(sd, name, dt.value).to(device).contiguous().reshape(-1)
            if t.numel() != numel.value:
                raise RuntimeError(f"clip weight {name}: packed {t.numel()} elements, expected {numel.value}")
            self.packed[name] = t
            _lib.check(lib.pdm_clip_set_param(h, name.encode(), _lib.ptr(t), dt.value, t.numel()), "pdm_clip_set_param")

    @staticmethod
    def _pack(sd, name, dtype):
        """LayerNorm folding as for the U-ViT blocks (native.NativeHandle._ln_fold): LN(x) W^T + b =
        rstd * (x (W diag(g))^T - mean * colsum) + (W beta + b), colsum over the bf16 folded weight."""
        for lin, norm, parts in ((".self_attn.qkv", ".layer_norm1", ("q_proj", "k_proj", "v_proj")),
                                 (".mlp.fc1", ".layer_norm2", ("mlp.fc1",))):
            for part in (".weight", ".ln_colsum", ".ln_bias"):
                if not name.endswith(lin + part):
                    continue
                pre = name[: -len(lin + part)]
                if len(parts) == 3:
                    w = torch.cat([sd[f"{pre}.self_attn.{n}.weight"] for n in parts]).float()
                    b = torch.cat([sd[f"{pre}.self_attn.{n}.bias"] for n in parts]).double()
                else:
                    w = sd[pre + ".mlp.fc1.weight"].float()
                    b = sd[pre + ".mlp.fc1.bias"].double()
                g = sd[pre + norm + ".weight"].float()
                wg = (w * g[None, :]).to(torch.bfloat16)
                if part == ".weight":
                    return wg
                if part == ".ln_colsum":
                    return wg.double().sum(1).float()
                return (w.double() @ sd[pre + norm + ".bias"].double() + b).float()
        src = sd[name]
        return src.to(torch.bfloat16) if dtype == _lib.PDM_BF16 else src.float()

    def workspace(self, B):
        need = ctypes.c_size_t()
        _lib.check(self.lib.pdm_clip_workspace_size(self.h, B, ctypes.byref(need)), "pdm_clip_workspace_size")
        if self.ws is None or self.ws.numel() < need.value:
            self.ws = torch.empty(need.value, dtype=torch.uint8, device=self.device)
        return self.ws

    def __del__(self):
        try:
            self.lib.pdm_clip_destroy(self.h)
        except Exception:
            pass


class CLIPTextEncoder(nn.Module):
    """Parameter container with CLIPTextModel's state_dict keys (embeddings.*, encoder.layers.i.*,
    final_layer_norm.*); forward(input_ids) -> last_hidden_state on the HIP encoder."""

    def __init__(self, vocab_size=49408, hidden_size=768, intermediate_size=3072, num_hidden_layers=12,
                 num_attention_heads=12, max_position_embeddings=77, layer_norm_eps=1e-5, hidden_act="quick_gelu",
                 **unused):
        super().__init__()
        if hidden_act != "quick_gelu":
            raise ValueError(f"hidden_act {hidden_act!r}: the HIP CLIP encoder implements quick_gelu (CLIP ViT-L/14)")
        self.vocab_size, self.hidden_size, self.intermediate_size = vocab_size, hidden_size, intermediate_size
        self.num_hidden_layers, self.num_attention_heads = num_hidden_layers, num_attention_heads
        self.max_position_embeddings, self.layer_norm_eps = max_position_embeddings, float(layer_norm_eps)
        self.embeddings = _Embeddings(vocab_size, hidden_size, max_position_embeddings)
        self.encoder = _Encoder(hidden_size, intermediate_size, num_hidden_layers)
        self.final_layer_norm = nn.LayerNorm(hidden_size, eps=layer_norm_eps)
        self._native = None
        # encoding with the constructor's default init is refused unless weights were loaded or the caller opted
        # into synthetic weights (benchmarks): a ported sample script must not silently run an untrained encoder
        self.weights_loaded = False
        self.allow_synthetic_weights = False

    def _apply(self, fn, *args, **kwargs):
        self._native = None
        return super()._apply(fn, *args, **kwargs)

    def load_state_dict(self, state_dict, strict=True, *args, **kwargs):
        """Accepts CLIPTextModel keys with or without the `text_model.` / reference `transformer.text_model.`
        prefix; position_ids buffers are dropped.  strict=True (the default) fails on any missing or unexpected
        key."""
        self._native = None
        sd = {}
        for k, v in state_dict.items():
            for pre in ("transformer.text_model.", "text_model.", "transformer."):
                if k.startswith(pre):
                    k = k[len(pre):]
                    break
            if k.endswith("position_ids"):   # buffer of older transformers checkpoints
                continue
            sd[k] = v
        res = super().load_state_dict(sd, strict, *args, **kwargs)
        self.weights_loaded = True
        return res

    @torch.no_grad()
    def forward(self, input_ids):
        if not (self.weights_loaded or self.allow_synthetic_weights):
            raise RuntimeError("CLIP text encoder: no weights loaded (FrozenCLIPEmbedder(version=<local checkpoint "
                               "dir>) or load_state_dict); pass synthetic=True to encode with the default init")
        dev = self.final_layer_norm.weight.device
        _lib.require_gpu(self.final_layer_norm.weight)
        ids = torch.as_tensor(input_ids).to(device=dev, dtype=torch.int64)
        if ids.dim() == 1:
            ids = ids[None]
        B, L = ids.shape
        if L > self.max_position_embeddings:
            raise ValueError(f"sequence length {L} exceeds max_position_embeddings {self.max_position_embeddings}")
        lo, hi = int(ids.min()), int(ids.max())   # nn.Embedding raises on out-of-range ids
        if lo < 0 or hi >= self.vocab_size:
            raise IndexError("index out of range in self")
        if self._native is None or self._native.device != dev:
            self._native = _ClipHandle(self, dev)
        h = self._native
        ws = h.workspace(B)
        out = torch.empty(B, L, self.hidden_size, device=dev, dtype=torch.float32)
        ids = ids.contiguous()
        _lib.check(h.lib.pdm_clip_encode(h.h, _lib.ptr(ids), B, L, _lib.ptr(out), _lib.ptr(ws), ws.numel(),
                                         _lib.stream_ptr(dev)), "pdm_clip_encode")
        return out


class FrozenCLIPEmbedder(nn.Module):
    """libs/clip.py:13-38.  `version` is a LOCAL directory holding the CLIP checkpoint (config.json +
    pytorch_model.bin / model.safetensors) and tokenizer files (loaded strictly: every text-tower key must be
    present), or None for the ViT-L/14 text shape with weights loaded later through
    `transformer.load_state_dict` -- encoding before that raises unless synthetic=True (benchmarks on seeded
    weights).  `tokenizer` overrides the tokenizer (a callable with the transformers CLIPTokenizer call
    signature, or None when only `encode_tokens` is used).  Unlike the reference's no-argument constructor,
    nothing is downloaded: there is no implicit openai/clip-vit-large-patch14."""

    def __init__(self, version=None, device="cuda", max_length=77, tokenizer=None, config=None, synthetic=False):
        super().__init__()
        cfg = dict(VIT_L14_TEXT)
        self.tokenizer = tokenizer
        if version is not None:
            if not os.path.isdir(version):
                raise FileNotFoundError(f"{version!r}: pass a local checkpoint directory (nothing is downloaded)")
            import json
            with open(os.path.join(version, "config.json")) as f:
                c = json.load(f)
            c = c.get("text_config", c)
            cfg.update({k: c[k] for k in cfg if k in c})
            if self.tokenizer is None:
                from transformers import CLIPTokenizer
                self.tokenizer = CLIPTokenizer.from_pretrained(version, local_files_only=True)
        if config is not None:
            cfg.update(config)
        self.transformer = CLIPTextEncoder(**cfg)
        self.transformer.allow_synthetic_weights = bool(synthetic)
        if version is not None:
            self.transformer.load_state_dict(_load_local_weights(version), strict=True)
        self.device = device
        self.max_length = max_length
        self.freeze()

    def freeze(self):
        self.transformer = self.transformer.eval()
        for param in self.parameters():
            param.requires_grad = False

    def encode_tokens(self, tokens):
        """input_ids [B, L] -> last_hidden_state [B, L, width] (libs/clip.py:33-36 after tokenisation)."""
        return self.transformer(tokens)

    def forward(self, text):
        if self.tokenizer is None:
            raise RuntimeError("FrozenCLIPEmbedder: no tokenizer (pass version=<local dir> or tokenizer=...); "
                               "use encode_tokens(input_ids) for pre-tokenised prompts")
        batch_encoding = self.tokenizer(text, truncation=True, max_length=self.max_length, return_length=True,
                                        return_overflowing_tokens=False, padding="max_length", return_tensors="pt")
        return self.encode_tokens(batch_encoding["input_ids"].to(self.device))

    def encode(self, text):
        return self(text)


def _load_local_weights(path):
    for fn in ("model.safetensors", "pytorch_model.bin"):
        p = os.path.join(path, fn)
        if os.path.exists(p):
            if fn.endswith(".safetensors"):
                from safetensors.torch import load_file
                sd = load_file(p)
            else:
                sd = torch.load(p, map_location="cpu", weights_only=True)
            return {k: v for k, v in sd.items() if k.startswith(("text_model.", "embeddings.", "encoder.",
                                                                  "final_layer_norm."))}
    raise FileNotFoundError(f"no model.safetensors / pytorch_model.bin under {path!r}")
