"""KL-f8 latent decoder — API of libs/autoencoder.py (`get_model(...).decode(z)`, 446-450, 471-484).

Decode-only: the sampling path never encodes.  `FrozenAutoencoderKL` keeps the
reference's state_dict keys for `post_quant_conv.*` and `decoder.*` (the encoder keys of a reference
checkpoint are accepted and ignored), so `get_model(path)` loads the reference's
assets/stable-diffusion/autoencoder_kl*.pth with `torch.load(..., weights_only=True)`.

INTERIM (round 1): the decoder's convolutions / GroupNorm run as PyTorch-ROCm (MIOpen) ops in bf16 on the
GPU.  The hand-written implicit-GEMM HIP decoder is the next row of SURVEY.md §8(f).
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import _lib
from .. import weights as W

DDCONFIG = dict(W.DECODER_DDCONFIG)


def _gn_swish(x, w, b):
    return F.silu(F.group_norm(x, 32, w, b, eps=1e-6))


class FrozenAutoencoderKL(nn.Module):
    def __init__(self, ddconfig=None, embed_dim=4, pretrained_path=None, scale_factor=0.18215, seed=0,
                 dtype=torch.bfloat16, state_dict=None):
        super().__init__()
        dd = dict(DDCONFIG if ddconfig is None else ddconfig)
        self.ch_mult = tuple(dd["ch_mult"])
        self.num_res_blocks = dd["num_res_blocks"]
        self.scale_factor = scale_factor
        self.embed_dim = embed_dim
        self.compute_dtype = dtype
        spec = W.decoder_spec(ch=dd["ch"], out_ch=dd["out_ch"], ch_mult=self.ch_mult,
                              num_res_blocks=self.num_res_blocks, z_channels=dd["z_channels"], embed_dim=embed_dim)
        if state_dict is not None or pretrained_path is not None:
            full = state_dict if state_dict is not None else torch.load(pretrained_path, map_location="cpu",
                                                                        weights_only=True)
            sd = {k: v for k, v in full.items() if k.startswith("decoder.") or k.startswith("post_quant_conv.")}
            missing = [k for k, _, _ in spec if k not in sd]
            if missing:
                raise RuntimeError(f"autoencoder checkpoint is missing {len(missing)} decoder keys, e.g. {missing[:3]}")
        else:
            sd = W.make_state_dict(spec, seed=seed, init="reference")
        self._names = [k for k, _, _ in spec]
        for k in self._names:
            self.register_buffer(k.replace(".", "__"), sd[k].float().clone())
        self.requires_grad_(False)
        self.eval()

    def _p(self, name):
        return getattr(self, name.replace(".", "__"))

    def _conv(self, name, x, pad):
        return F.conv2d(x, self._p(f"{name}.weight").to(x.dtype), self._p(f"{name}.bias").to(x.dtype), padding=pad)

    def _res(self, p, x):
        h = self._conv(f"{p}.conv1", _gn_swish(x, self._p(f"{p}.norm1.weight").to(x.dtype), self._p(f"{p}.norm1.bias").to(x.dtype)), 1)
        h = self._conv(f"{p}.conv2", _gn_swish(h, self._p(f"{p}.norm2.weight").to(x.dtype), self._p(f"{p}.norm2.bias").to(x.dtype)), 1)
        if hasattr(self, f"{p}.nin_shortcut.weight".replace(".", "__")):
            x = self._conv(f"{p}.nin_shortcut", x, 0)
        return x + h

    def _attn(self, p, x):
        h = F.group_norm(x, 32, self._p(f"{p}.norm.weight").to(x.dtype), self._p(f"{p}.norm.bias").to(x.dtype), eps=1e-6)
        q = self._conv(f"{p}.q", h, 0)
        k = self._conv(f"{p}.k", h, 0)
        v = self._conv(f"{p}.v", h, 0)
        b, c, hh, ww = q.shape
        q = q.reshape(b, c, hh * ww).transpose(1, 2)[:, None]
        k = k.reshape(b, c, hh * ww).transpose(1, 2)[:, None]
        v = v.reshape(b, c, hh * ww).transpose(1, 2)[:, None]
        o = F.scaled_dot_product_attention(q, k, v)[:, 0].transpose(1, 2).reshape(b, c, hh, ww)
        return x + self._conv(f"{p}.proj_out", o, 0)

    @torch.no_grad()
    def decode(self, z):
        """libs/autoencoder.py:446-450 + Decoder.forward 376-409."""
        _lib.require_gpu(z)
        x = (z.float() / self.scale_factor).to(self.compute_dtype).contiguous(memory_format=torch.channels_last)
        x = self._conv("post_quant_conv", x, 0)
        h = self._conv("decoder.conv_in", x, 1)
        h = self._res("decoder.mid.block_1", h)
        h = self._attn("decoder.mid.attn_1", h)
        h = self._res("decoder.mid.block_2", h)
        for i_level in reversed(range(len(self.ch_mult))):
            for i_block in range(self.num_res_blocks + 1):
                h = self._res(f"decoder.up.{i_level}.block.{i_block}", h)
            if i_level != 0:
                h = F.interpolate(h, scale_factor=2.0, mode="nearest")
                h = self._conv(f"decoder.up.{i_level}.upsample.conv", h, 1)
        h = _gn_swish(h, self._p("decoder.norm_out.weight").to(h.dtype), self._p("decoder.norm_out.bias").to(h.dtype))
        return self._conv("decoder.conv_out", h, 1).float()

    def forward(self, inputs, fn):
        if fn == "decode":
            return self.decode(inputs)
        raise NotImplementedError(f"{fn}: only decode is on the sampling path")


def get_model(pretrained_path=None, scale_factor=0.18215, **kw):
    """libs/autoencoder.py:471-484 (pretrained_path=None -> synthetic seeded weights)."""
    return FrozenAutoencoderKL(DDCONFIG, 4, pretrained_path, scale_factor, **kw)
