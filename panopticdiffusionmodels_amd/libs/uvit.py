"""U-ViT (class-conditional / unconditional), reference API of libs/uvit.py:138-230, HIP forward.

`UViT(**config.nnet)` keeps the reference constructor signature and state_dict keys; `forward(x,
timesteps, y=None)` returns the same tensor the reference returns (libs/uvit.py:201-230) but runs as
libpdm kernels on the GPU: token assembly -> [LN -> qkv GEMM -> fused attention -> proj GEMM(+res) -> LN
-> fc1 GEMM(+GELU) -> fc2 GEMM(+res)] x depth+1 with split-K long skips -> LN -> decoder_pred +
unpatchify -> final 3x3 conv.  There is no CPU path.
"""
import math

import torch
import torch.nn as nn

from .. import _lib
from ..native import HipNet


def timestep_embedding(timesteps, dim, max_period=10000):
    """libs/uvit.py:20-38 (host helper with the reference semantics; the HIP path computes it on device)."""
    half = dim // 2
    freqs = torch.exp(-math.log(max_period) * torch.arange(start=0, end=half, dtype=torch.float32) / half).to(
        device=timesteps.device)
    args = timesteps[:, None].float() * freqs[None]
    emb = torch.cat([torch.cos(args), torch.sin(args)], dim=-1)
    if dim % 2:
        emb = torch.cat([emb, torch.zeros_like(emb[:, :1])], dim=-1)
    return emb


class _Attention(nn.Module):
    def __init__(self, dim, num_heads, qkv_bias):
        super().__init__()
        self.num_heads = num_heads
        self.qkv = nn.Linear(dim, dim * 3, bias=qkv_bias)
        self.proj = nn.Linear(dim, dim)


class _Mlp(nn.Module):
    def __init__(self, dim, hidden):
        super().__init__()
        self.fc1 = nn.Linear(dim, hidden)
        self.fc2 = nn.Linear(hidden, dim)


class Block(nn.Module):
    """Parameter container with the key layout of libs/uvit.py:95-113."""

    def __init__(self, dim, num_heads, mlp_ratio=4., qkv_bias=False, skip=False):
        super().__init__()
        self.norm1 = nn.LayerNorm(dim)
        self.attn = _Attention(dim, num_heads, qkv_bias)
        self.norm2 = nn.LayerNorm(dim)
        self.mlp = _Mlp(dim, int(dim * mlp_ratio))
        self.skip_linear = nn.Linear(2 * dim, dim) if skip else None


class PatchEmbed(nn.Module):
    def __init__(self, patch_size, in_chans=3, embed_dim=768):
        super().__init__()
        self.patch_size = patch_size
        self.proj = nn.Conv2d(in_chans, embed_dim, kernel_size=patch_size, stride=patch_size)


def _init_weights(m):
    """libs/uvit.py:185-195."""
    if isinstance(m, nn.Linear):
        nn.init.trunc_normal_(m.weight, std=.02)
        if m.bias is not None:
            nn.init.constant_(m.bias, 0)
    elif isinstance(m, nn.LayerNorm):
        nn.init.constant_(m.bias, 0)
        nn.init.constant_(m.weight, 1.0)


class UViT(HipNet):
    def __init__(self, img_size=224, patch_size=16, in_chans=3, embed_dim=768, depth=12, num_heads=12, mlp_ratio=4.,
                 qkv_bias=False, qk_scale=None, norm_layer=nn.LayerNorm, mlp_time_embed=False, num_classes=-1,
                 use_checkpoint=False, conv=True, skip=True):
        super().__init__()
        self.precision = "bf16"
        if qk_scale is not None:
            raise ValueError("qk_scale other than the default head_dim ** -0.5 is not supported")
        self.num_features = self.embed_dim = embed_dim
        self.num_classes = num_classes
        self.in_chans = in_chans
        self.img_size, self.patch_size, self.depth, self.num_heads = img_size, patch_size, depth, num_heads
        self.mlp_ratio, self.qkv_bias, self.mlp_time_embed, self.conv, self.skip = mlp_ratio, qkv_bias, mlp_time_embed, conv, skip
        self.patch_embed = PatchEmbed(patch_size=patch_size, in_chans=in_chans, embed_dim=embed_dim)
        num_patches = (img_size // patch_size) ** 2
        self.time_embed = nn.Sequential(nn.Linear(embed_dim, 4 * embed_dim), nn.SiLU(),
                                        nn.Linear(4 * embed_dim, embed_dim)) if mlp_time_embed else nn.Identity()
        if self.num_classes > 0:
            self.label_emb = nn.Embedding(self.num_classes, embed_dim)
            self.extras = 2
        else:
            self.extras = 1
        self.pos_embed = nn.Parameter(torch.zeros(1, self.extras + num_patches, embed_dim))
        self.in_blocks = nn.ModuleList([Block(embed_dim, num_heads, mlp_ratio, qkv_bias) for _ in range(depth // 2)])
        self.mid_block = Block(embed_dim, num_heads, mlp_ratio, qkv_bias)
        self.out_blocks = nn.ModuleList([Block(embed_dim, num_heads, mlp_ratio, qkv_bias, skip=skip)
                                         for _ in range(depth // 2)])
        self.norm = nn.LayerNorm(embed_dim)
        self.patch_dim = patch_size ** 2 * in_chans
        self.decoder_pred = nn.Linear(embed_dim, self.patch_dim, bias=True)
        self.final_layer = nn.Conv2d(self.in_chans, self.in_chans, 3, padding=1) if conv else nn.Identity()
        nn.init.trunc_normal_(self.pos_embed, std=.02)
        self.apply(_init_weights)

    def _native_cfg_kwargs(self):
        return dict(img_size=self.img_size, patch_size=self.patch_size, in_chans=self.in_chans,
                    embed_dim=self.embed_dim, depth=self.depth, num_heads=self.num_heads, mlp_ratio=self.mlp_ratio,
                    num_classes=self.num_classes, conv=self.conv, skip=self.skip, qkv_bias=self.qkv_bias,
                    mlp_time_embed=self.mlp_time_embed, fp8=self.precision != "bf16",
                    fp8_linears=self.FP8_LINEARS[self.precision], residual=self.residual)

    # include/pdm.h pdm_uvit_cfg.fp8_linears: bit 0 attn.qkv, 1 attn.proj, 2 mlp.fc1, 3 mlp.fc2
    FP8_LINEARS = {"bf16": 0, "fp8": 0xB, "fp8-all": 0xF}

    def set_precision(self, precision):
        """Precision of the block Linears (BASELINE configs[4], imagenet512_uvit_huge; include/pdm.h
        pdm_uvit_cfg.fp8 / fp8_linears).  Not a reference option: the reference computes in the autocast dtype.
          'bf16'    (default) every GEMM bf16
          'fp8'     attn.qkv, attn.proj, mlp.fc2 as MXFP8 GEMMs on the block-scaled MFMA, mlp.fc1 and
                    skip_linear bf16: H/4 forward 5.0e-2 rel-L2 vs fp32 (within SURVEY.md §8c's 6e-2)
          'fp8-all' mlp.fc1 MXFP8 too (6.9e-2; tools/fp8_ablation.py prints the per-Linear ablation)
        Everything else (attention, norms, heads) is unchanged.  Re-packs the weights (invalidates the handle; a
        sampler's captured graph is recaptured on the next sample)."""
        if precision not in self.FP8_LINEARS:
            raise ValueError(f"precision must be one of {sorted(self.FP8_LINEARS)}, got {precision!r}")
        self.precision = precision
        self.invalidate()
        return self

    @torch.jit.ignore
    def no_weight_decay(self):
        return {'pos_embed'}

    # ---- HIP path ------------------------------------------------------------------------------
    def forward_pre(self, x, timesteps, y=None, out=None, workspace=None):
        """Everything up to the final conv: returns the unpatchified decoder_pred output [B, C, H, W] fp32.
        workspace: a caller-owned uint8 device tensor of >= workspace_bytes(B) (default: the handle's own), so
        independent batches can run concurrently on different streams."""
        _lib.require_gpu(x)
        nat = self.native()
        x = x.float().contiguous()
        B = x.shape[0]
        t = timesteps.to(device=x.device, dtype=torch.float32).reshape(-1)
        if t.numel() == 1 and B > 1:
            t = t.expand(B)
        t = t.contiguous()
        if t.numel() != B:
            raise ValueError(f"timesteps has {t.numel()} entries for a batch of {B}")
        if (self.num_classes > 0) != (y is not None):
            raise ValueError("labels y must be given iff num_classes > 0")
        if y is not None:
            y = y.to(device=x.device, dtype=torch.int64).reshape(-1).contiguous()
        if out is None:
            out = torch.empty(B, self.in_chans, self.img_size, self.img_size, dtype=torch.float32, device=x.device)
        ws = nat.workspace(B, x.device) if workspace is None else workspace
        _lib.check(nat.lib.pdm_uvit_forward(nat.h, _lib.ptr(x), _lib.ptr(t), _lib.ptr(y), _lib.ptr(out), B,
                                            _lib.ptr(ws), ws.numel(), _lib.stream_ptr(x.device)), "pdm_uvit_forward")
        return out

    def final_conv_params(self):
        nat = self.native()
        if not self.conv:
            return None, None
        w = nat.packed.get("final_layer.weight")
        if w is None:
            nat.packed["final_layer.weight"] = self.final_layer.weight.detach().float().contiguous()
            nat.packed["final_layer.bias"] = self.final_layer.bias.detach().float().contiguous()
        return nat.packed["final_layer.weight"], nat.packed["final_layer.bias"]

    def forward(self, x, timesteps, y=None):
        pre = self.forward_pre(x, timesteps, y)
        if not self.conv:
            return pre
        w, b = self.final_conv_params()
        out = torch.empty_like(pre)
        _lib.stage_epilogue(pre, pre.shape[0], conv_w=w, conv_b=b, m_out=out)
        return out
