"""Text-conditioned U-ViT with panoptic-mask co-generation — API of libs/uvit_t2i.py:258-525, HIP forward.

Keeps the reference constructor and state_dict keys.  With `separate=True` and a mask token the forward
runs the two block stacks of the reference (image stream over [time, context, patches]; mask stream over
mx = cat(x, m) with zero-initialised 1x1 `zeroconv` injections back into the image stream) as one native
call (pdm_uvit_t2i_forward); the heads, final convs, tanh and CFG are applied by pdm_stage_epilogue.
"""
import torch
import torch.nn as nn

from .. import _lib
from ..native import HipNet
from .uvit import Block, PatchEmbed, _init_weights


class zeroconv(nn.Module):
    """libs/uvit_t2i.py:246-257 (Conv1d(D, D, 1) over tokens)."""

    def __init__(self, embed_dim):
        super().__init__()
        self.conv = nn.Conv1d(embed_dim, embed_dim, 1, padding=0)


class UViT(HipNet):
    _t2i = True

    def __init__(self, img_size=224, patch_size=16, in_chans=3, embed_dim=768, depth=12, num_heads=12, mlp_ratio=4.,
                 qkv_bias=False, qk_scale=None, norm_layer=nn.LayerNorm, mlp_time_embed=False, use_checkpoint=False,
                 clip_dim=768, num_clip_token=77, conv=True, skip=True, num_panoptic_class=8, enable_panoptic=True,
                 use_ground_truth=False, separate=False):
        super().__init__()
        if qk_scale is not None:
            raise ValueError("qk_scale other than the default head_dim ** -0.5 is not supported")
        self.num_features = self.embed_dim = embed_dim
        self.in_chans = in_chans
        self.enable_panoptic = enable_panoptic
        self.separate = separate
        self.depth = depth
        self.img_size, self.patch_size, self.num_heads, self.mlp_ratio = img_size, patch_size, num_heads, mlp_ratio
        self.qkv_bias, self.mlp_time_embed, self.conv, self.skip = qkv_bias, mlp_time_embed, conv, skip
        self.clip_dim, self.num_clip_token = clip_dim, num_clip_token
        self.patch_embed = PatchEmbed(patch_size=patch_size, in_chans=in_chans, embed_dim=embed_dim)
        num_patches = (img_size // patch_size) ** 2
        self.time_embed = nn.Sequential(nn.Linear(embed_dim, 4 * embed_dim), nn.SiLU(),
                                        nn.Linear(4 * embed_dim, embed_dim)) if mlp_time_embed else nn.Identity()
        self.context_embed = nn.Linear(clip_dim, embed_dim)
        self.extras = 1 + num_clip_token
        if enable_panoptic and not separate:
            self.pos_embed = nn.Parameter(torch.zeros(1, self.extras + 2 * num_patches, embed_dim))
        else:
            self.pos_embed = nn.Parameter(torch.zeros(1, self.extras + num_patches, embed_dim))
        if enable_panoptic and separate:
            self.pos_embed_mask = nn.Parameter(torch.zeros(1, num_patches, embed_dim))
            nn.init.trunc_normal_(self.pos_embed_mask, std=.02)
        mk = lambda skip_=False: Block(embed_dim, num_heads, mlp_ratio, qkv_bias, skip=skip_)  # noqa: E731
        self.in_blocks = nn.ModuleList([mk() for _ in range(depth // 2)])
        self.mid_block = mk()
        self.out_blocks = nn.ModuleList([mk(skip) for _ in range(depth // 2)])
        if separate:
            self.in_blocks_mask = nn.ModuleList([mk() for _ in range(depth // 2)])
            self.mid_block_mask = mk()
            self.out_blocks_mask = nn.ModuleList([mk(skip) for _ in range(depth // 2)])
            self.zero_convs = nn.ModuleList([zeroconv(embed_dim) for _ in range(depth * 2 + 2)])
        self.norm = nn.LayerNorm(embed_dim)
        self.patch_dim = patch_size ** 2 * in_chans
        self.decoder_pred = nn.Linear(embed_dim, self.patch_dim, bias=True)
        self.final_layer = nn.Conv2d(self.in_chans, self.in_chans, 3, padding=1) if conv else nn.Identity()
        if enable_panoptic:
            self.mask_embed = PatchEmbed(patch_size=patch_size, in_chans=num_panoptic_class, embed_dim=embed_dim)
            self.mask_embed_0 = PatchEmbed(patch_size=patch_size, in_chans=num_panoptic_class, embed_dim=embed_dim)
            self.decoder_pred_mask = nn.Linear(embed_dim, patch_size ** 2 * num_panoptic_class, bias=True)
            self.num_panoptic_class = num_panoptic_class
            self.final_layer_mask = nn.Conv2d(num_panoptic_class, num_panoptic_class, 3, padding=1) if conv else nn.Identity()
            self.final_act = nn.Tanh()
        self.use_ground_truth = use_ground_truth
        nn.init.trunc_normal_(self.pos_embed, std=.02)
        self.apply(_init_weights)
        for m in self.modules():  # zero-initialised zeroconvs (libs/uvit_t2i.py:366-369)
            if isinstance(m, nn.Conv1d):
                nn.init.constant_(m.weight, 0)
                nn.init.constant_(m.bias, 0)

    def _native_cfg_kwargs(self):
        return dict(img_size=self.img_size, patch_size=self.patch_size, in_chans=self.in_chans,
                    embed_dim=self.embed_dim, depth=self.depth, num_heads=self.num_heads, mlp_ratio=self.mlp_ratio,
                    conv=self.conv, skip=self.skip, qkv_bias=self.qkv_bias, mlp_time_embed=self.mlp_time_embed,
                    clip_dim=self.clip_dim, num_clip_token=self.num_clip_token, separate=self.separate,
                    enable_panoptic=self.enable_panoptic,
                    num_panoptic_class=getattr(self, "num_panoptic_class", 8), residual=self.residual)

    @torch.jit.ignore
    def no_weight_decay(self):
        return {'pos_embed'}

    def conv_params(self, mask=False):
        nat = self.native()
        if not self.conv:
            return None, None
        key = "final_layer_mask" if mask else "final_layer"
        if f"{key}.weight" not in nat.packed:
            layer = getattr(self, key)
            nat.packed[f"{key}.weight"] = layer.weight.detach().float().contiguous()
            nat.packed[f"{key}.bias"] = layer.bias.detach().float().contiguous()
        return nat.packed[f"{key}.weight"], nat.packed[f"{key}.bias"]

    def forward_pre(self, x, timesteps, context, mask_token=None, use_ground_truth=False, out=None, mask_out=None,
                    workspace=None):
        """Up to the heads: returns (eps_pre, mask_pre or None), both unpatchified, before conv / tanh."""
        _lib.require_gpu(x)
        nat = self.native()
        x = x.float().contiguous()
        B = x.shape[0]
        t = timesteps.to(device=x.device, dtype=torch.float32).reshape(-1)
        if t.numel() == 1 and B > 1:
            t = t.expand(B)
        t = t.contiguous()
        context = context.to(device=x.device, dtype=torch.float32).contiguous()
        if context.shape[0] != B:
            context = context.expand(B, -1, -1).contiguous()
        mt = None
        if mask_token is not None:
            if not (self.enable_panoptic and self.separate):
                raise NotImplementedError("mask tokens are supported for separate=True networks (the BASELINE "
                                          "panoptic config); separate=False is not on the HIP path")
            mt = mask_token.to(device=x.device, dtype=torch.float32).contiguous()
        if out is None:
            out = torch.empty(B, self.in_chans, self.img_size, self.img_size, device=x.device)
        if mt is not None and not use_ground_truth and mask_out is None:
            mask_out = torch.empty(B, self.num_panoptic_class, self.img_size, self.img_size, device=x.device)
        ws = nat.workspace(B, x.device) if workspace is None else workspace   # a lane's private workspace
        _lib.check(nat.lib.pdm_uvit_t2i_forward(nat.h, _lib.ptr(x), _lib.ptr(t), _lib.ptr(context), _lib.ptr(mt),
                                                int(bool(use_ground_truth)), _lib.ptr(out),
                                                _lib.ptr(mask_out if mt is not None else None), B, _lib.ptr(ws),
                                                ws.numel(), _lib.stream_ptr(x.device)), "pdm_uvit_t2i_forward")
        return out, (mask_out if mt is not None and not use_ground_truth else None)

    def forward(self, x, timesteps, context, mask_token=None, mask_0=None, use_ground_truth=False,
                enable_panoptic=False):
        """libs/uvit_t2i.py:378-525 (mask_0 is ignored there too: 392-396)."""
        self.use_ground_truth = use_ground_truth
        pre, mpre = self.forward_pre(x, timesteps, context, mask_token, use_ground_truth)
        B = pre.shape[0]
        if self.conv:
            w, b = self.conv_params()
            noise = torch.empty_like(pre)
            _lib.stage_epilogue(pre, B, conv_w=w, conv_b=b, m_out=noise)
        else:
            noise = pre
        if mask_token is None:
            return noise
        if use_ground_truth:
            return noise, mask_token
        y = torch.empty_like(mpre)
        w, b = self.conv_params(mask=True)
        _lib.stage_epilogue(mpre, B, conv_w=w, conv_b=b, act_tanh=True, m_out=y)
        return noise, y
