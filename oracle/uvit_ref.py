"""ORACLE (test infrastructure): fp32 CPU restatement of the U-ViT forwards.

Follows libs/uvit.py (class-conditional / unconditional U-ViT) and libs/uvit_t2i.py (text + panoptic
mask co-generation) of the reference.  Parameters are passed as a state_dict with the reference key
names.
"""
import math

import torch
import torch.nn.functional as F


def timestep_embedding(timesteps, dim, max_period=10000):
    """libs/uvit.py:20-38 — [cos(t f_i), sin(t f_i)], f_i = exp(-ln(max_period) i / half), zero pad if odd."""
    half = dim // 2
    i = torch.arange(half, dtype=torch.float32)
    freqs = torch.exp(-math.log(max_period) * i / half)
    args = timesteps.float()[:, None] * freqs[None, :]
    emb = torch.cat([torch.cos(args), torch.sin(args)], dim=-1)
    if dim % 2:
        emb = torch.cat([emb, torch.zeros_like(emb[:, :1])], dim=-1)
    return emb


def unpatchify(x, channels):
    """libs/uvit.py:46-51 — B (h w) (p1 p2 C) -> B C (h p1) (w p2)."""
    B, N, P = x.shape
    p = int(round((P // channels) ** 0.5))
    h = int(round(N ** 0.5))
    assert h * h == N and p * p * channels == P
    x = x.reshape(B, h, h, p, p, channels)
    x = x.permute(0, 5, 1, 3, 2, 4)  # B C h p1 w p2
    return x.reshape(B, channels, h * p, h * p)


def patch_embed(sd, prefix, x, p):
    """libs/uvit.py:123-135 — Conv2d(k=s=p) then flatten(2).transpose(1,2)."""
    y = F.conv2d(x, sd[f"{prefix}.proj.weight"], sd[f"{prefix}.proj.bias"], stride=p)
    return y.flatten(2).transpose(1, 2)


def attention(sd, prefix, x, num_heads):
    """libs/uvit.py:66-92 (flash branch): qkv -> (3,H,Dh) split -> fp32 SDPA (scale Dh^-1/2) -> proj."""
    B, L, D = x.shape
    qkv = F.linear(x, sd[f"{prefix}.qkv.weight"], sd.get(f"{prefix}.qkv.bias"))
    qkv = qkv.reshape(B, L, 3, num_heads, D // num_heads).permute(2, 0, 3, 1, 4).float()
    q, k, v = qkv[0], qkv[1], qkv[2]
    s = (q @ k.transpose(-2, -1)) * (D // num_heads) ** -0.5
    o = torch.softmax(s, dim=-1) @ v
    o = o.permute(0, 2, 1, 3).reshape(B, L, D)
    return F.linear(o, sd[f"{prefix}.proj.weight"], sd[f"{prefix}.proj.bias"])


def block(sd, prefix, x, num_heads, skip=None):
    """libs/uvit.py:115-120 (= libs/uvit_t2i.py:177-226 with the mask branch disabled at 183)."""
    if skip is not None:
        x = F.linear(torch.cat([x, skip], dim=-1), sd[f"{prefix}.skip_linear.weight"], sd[f"{prefix}.skip_linear.bias"])
    D = x.shape[-1]
    h = F.layer_norm(x, (D,), sd[f"{prefix}.norm1.weight"], sd[f"{prefix}.norm1.bias"], eps=1e-5)
    x = x + attention(sd, f"{prefix}.attn", h, num_heads)
    h = F.layer_norm(x, (D,), sd[f"{prefix}.norm2.weight"], sd[f"{prefix}.norm2.bias"], eps=1e-5)
    h = F.linear(h, sd[f"{prefix}.mlp.fc1.weight"], sd[f"{prefix}.mlp.fc1.bias"])
    h = F.gelu(h)  # nn.GELU exact (erf): libs/uvit.py:98 act_layer default
    h = F.linear(h, sd[f"{prefix}.mlp.fc2.weight"], sd[f"{prefix}.mlp.fc2.bias"])
    return x + h


def _time_token(sd, timesteps, D, mlp_time_embed):
    te = timestep_embedding(timesteps, D)
    if mlp_time_embed:  # libs/uvit.py:150-154
        te = F.linear(te, sd["time_embed.0.weight"], sd["time_embed.0.bias"])
        te = F.silu(te)
        te = F.linear(te, sd["time_embed.2.weight"], sd["time_embed.2.bias"])
    return te


def uvit_forward(sd, cfg, x, timesteps, y=None):
    """libs/uvit.py:201-230 — tokens [label, time, patches] + pos_embed, in-blocks, mid, out-blocks with
    long skips, LN, decoder_pred, drop extras, unpatchify, optional 3x3 final conv."""
    D, p, C = cfg["embed_dim"], cfg["patch_size"], cfg.get("in_chans", 3)
    depth, heads = cfg["depth"], cfg["num_heads"]
    num_classes = cfg.get("num_classes", -1)
    x = patch_embed(sd, "patch_embed", x, p)
    B, L, _ = x.shape
    tt = _time_token(sd, timesteps, D, cfg.get("mlp_time_embed", False)).unsqueeze(1)
    x = torch.cat([tt, x], dim=1)
    if y is not None:
        x = torch.cat([sd["label_emb.weight"][y].unsqueeze(1), x], dim=1)
    x = x + sd["pos_embed"]
    extras = 2 if num_classes > 0 else 1
    skips = []
    for i in range(depth // 2):
        x = block(sd, f"in_blocks.{i}", x, heads)
        skips.append(x)
    x = block(sd, "mid_block", x, heads)
    for i in range(depth // 2):
        x = block(sd, f"out_blocks.{i}", x, heads, skip=skips.pop())
    x = F.layer_norm(x, (D,), sd["norm.weight"], sd["norm.bias"], eps=1e-5)
    x = F.linear(x, sd["decoder_pred.weight"], sd["decoder_pred.bias"])
    assert x.shape[1] == extras + L
    x = unpatchify(x[:, extras:, :], C)
    if cfg.get("conv", True):
        x = F.conv2d(x, sd["final_layer.weight"], sd["final_layer.bias"], padding=1)
    return x


def _zeroconv(sd, idx, x):
    """libs/uvit_t2i.py:246-257 — Conv1d(D, D, 1) over the token axis == per-token Linear."""
    w = sd[f"zero_convs.{idx}.conv.weight"][:, :, 0]
    return F.linear(x, w, sd[f"zero_convs.{idx}.conv.bias"])


def uvit_t2i_forward(sd, cfg, x, timesteps, context, mask_token=None, mask_0=None,
                     use_ground_truth=False, enable_panoptic=False):
    """libs/uvit_t2i.py:378-525.

    Image stream tokens [time, context x num_clip_token, patches]; with `separate=True` and a mask token,
    a second block stack runs over mx = cat(x_before_block, m) (L = extras + 2*patches) and injects
    zeroconv(mx[:, :extras+L]) into x after every layer (odd zero_convs indices).  mask_0 is ignored
    (392-396 commented out).  Returns eps or (eps, tanh(conv3x3(unpatchify(decoder_pred_mask(m))))).
    """
    D, p, C = cfg["embed_dim"], cfg["patch_size"], cfg.get("in_chans", 3)
    depth, heads = cfg["depth"], cfg["num_heads"]
    separate = cfg.get("separate", False)
    n_tok = cfg.get("num_clip_token", 77)
    K = cfg.get("num_panoptic_class", 8)
    conv = cfg.get("conv", True)
    extras = 1 + n_tok
    x = patch_embed(sd, "patch_embed", x, p)
    B, L, _ = x.shape
    tt = _time_token(sd, timesteps, D, cfg.get("mlp_time_embed", False)).unsqueeze(1)
    ctx = F.linear(context, sd["context_embed.weight"], sd["context_embed.bias"])
    m = None
    if mask_token is not None:
        me = patch_embed(sd, "mask_embed", mask_token, p)
        if not separate:
            x = torch.cat([tt, ctx, x, me], dim=1) + sd["pos_embed"]
        else:
            x = torch.cat([tt, ctx, x], dim=1) + sd["pos_embed"]
            m = me + sd["pos_embed_mask"]
    else:
        x = torch.cat([tt, ctx, x], dim=1) + sd["pos_embed"][:, :extras + L, :]
    two = separate and mask_token is not None
    skips, skips_mask = [], []
    layer_i = 0
    for i in range(depth // 2):
        if two:
            mx = torch.cat([x, m], dim=1)
        x = block(sd, f"in_blocks.{i}", x, heads)
        if two:
            mx = block(sd, f"in_blocks_mask.{i}", mx, heads)
            m = mx[:, extras + L:, :]
            x = x + _zeroconv(sd, 2 * layer_i + 1, mx[:, :extras + L, :])
            skips_mask.append(mx)
        skips.append(x)
        layer_i += 1
    if two:
        mx = torch.cat([x, m], dim=1)
    x = block(sd, "mid_block", x, heads)
    if two:
        mx = block(sd, "mid_block_mask", mx, heads)
        m = mx[:, extras + L:, :]
        x = x + _zeroconv(sd, 2 * layer_i + 1, mx[:, :extras + L, :])
        layer_i += 1
    for i in range(depth // 2):
        if two:
            mx = torch.cat([x, m], dim=1)
        x = block(sd, f"out_blocks.{i}", x, heads, skip=skips.pop())
        if two:
            mx = block(sd, f"out_blocks_mask.{layer_i - 1 - depth // 2}", mx, heads, skip=skips_mask.pop())
            m = mx[:, extras + L:, :]
            x = x + _zeroconv(sd, 2 * layer_i + 1, mx[:, :extras + L, :])
        layer_i += 1
    x = F.layer_norm(x, (D,), sd["norm.weight"], sd["norm.bias"], eps=1e-5)
    y = None
    if mask_token is not None:
        if use_ground_truth:  # 486-496
            img = x[:, extras:extras + L, :]
            msk = x[:, extras + L:, :] if not separate else m
            noise = F.linear(img + msk, sd["decoder_pred.weight"], sd["decoder_pred.bias"])
            y = mask_token
        else:
            if not separate:
                noise = F.linear(x[:, extras:extras + L, :], sd["decoder_pred.weight"], sd["decoder_pred.bias"])
                y = F.linear(x[:, extras + L:, :], sd["decoder_pred_mask.weight"], sd["decoder_pred_mask.bias"])
            else:
                noise = F.linear(x[:, extras:, :], sd["decoder_pred.weight"], sd["decoder_pred.bias"])
                y = F.linear(m, sd["decoder_pred_mask.weight"], sd["decoder_pred_mask.bias"])
            y = unpatchify(y, K)
            if conv:
                y = F.conv2d(y, sd["final_layer_mask.weight"], sd["final_layer_mask.bias"], padding=1)
            y = torch.tanh(y)
    else:
        noise = F.linear(x[:, extras:extras + L, :], sd["decoder_pred.weight"], sd["decoder_pred.bias"])
    noise = unpatchify(noise, C)
    if conv:
        noise = F.conv2d(noise, sd["final_layer.weight"], sd["final_layer.bias"], padding=1)
    if mask_token is not None:
        return noise, y
    return noise
