"""Deterministic synthetic weights with the reference's state_dict key names and shapes.

No checkpoints exist offline, so every parity test and the benchmark use weights
from this generator.  Key names / shapes follow the probe listing in SURVEY.md §8a row a20:

  * U-ViT          libs/uvit.py:138-195        (PatchEmbed 123-135, Block 95-120, Mlp libs/timm.py:96-112)
  * U-ViT t2i      libs/uvit_t2i.py:258-359    (zeroconv 246-257, mask stream 307-326, mask head 335-348)
  * KL-f8 decoder  libs/autoencoder.py:303-409 (+ post_quant_conv 420, get_model ddconfig 471-484)

`init="reference"` mimics the reference init (libs/uvit.py:185-195: trunc_normal(.02) Linear
weights and pos_embed, zero biases, LayerNorm 1/0, default Conv init, zero zeroconv); `init="random"`
additionally randomises biases, norms and zeroconvs so fixtures exercise every term.
"""
import math
from collections import OrderedDict

import torch

# --------------------------------------------------------------------------------------------
# parameter specs: list of (name, shape, kind)
#   kinds: lin_w, lin_b, ln_w, ln_b, pos, emb, conv_w(fan_in), conv_b(fan_in), zero_w, zero_b, gn_w, gn_b


def _block_spec(prefix, D, mlp_ratio, qkv_bias, skip):
    H = int(D * mlp_ratio)
    s = [(f"{prefix}.norm1.weight", (D,), "ln_w"), (f"{prefix}.norm1.bias", (D,), "ln_b"),
         (f"{prefix}.attn.qkv.weight", (3 * D, D), "lin_w")]
    if qkv_bias:
        s.append((f"{prefix}.attn.qkv.bias", (3 * D,), "lin_b"))
    s += [(f"{prefix}.attn.proj.weight", (D, D), "lin_w"), (f"{prefix}.attn.proj.bias", (D,), "lin_b"),
          (f"{prefix}.norm2.weight", (D,), "ln_w"), (f"{prefix}.norm2.bias", (D,), "ln_b"),
          (f"{prefix}.mlp.fc1.weight", (H, D), "lin_w"), (f"{prefix}.mlp.fc1.bias", (H,), "lin_b"),
          (f"{prefix}.mlp.fc2.weight", (D, H), "lin_w"), (f"{prefix}.mlp.fc2.bias", (D,), "lin_b")]
    if skip:
        s += [(f"{prefix}.skip_linear.weight", (D, 2 * D), "lin_w"),
              (f"{prefix}.skip_linear.bias", (D,), "lin_b")]
    return s


def uvit_spec(img_size=224, patch_size=16, in_chans=3, embed_dim=768, depth=12, num_heads=12,
              mlp_ratio=4., qkv_bias=False, mlp_time_embed=False, num_classes=-1, conv=True,
              skip=True, **_ignored):
    D, p, C = embed_dim, patch_size, in_chans
    n_patches = (img_size // p) ** 2
    extras = 2 if num_classes > 0 else 1
    s = [("pos_embed", (1, extras + n_patches, D), "pos"),
         ("patch_embed.proj.weight", (D, C, p, p), "conv_w"), ("patch_embed.proj.bias", (D,), "conv_b")]
    if mlp_time_embed:
        s += [("time_embed.0.weight", (4 * D, D), "lin_w"), ("time_embed.0.bias", (4 * D,), "lin_b"),
              ("time_embed.2.weight", (D, 4 * D), "lin_w"), ("time_embed.2.bias", (D,), "lin_b")]
    if num_classes > 0:
        s.append(("label_emb.weight", (num_classes, D), "emb"))
    for i in range(depth // 2):
        s += _block_spec(f"in_blocks.{i}", D, mlp_ratio, qkv_bias, False)
    s += _block_spec("mid_block", D, mlp_ratio, qkv_bias, False)
    for i in range(depth // 2):
        s += _block_spec(f"out_blocks.{i}", D, mlp_ratio, qkv_bias, skip)
    s += [("norm.weight", (D,), "ln_w"), ("norm.bias", (D,), "ln_b"),
          ("decoder_pred.weight", (p * p * C, D), "lin_w"), ("decoder_pred.bias", (p * p * C,), "lin_b")]
    if conv:
        s += [("final_layer.weight", (C, C, 3, 3), "conv_w"), ("final_layer.bias", (C,), "conv_b")]
    return s


def uvit_t2i_spec(img_size=224, patch_size=16, in_chans=3, embed_dim=768, depth=12, num_heads=12,
                  mlp_ratio=4., qkv_bias=False, mlp_time_embed=False, clip_dim=768, num_clip_token=77,
                  conv=True, skip=True, num_panoptic_class=8, enable_panoptic=True, separate=False,
                  **_ignored):
    D, p, C = embed_dim, patch_size, in_chans
    n_patches = (img_size // p) ** 2
    extras = 1 + num_clip_token
    s = []
    if enable_panoptic and not separate:
        s.append(("pos_embed", (1, extras + 2 * n_patches, D), "pos"))
    else:
        s.append(("pos_embed", (1, extras + n_patches, D), "pos"))
    if enable_panoptic and separate:
        s.append(("pos_embed_mask", (1, n_patches, D), "pos"))
    s += [("patch_embed.proj.weight", (D, C, p, p), "conv_w"), ("patch_embed.proj.bias", (D,), "conv_b")]
    if mlp_time_embed:
        s += [("time_embed.0.weight", (4 * D, D), "lin_w"), ("time_embed.0.bias", (4 * D,), "lin_b"),
              ("time_embed.2.weight", (D, 4 * D), "lin_w"), ("time_embed.2.bias", (D,), "lin_b")]
    s += [("context_embed.weight", (D, clip_dim), "lin_w"), ("context_embed.bias", (D,), "lin_b")]
    for i in range(depth // 2):
        s += _block_spec(f"in_blocks.{i}", D, mlp_ratio, qkv_bias, False)
    s += _block_spec("mid_block", D, mlp_ratio, qkv_bias, False)
    for i in range(depth // 2):
        s += _block_spec(f"out_blocks.{i}", D, mlp_ratio, qkv_bias, skip)
    if separate:
        for i in range(depth // 2):
            s += _block_spec(f"in_blocks_mask.{i}", D, mlp_ratio, qkv_bias, False)
        s += _block_spec("mid_block_mask", D, mlp_ratio, qkv_bias, False)
        for i in range(depth // 2):
            s += _block_spec(f"out_blocks_mask.{i}", D, mlp_ratio, qkv_bias, skip)
        for i in range(depth * 2 + 2):
            s += [(f"zero_convs.{i}.conv.weight", (D, D, 1), "zero_w"), (f"zero_convs.{i}.conv.bias", (D,), "zero_b")]
    s += [("norm.weight", (D,), "ln_w"), ("norm.bias", (D,), "ln_b"),
          ("decoder_pred.weight", (p * p * C, D), "lin_w"), ("decoder_pred.bias", (p * p * C,), "lin_b")]
    if conv:
        s += [("final_layer.weight", (C, C, 3, 3), "conv_w"), ("final_layer.bias", (C,), "conv_b")]
    if enable_panoptic:
        K = num_panoptic_class
        s += [("mask_embed.proj.weight", (D, K, p, p), "conv_w"), ("mask_embed.proj.bias", (D,), "conv_b"),
              ("mask_embed_0.proj.weight", (D, K, p, p), "conv_w"), ("mask_embed_0.proj.bias", (D,), "conv_b"),
              ("decoder_pred_mask.weight", (p * p * K, D), "lin_w"), ("decoder_pred_mask.bias", (p * p * K,), "lin_b")]
        if conv:
            s += [("final_layer_mask.weight", (K, K, 3, 3), "conv_w"), ("final_layer_mask.bias", (K,), "conv_b")]
    return s


DECODER_DDCONFIG = dict(double_z=True, z_channels=4, resolution=256, in_channels=3, out_ch=3, ch=128,
                        ch_mult=[1, 2, 4, 4], num_res_blocks=2, attn_resolutions=[], dropout=0.0)


def _resblock_spec(prefix, cin, cout):
    s = [(f"{prefix}.norm1.weight", (cin,), "gn_w"), (f"{prefix}.norm1.bias", (cin,), "gn_b"),
         (f"{prefix}.conv1.weight", (cout, cin, 3, 3), "conv_w"), (f"{prefix}.conv1.bias", (cout,), "conv_b"),
         (f"{prefix}.norm2.weight", (cout,), "gn_w"), (f"{prefix}.norm2.bias", (cout,), "gn_b"),
         (f"{prefix}.conv2.weight", (cout, cout, 3, 3), "conv_w"), (f"{prefix}.conv2.bias", (cout,), "conv_b")]
    if cin != cout:
        s += [(f"{prefix}.nin_shortcut.weight", (cout, cin, 1, 1), "conv_w"),
              (f"{prefix}.nin_shortcut.bias", (cout,), "conv_b")]
    return s


def decoder_spec(ch=128, out_ch=3, ch_mult=(1, 2, 4, 4), num_res_blocks=2, z_channels=4, embed_dim=4,
                 prefix="decoder", **_ignored):
    """Parameters used by FrozenAutoencoderKL.decode (libs/autoencoder.py:446-450): post_quant_conv + Decoder."""
    n = len(ch_mult)
    block_in = ch * ch_mult[-1]
    s = [("post_quant_conv.weight", (z_channels, embed_dim, 1, 1), "conv_w"),
         ("post_quant_conv.bias", (z_channels,), "conv_b"),
         (f"{prefix}.conv_in.weight", (block_in, z_channels, 3, 3), "conv_w"),
         (f"{prefix}.conv_in.bias", (block_in,), "conv_b")]
    s += _resblock_spec(f"{prefix}.mid.block_1", block_in, block_in)
    s += [(f"{prefix}.mid.attn_1.norm.weight", (block_in,), "gn_w"), (f"{prefix}.mid.attn_1.norm.bias", (block_in,), "gn_b")]
    for nm in ("q", "k", "v", "proj_out"):
        s += [(f"{prefix}.mid.attn_1.{nm}.weight", (block_in, block_in, 1, 1), "conv_w"),
              (f"{prefix}.mid.attn_1.{nm}.bias", (block_in,), "conv_b")]
    s += _resblock_spec(f"{prefix}.mid.block_2", block_in, block_in)
    for i_level in reversed(range(n)):
        block_out = ch * ch_mult[i_level]
        for i_block in range(num_res_blocks + 1):
            s += _resblock_spec(f"{prefix}.up.{i_level}.block.{i_block}", block_in, block_out)
            block_in = block_out
        if i_level != 0:
            s += [(f"{prefix}.up.{i_level}.upsample.conv.weight", (block_in, block_in, 3, 3), "conv_w"),
                  (f"{prefix}.up.{i_level}.upsample.conv.bias", (block_in,), "conv_b")]
    s += [(f"{prefix}.norm_out.weight", (block_in,), "gn_w"), (f"{prefix}.norm_out.bias", (block_in,), "gn_b"),
          (f"{prefix}.conv_out.weight", (out_ch, block_in, 3, 3), "conv_w"), (f"{prefix}.conv_out.bias", (out_ch,), "conv_b")]
    return s


def _fan_in(shape):
    f = 1
    for d in shape[1:]:
        f *= d
    return f


def _fill(t, name, shape, kind, init, gen, fan_in_of):
    if kind == "lin_w" or kind == "pos":
        t.normal_(0.0, 0.02, generator=gen).clamp_(-2.0, 2.0)
    elif kind == "emb":
        t.normal_(0.0, 1.0, generator=gen)
    elif kind in ("conv_w", "conv_b"):
        bound = 1.0 / math.sqrt(fan_in_of)
        t.uniform_(-bound, bound, generator=gen)
    elif kind in ("ln_w", "gn_w"):
        if init == "random":
            t.normal_(0.0, 0.1, generator=gen).add_(1.0)
        else:
            t.fill_(1.0)
    elif kind in ("ln_b", "gn_b", "lin_b"):
        if init == "random":
            t.normal_(0.0, 0.05 if kind == "lin_b" else 0.1, generator=gen)
        else:
            t.zero_()
    elif kind in ("zero_w", "zero_b"):
        if init == "random":
            t.normal_(0.0, 0.02, generator=gen)
        else:
            t.zero_()
    else:
        raise ValueError(kind)


def make_state_dict(spec, seed=0, init="reference", device="cpu", dtype=torch.float32):
    """Materialise a spec with a seeded generator (one generator, spec order)."""
    if init not in ("reference", "random"):
        raise ValueError(f"init must be 'reference' or 'random', got {init!r}")
    dev = torch.device(device)
    gen = torch.Generator(device=dev)
    gen.manual_seed(seed)
    sd = OrderedDict()
    conv_fan = {}
    for name, shape, kind in spec:
        if kind == "conv_w":
            conv_fan[name.rsplit(".", 1)[0]] = _fan_in(shape)
    for name, shape, kind in spec:
        t = torch.empty(shape, dtype=torch.float32, device=dev)
        fan = conv_fan.get(name.rsplit(".", 1)[0], 1) if kind in ("conv_w", "conv_b") else 1
        _fill(t, name, shape, kind, init, gen, fan)
        sd[name] = t.to(dtype)
    return sd


def nnet_state_dict(nnet_cfg, seed=0, init="reference", device="cpu"):
    cfg = dict(nnet_cfg)
    name = cfg.pop("name")
    if name == "uvit":
        spec = uvit_spec(**cfg)
    elif name == "uvit_t2i":
        spec = uvit_t2i_spec(**cfg)
    else:
        raise NotImplementedError(name)
    return make_state_dict(spec, seed=seed, init=init, device=device)


def decoder_state_dict(seed=0, init="reference", device="cpu", ch=128, ch_mult=(1, 2, 4, 4),
                       num_res_blocks=2):
    return make_state_dict(decoder_spec(ch=ch, ch_mult=ch_mult, num_res_blocks=num_res_blocks),
                           seed=seed, init=init, device=device)


def param_count(spec):
    n = 0
    for _, shape, _ in spec:
        k = 1
        for d in shape:
            k *= d
        n += k
    return n
