"""ORACLE (test infrastructure): fp32 CPU restatement of FrozenAutoencoderKL.decode.

libs/autoencoder.py: Normalize = GroupNorm(32, eps=1e-6) (31-32), swish (26-28), Upsample nearest x2 +
conv3x3 (35-50), ResnetBlock (75-134, temb None, nin_shortcut 1x1 when channels change), AttnBlock
(143-195, single head over h*w, scale C^-1/2), Decoder.forward (376-409), decode (446-450:
z / scale_factor -> post_quant_conv -> decoder), ddconfig of get_model (471-484).
"""
import torch
import torch.nn.functional as F


def _gn(sd, p, x):
    return F.group_norm(x, 32, sd[f"{p}.weight"], sd[f"{p}.bias"], eps=1e-6)


def _swish(x):
    return x * torch.sigmoid(x)


def _conv(sd, p, x, pad):
    return F.conv2d(x, sd[f"{p}.weight"], sd[f"{p}.bias"], padding=pad)


def resnet_block(sd, p, x):
    h = _conv(sd, f"{p}.conv1", _swish(_gn(sd, f"{p}.norm1", x)), 1)
    h = _conv(sd, f"{p}.conv2", _swish(_gn(sd, f"{p}.norm2", h)), 1)
    if f"{p}.nin_shortcut.weight" in sd:
        x = _conv(sd, f"{p}.nin_shortcut", x, 0)
    return x + h


def attn_block(sd, p, x):
    h = _gn(sd, f"{p}.norm", x)
    q = _conv(sd, f"{p}.q", h, 0)
    k = _conv(sd, f"{p}.k", h, 0)
    v = _conv(sd, f"{p}.v", h, 0)
    b, c, hh, ww = q.shape
    q = q.reshape(b, c, hh * ww).permute(0, 2, 1)
    k = k.reshape(b, c, hh * ww)
    w = torch.softmax(torch.bmm(q, k) * (int(c) ** -0.5), dim=2)
    o = torch.bmm(v.reshape(b, c, hh * ww), w.permute(0, 2, 1)).reshape(b, c, hh, ww)
    return x + _conv(sd, f"{p}.proj_out", o, 0)


def decode(sd, z, scale_factor=0.18215, ch_mult=(1, 2, 4, 4), num_res_blocks=2, prefix="decoder"):
    z = z / scale_factor
    z = _conv(sd, "post_quant_conv", z, 0)
    h = _conv(sd, f"{prefix}.conv_in", z, 1)
    h = resnet_block(sd, f"{prefix}.mid.block_1", h)
    h = attn_block(sd, f"{prefix}.mid.attn_1", h)
    h = resnet_block(sd, f"{prefix}.mid.block_2", h)
    for i_level in reversed(range(len(ch_mult))):
        for i_block in range(num_res_blocks + 1):
            h = resnet_block(sd, f"{prefix}.up.{i_level}.block.{i_block}", h)
        if i_level != 0:
            h = F.interpolate(h, scale_factor=2.0, mode="nearest")
            h = _conv(sd, f"{prefix}.up.{i_level}.upsample.conv", h, 1)
    h = _swish(_gn(sd, f"{prefix}.norm_out", h))
    return _conv(sd, f"{prefix}.conv_out", h, 1)
