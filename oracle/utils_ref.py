"""ORACLE (test infrastructure): integer / small helpers around the sampler.

* int2bits / bits2int   utils.py:475-488 / 490-518 (8 analog bits, MSB first)
* unpreprocess          datasets.py:104-108 (clamp(0.5 (v + 1), 0, 1))
* amortize              utils.py:452-455
* save_image_u8         torchvision save_image as called by utils.py:629/633 on unpreprocessed samples
* color_map             utils.py:532-543 (colormap[id], B x H x W x 3)
"""
import numpy as np


def int2bits(x, n=8):
    """x int [b, c, h, w] -> bits [b, n*c, h, w]: channel i holds bit (n-1-i) (MSB first)."""
    x = np.asarray(x).astype(np.int64)
    planes = [(x >> (n - 1 - i)) & 1 for i in range(n)]
    return np.concatenate(planes, axis=1)


def bits2int(bits, n=8):
    """bits [b, n, h, w] (0/1) -> int [b, 1, h, w] = sum_i b_i 2^(n-1-i)."""
    b = np.asarray(bits).astype(np.int64)
    out = np.zeros((b.shape[0], 1) + b.shape[2:], dtype=np.int64)
    for i in range(n):
        out[:, 0] += b[:, i] << (n - 1 - i)
    return out


def unpreprocess(v):
    return np.clip(0.5 * (np.asarray(v, dtype=np.float32) + 1.0), 0.0, 1.0)


def amortize(n_samples, batch_size):
    k = n_samples // batch_size
    r = n_samples % batch_size
    return k * [batch_size] if r == 0 else k * [batch_size] + [r]


def save_image_u8(img):
    """[B, C, H, W] fp32 -> [B, H, W, C] uint8: unpreprocess, then `mul(255).add_(0.5).clamp_(0, 255)` and a
    truncating cast (torchvision save_image); every op rounded to fp32 separately, as torch does."""
    v = unpreprocess(img)
    u = (v * np.float32(255.0)).astype(np.float32)
    u = (u + np.float32(0.5)).astype(np.float32)
    u = np.clip(u, 0.0, 255.0)
    return u.astype(np.uint8).transpose(0, 2, 3, 1)


def color_map(ids, colormap):
    """ids [B, 1, H, W] or [B, H, W] integers -> [B, H, W, 3] uint8 = colormap[id]."""
    ids = np.asarray(ids).astype(np.int64)
    if ids.ndim == 4:
        ids = ids[:, 0]
    return np.asarray(colormap)[ids].astype(np.uint8)
