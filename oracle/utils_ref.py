"""ORACLE (test infrastructure): integer / small helpers around the sampler.

* int2bits / bits2int   utils.py:475-488 / 490-518 (8 analog bits, MSB first)
* unpreprocess          datasets.py:104-108 (clamp(0.5 (v + 1), 0, 1))
* amortize              utils.py:452-455
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
