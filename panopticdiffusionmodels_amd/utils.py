"""Host helpers on the sampling path (utils.py of the reference, hot-path subset).

* get_nnet        utils.py:291-299
* amortize        utils.py:452-455
* int2bits/bits2int  utils.py:475-518 (analog bits, MSB first; bits2int returns on CPU like the reference)
* unpreprocess    datasets.py:104-108
"""
import torch


def get_nnet(name, **kwargs):
    if name == "uvit":
        from .libs.uvit import UViT
        return UViT(**kwargs)
    if name == "uvit_t2i":
        from .libs.uvit_t2i import UViT
        return UViT(**kwargs)
    raise NotImplementedError(name)


def amortize(n_samples, batch_size):
    k = n_samples // batch_size
    r = n_samples % batch_size
    return k * [batch_size] if r == 0 else k * [batch_size] + [r]


def int2bits(x, n=8, out_dtype=None):
    """(b, c, h, w) integers -> (b, n*c, h, w) bits, channel i = bit n-1-i (utils.py:475-488)."""
    x = x.to(torch.int32)
    y = torch.cat([torch.bitwise_right_shift(x, n - 1 - i) for i in range(n)], dim=1).remainder(2)
    if out_dtype is not None and out_dtype != y.dtype:
        y = y.to(out_dtype)
    return y


def bits2int(x, out_dtype=torch.int, n=8, c=1):
    """(b, n, h, w) bits -> (b, 1, h, w) float integer map on the CPU (utils.py:490-518)."""
    x = x.to(out_dtype)
    w = torch.tensor([2 ** (n - 1 - i) for i in range(n)], dtype=torch.float32, device=x.device)
    y = (x[:, :n].float() * w[None, :, None, None]).sum(dim=1, keepdim=True)
    return y.cpu()


def unpreprocess(v):
    return (0.5 * (v + 1.0)).float().clamp_(0.0, 1.0)
