"""Output stage of the sampling path: `utils.sample2dir` (utils.py:561-640) minus
the wandb/FID plumbing.

* `images_to_u8`      decoded fp32 [B, 3, H, W] -> uint8 [B, H, W, 3] on the GPU (pdm_images_to_u8):
                      unpreprocess (datasets.py:104-108) + torchvision `save_image` quantisation, bit-exact
* `masks_to_ids_rgb`  analog-bit masks [B, 8, h, w] -> ids = bits2int(pred_mask > 0) (utils.py:490-518) and
                      colour-mapped uint8 pixels colormap[id] (utils.py:532-543), on the GPU
* `write_samples`     PNG files named like the reference (`{sample_idx + 10000 * (idx // 4992)}.png`,
                      utils.py:629-635), images under `path`, colour masks under `mask_path`
"""
import os
import warnings

import numpy as np
import torch

from . import _lib


def default_colormap(seed=0):
    """The reference draws `torch.randint(0, 255, (256, 3))` once and caches it in colormap.pt
    (utils.py:521-530); here it is seeded so runs are reproducible.  Pass the reference's own table to
    reproduce its colours."""
    g = torch.Generator().manual_seed(seed)
    return torch.randint(0, 255, (256, 3), generator=g)


def images_to_u8(img, check_finite=True):
    """check_finite: warn when the batch holds NaN/inf (the kernel writes NaN pixels as 0, csrc/output.hip)."""
    lib = _lib.load()
    _lib.require_gpu(img)
    img = img.float().contiguous()
    if check_finite:
        bad = int((~torch.isfinite(img)).sum())
        if bad:
            warnings.warn(f"images_to_u8: {bad} non-finite values in the decoded batch (written as 0 / 255)")
    B, C, H, W = img.shape
    out = torch.empty(B, H, W, C, dtype=torch.uint8, device=img.device)
    _lib.check(lib.pdm_images_to_u8(_lib.ptr(img), _lib.ptr(out), B, C, H, W, _lib.stream_ptr(img.device)),
               "pdm_images_to_u8")
    return out


def masks_to_ids_rgb(pred_mask, colormap=None):
    lib = _lib.load()
    _lib.require_gpu(pred_mask)
    pm = pred_mask.float().contiguous()
    B, n, H, W = pm.shape
    cmap = (default_colormap() if colormap is None else colormap).to(device=pm.device, dtype=torch.int32).contiguous()
    if tuple(cmap.shape) != (256, 3):
        raise ValueError(f"colormap must be [256, 3], got {tuple(cmap.shape)}")
    ids = torch.empty(B, H, W, dtype=torch.int32, device=pm.device)
    rgb = torch.empty(B, H, W, 3, dtype=torch.uint8, device=pm.device)
    _lib.check(lib.pdm_mask_bits_to_rgb(_lib.ptr(pm), n, _lib.ptr(cmap), _lib.ptr(ids), _lib.ptr(rgb), B, H, W,
                                        _lib.stream_ptr(pm.device)), "pdm_mask_bits_to_rgb")
    return ids, rgb


def sample_file_name(sample_idx, idx):
    """utils.py:629-635: `{sample_idx + 10000 * (idx // 4992)}.png` (idx = running count of saved images)."""
    return f"{int(sample_idx) + 10000 * (int(idx) // 4992)}.png"


def save_png(arr_hwc_u8, path):
    from PIL import Image
    Image.fromarray(np.ascontiguousarray(arr_hwc_u8)).save(path)


def write_samples(path, images_u8, sample_idx, start_idx=0, mask_path=None, masks_rgb_u8=None):
    """Write one PNG per image (uint8 HWC, host or device tensors/arrays); returns the next running idx."""
    os.makedirs(path, exist_ok=True)
    if mask_path is not None:
        os.makedirs(mask_path, exist_ok=True)
    imgs = images_u8.cpu().numpy() if torch.is_tensor(images_u8) else np.asarray(images_u8)
    masks = None
    if masks_rgb_u8 is not None:
        masks = masks_rgb_u8.cpu().numpy() if torch.is_tensor(masks_rgb_u8) else np.asarray(masks_rgb_u8)
    idx = start_idx
    for i in range(imgs.shape[0]):
        name = sample_file_name(sample_idx[i], idx)
        save_png(imgs[i], os.path.join(path, name))
        if masks is not None and mask_path is not None:
            save_png(masks[i], os.path.join(mask_path, name))
        idx += 1
    return idx
