"""Binding between an nn.Module holding the reference-named parameters and a pdm_uvit handle.

The module keeps fp32 parameters under the reference's state_dict keys (so `load_state_dict` of a
reference checkpoint works unchanged, eval_ldm_discrete.py:46).  On first GPU use the parameters are
packed once into the layouts libpdm expects (Linear weights -> bf16 [out, in]; decoder heads padded to a
multiple of 16 rows; conv / embedding tables fp32; norm1 / norm2 folded into attn.qkv / mlp.fc1, see
`_ln_fold`; with fp8=True the block Linears as MXFP8, see `_mx_weight`) and their device addresses are
registered with the handle.  Any load_state_dict / .to() invalidates the packed copy.
"""
import ctypes
import math

import torch
import torch.nn as nn

from . import _lib


def cfg_struct(kw, t2i):
    c = _lib.PdmUvitCfg()
    D = int(kw["embed_dim"])
    c.img_size = int(kw["img_size"])
    c.patch_size = int(kw["patch_size"])
    c.in_chans = int(kw.get("in_chans", 3))
    c.embed_dim = D
    c.depth = int(kw["depth"])
    c.num_heads = int(kw["num_heads"])
    c.mlp_hidden = int(D * kw.get("mlp_ratio", 4.0))
    c.num_classes = int(kw.get("num_classes", -1)) if not t2i else -1
    c.conv = int(bool(kw.get("conv", True)))
    c.skip = int(bool(kw.get("skip", True)))
    c.qkv_bias = int(bool(kw.get("qkv_bias", False)))
    c.mlp_time_embed = int(bool(kw.get("mlp_time_embed", False)))
    c.t2i = int(t2i)
    c.clip_dim = int(kw.get("clip_dim", 768)) if t2i else 0
    c.num_clip_token = int(kw.get("num_clip_token", 77)) if t2i else 0
    c.separate = int(bool(kw.get("separate", False))) if t2i else 0
    c.enable_panoptic = int(bool(kw.get("enable_panoptic", True))) if t2i else 0
    c.num_panoptic_class = int(kw.get("num_panoptic_class", 8)) if t2i else 0
    c.fp8 = int(bool(kw.get("fp8", False)))
    c.fp8_linears = int(kw.get("fp8_linears", 0)) if c.fp8 else 0
    c.residual_fp32 = int(kw.get("residual", "bf16") == "fp32")
    return c


def gcol_table(w):
    """[N, K] (dequantised) weight -> bf16 [N, 16]: per row n the sums c_t of its 256-column groups t < 8 as a
    bf16 pair, hi at [t], lo = bf16(c_t - hi) at [8 + t] (include/pdm.h pdm_gemm_args.ln_gcol)."""
    N, K = w.shape
    G = (K + 255) // 256
    if G > 8:
        raise ValueError(f"centred LayerNorm supports K <= 2048, got {K}")
    c = torch.zeros(N, 8, dtype=torch.float64, device=w.device)
    for t in range(G):
        c[:, t] = w[:, 256 * t: 256 * (t + 1)].double().sum(1)
    hi = c.float().bfloat16()
    lo = (c.float() - hi.float()).bfloat16()
    return torch.cat([hi, lo], 1).contiguous()


class NativeHandle:
    """Owns a pdm_uvit handle plus the packed device copies of the weights it points at."""

    def __init__(self, module, cfg):
        lib = _lib.load()
        h = ctypes.c_void_p()
        _lib.check(lib.pdm_uvit_create(ctypes.byref(cfg), ctypes.byref(h)), "pdm_uvit_create")
        self.h = h
        self.lib = lib
        self.cfg = cfg
        self.packed = {}
        self.ws = None
        self._mx = {}   # MXFP8 copies of the block Linears while packing (fp8 only)
        sd = module.state_dict()
        dev = next(iter(sd.values())).device
        n = lib.pdm_uvit_param_count(h)
        buf = ctypes.create_string_buffer(256)
        self.dtypes = {}
        for i in range(n):
            dt = ctypes.c_int()
            numel = ctypes.c_longlong()
            _lib.check(lib.pdm_uvit_param_info(h, i, buf, 256, ctypes.byref(dt), ctypes.byref(numel)))
            self.dtypes[buf.value.decode()] = (dt.value, numel.value)
        for name, (dt, numel) in self.dtypes.items():
            t = self._pack(sd, name, dt, numel, dev)
            self.packed[name] = t
            _lib.check(lib.pdm_uvit_set_param(h, name.encode(), ctypes.c_void_p(t.data_ptr()), dt, t.numel()),
                       "pdm_uvit_set_param")
        _lib.check(lib.pdm_uvit_validate(h), "pdm_uvit_validate")
        self._mx = {}

    def _ln_fold(self, sd, name, fp32=False):
        """norm1 -> attn.qkv and norm2 -> mlp.fc1 are fused (libs/uvit.py:115-120): LN(x) W^T + b =
        rstd * (x (W diag(g))^T - mean * colsum) + (W beta + b).  attn.qkv's q rows (the first embed_dim) also
        carry the softmax scale in base 2, Dh^-0.5 log2(e) (libs/uvit.py:64,73), so the attention kernels take
        exp2 of the scores directly (include/pdm.h).  Returns the packed tensor for the folded weight / its row
        sums / the folded bias, or None when `name` is not one of them."""
        for lin, norm in ((".attn.qkv", ".norm1"), (".mlp.fc1", ".norm2")):
            for part in (".weight", ".ln_colsum", ".ln_bias"):
                if not name.endswith(lin + part):
                    continue
                pre = name[: -len(lin + part)]
                w = sd[pre + lin + ".weight"].detach().float()
                g = sd[pre + norm + ".weight"].detach().float()
                rs = None
                if lin == ".attn.qkv":
                    D, H = int(self.cfg.embed_dim), int(self.cfg.num_heads)
                    rs = torch.ones(w.shape[0], dtype=torch.float64, device=w.device)
                    rs[:D] = (D // H) ** -0.5 * math.log2(math.e)
                    w = (w.double() * rs[:, None]).float()
                if part == ".weight" and fp32:
                    return w * g[None, :]
                wg = (w * g[None, :]).to(torch.bfloat16)
                if part == ".weight":
                    return wg
                if part == ".ln_colsum":
                    return wg.double().sum(1).float()
                b = (w.double() @ sd[pre + norm + ".bias"].detach().double())
                if pre + lin + ".bias" in sd:
                    lb = sd[pre + lin + ".bias"].detach().double()
                    b = b + (lb * rs if rs is not None else lb)
                return b.float()
        return None

    def _mx_weight(self, sd, key, dev):
        """MXFP8 copy of a block Linear weight [N, K] (norm-folded for attn.qkv / mlp.fc1): e4m3 bytes, E8M0 scale
        dwords [K/128, N] (the quantiser of the GPU epilogues, _lib.mx_quantize), the row sums of the DEQUANTISED
        weight (what the fused LayerNorm's mean * colsum must cancel) and their per-256-column-group split as the
        bf16 hi / lo table [N, 16] of the centred LayerNorm (include/pdm.h pdm_gemm_args.ln_gcol)."""
        if key not in self._mx:
            w = self._ln_fold(sd, key, fp32=True)
            if w is None:
                w = sd[key].detach().float()
            q, s = _lib.mx_quantize(w.to(dev))
            dq = _lib.mx_dequantize(q, s).double()
            lnc = key.endswith((".attn.qkv.weight", ".mlp.fc1.weight"))   # the LayerNorm consumers
            self._mx[key] = (q, s, dq.sum(1).float(), gcol_table(dq) if lnc else None)
        return self._mx[key]

    def _pack(self, sd, name, dtype, numel, dev):
        if self.cfg.fp8:
            t = None
            if dtype == _lib.PDM_FP8:
                t = self._mx_weight(sd, name, dev)[0].view(torch.uint8).reshape(-1)
            elif dtype == _lib.PDM_E8M0:
                t = self._mx_weight(sd, name[: -len("_scale")], dev)[1].reshape(-1)
            elif name.endswith(".ln_gcol"):
                t = self._mx_weight(sd, name[: -len(".ln_gcol")] + ".weight", dev)[3].reshape(-1)
            elif name.endswith(".ln_colsum") and self.dtypes[name[: -len(".ln_colsum")] + ".weight"][0] == _lib.PDM_FP8:
                t = self._mx_weight(sd, name[: -len(".ln_colsum")] + ".weight", dev)[2]
            if t is not None:
                if t.numel() != numel:
                    raise RuntimeError(f"parameter {name!r}: {t.numel()} elements, the HIP layout expects {numel}")
                return t.contiguous()
        folded = self._ln_fold(sd, name)
        if folded is not None:
            t = folded.to(device=dev, dtype=torch.bfloat16 if dtype == _lib.PDM_BF16 else torch.float32)
            t = t.contiguous().reshape(-1)
            if t.numel() != numel:
                raise RuntimeError(f"parameter {name!r}: {t.numel()} elements, the HIP layout expects {numel}")
            return t
        if name not in sd:
            raise RuntimeError(f"parameter {name!r} missing from the module state_dict")
        src = sd[name].detach()
        if name.startswith("zero_convs."):
            src = src.reshape(src.shape[0], -1)
        if name in ("decoder_pred.weight", "decoder_pred_mask.weight"):
            P, D = src.shape
            Ppad = (P + 15) // 16 * 16
            pad = torch.zeros(Ppad, D, dtype=src.dtype, device=src.device)
            pad[:P] = src
            src = pad
        t = src.to(device=dev, dtype=torch.bfloat16 if dtype == _lib.PDM_BF16 else torch.float32).contiguous()
        t = t.reshape(-1)
        if t.numel() != numel:
            raise RuntimeError(f"parameter {name!r}: {t.numel()} elements, the HIP layout expects {numel}")
        return t

    def workspace_bytes(self, rows):
        need = ctypes.c_size_t()
        _lib.check(self.lib.pdm_uvit_workspace_size(self.h, rows, ctypes.byref(need)), "pdm_uvit_workspace_size")
        return need.value

    def workspace(self, rows, device):
        need = ctypes.c_size_t()
        _lib.check(self.lib.pdm_uvit_workspace_size(self.h, rows, ctypes.byref(need)), "pdm_uvit_workspace_size")
        if self.ws is None or self.ws.numel() < need.value or self.ws.device != device:
            self.ws = torch.empty(need.value, dtype=torch.uint8, device=device)
        return self.ws

    def __del__(self):
        try:
            self.lib.pdm_uvit_destroy(self.h)
        except Exception:
            pass


class HipNet(nn.Module):
    """Base class: lazily (re)builds the native handle for the module's current parameters."""

    _t2i = False

    def __init__(self):
        super().__init__()
        self._native = None
        self._generation = 0
        self.residual = "bf16"

    def set_residual(self, dtype):
        """Precision of the residual stream x between the block Linears: 'bf16' (default: the reference's GPU
        run under autocast adds every Linear output to x in the autocast dtype) or 'fp32' (include/pdm.h
        pdm_uvit_cfg.residual_fp32).  Re-packs the handle."""
        if dtype not in ("bf16", "fp32"):
            raise ValueError(f"residual must be 'bf16' or 'fp32', got {dtype!r}")
        self.residual = dtype
        self.invalidate()
        return self

    def _native_cfg_kwargs(self):
        raise NotImplementedError

    def invalidate(self):
        """Drops the packed weights and workspace.  Every (re)build of the handle bumps `generation`, so a
        holder of device addresses taken from an older handle (a captured HIP graph, sampler.py) can tell
        that they are stale."""
        self._native = None

    @property
    def generation(self):
        """Identifies the current native handle (and so every device address it owns); -1 = none built."""
        return self._generation if self._native is not None else -1

    def _apply(self, fn, *args, **kwargs):
        self.invalidate()
        return super()._apply(fn, *args, **kwargs)

    def load_state_dict(self, state_dict, strict=True, *args, **kwargs):
        self.invalidate()
        return super().load_state_dict(state_dict, strict, *args, **kwargs)

    def native(self):
        if self._native is None:
            p = next(self.parameters())
            _lib.require_gpu(p)
            self._native = NativeHandle(self, cfg_struct(self._native_cfg_kwargs(), self._t2i))
            self._generation += 1
        return self._native
