"""KL-f8 latent decoder — API of libs/autoencoder.py (`get_model(...).decode(z)`, 446-450, 471-484).

Decode-only: the sampling path never encodes.  `FrozenAutoencoderKL` keeps the
reference's state_dict keys for `post_quant_conv.*` and `decoder.*` (the encoder keys of a reference
checkpoint are accepted and ignored), so `get_model(path)` loads the reference's
assets/stable-diffusion/autoencoder_kl*.pth with `torch.load(..., weights_only=True)`.

`decode` runs the hand-written HIP decoder of libpdm (csrc/decoder.hip, `pdm_decoder_*` in include/pdm.h):
NHWC activations, fp32 residual stream, every 3x3 conv an implicit GEMM on the bf16 MFMA GEMM kernels with
GroupNorm+swish fused into the producer of its bf16 input.  On first use the fp32 parameters are repacked
once (3x3 convs -> bf16 [Cout][ky][kx][Cin]; q/k/v -> one [3C, C] matrix; conv_out padded to 4 rows).
Large batches are decoded in chunks of at most `chunk` latents (the reference decodes in chunks of 50,
decode_large_batch in eval_ldm_discrete.py:62-68) so the workspace stays bounded.  The chunks are balanced (50 ->
25 + 25, not 32 + 18) and alternate over `lanes` streams -- the caller's and the process's shared lane streams
(_lib.lane_streams, the sampler's) -- with a workspace each, so two chunks decode at once and one's small
low-resolution launches fill the CUs the other leaves idle (B = 50: 47.3 -> 45.1 ms at 256^2, 183.0 -> 179.8 ms at
512^2; B = 32, split 16 + 16: 29.1 -> 28.3 ms, 116.4 -> 113.6 ms; bit-identical; tools/decode_lanes.py).
"""
import ctypes

import torch
import torch.nn as nn

from .. import _lib
from .. import weights as W

DDCONFIG = dict(W.DECODER_DDCONFIG)


class _DecoderHandle:
    """pdm_decoder handle + packed device copies of the weights it points at."""

    def __init__(self, module, device):
        lib = _lib.load()
        cfg = _lib.PdmDecoderCfg()
        cfg.ch = module.ch
        for i, m in enumerate(module.ch_mult):
            cfg.ch_mult[i] = m
        cfg.num_levels = len(module.ch_mult)
        cfg.num_res_blocks = module.num_res_blocks
        cfg.z_channels = module.z_channels
        cfg.out_ch = module.out_ch
        cfg.latent_size = module.latent_size
        cfg.scale_factor = module.scale_factor
        h = ctypes.c_void_p()
        _lib.check(lib.pdm_decoder_create(ctypes.byref(cfg), ctypes.byref(h)), "pdm_decoder_create")
        self.lib, self.h, self.device = lib, h, device
        self.packed = {}
        self.ws = {}         # lane -> workspace tensor
        self.ws_batch = {}
        buf = ctypes.create_string_buffer(256)
        for i in range(lib.pdm_decoder_param_count(h)):
            dt, numel = ctypes.c_int(), ctypes.c_longlong()
            _lib.check(lib.pdm_decoder_param_info(h, i, buf, 256, ctypes.byref(dt), ctypes.byref(numel)))
            name = buf.value.decode()
            t = self._pack(module, name, dt.value).to(device).contiguous()
            if t.numel() != numel.value:
                raise RuntimeError(f"decoder weight {name}: packed {t.numel()} elements, expected {numel.value}")
            self.packed[name] = t
            _lib.check(lib.pdm_decoder_set_param(h, name.encode(), _lib.ptr(t), dt.value, t.numel()),
                       "pdm_decoder_set_param")

    @staticmethod
    def _pack(m, name, dtype):
        if name.endswith("mid.attn_1.qkv.weight"):
            p = name[: -len("qkv.weight")]
            w = torch.cat([m._p(p + f"{n}.weight") for n in "qkv"]).reshape(-1, m._p(p + "q.weight").shape[1])
            return w.to(torch.bfloat16)
        if name.endswith("mid.attn_1.qkv.bias"):
            p = name[: -len("qkv.bias")]
            return torch.cat([m._p(p + f"{n}.bias") for n in "qkv"]).float()
        src = m._p(name).detach().float()
        if name == "decoder.conv_out.weight":   # [out_ch, C, 3, 3] -> [4][ky][kx][C], zero rows
            w = torch.zeros(4, *src.shape[1:], dtype=src.dtype, device=src.device)
            w[: src.shape[0]] = src
            return w.permute(0, 2, 3, 1).reshape(4, -1).to(torch.bfloat16)
        if name == "decoder.conv_out.bias":
            b = torch.zeros(4, dtype=src.dtype, device=src.device)
            b[: src.shape[0]] = src
            return b
        if dtype == _lib.PDM_BF16:
            if src.dim() == 4 and src.shape[-1] == 3:   # 3x3 conv -> [Cout][ky][kx][Cin]
                return src.permute(0, 2, 3, 1).reshape(src.shape[0], -1).to(torch.bfloat16)
            return src.reshape(src.shape[0], -1).to(torch.bfloat16)   # 1x1 conv
        return src.reshape(-1)

    def workspace(self, batch, lane=0):
        if self.ws.get(lane) is None or self.ws_batch[lane] < batch:
            nbytes = ctypes.c_size_t()
            _lib.check(self.lib.pdm_decoder_workspace_size(self.h, batch, ctypes.byref(nbytes)),
                       "pdm_decoder_workspace_size")
            self.ws[lane] = None
            self.ws[lane] = torch.empty(nbytes.value, dtype=torch.uint8, device=self.device)
            self.ws_batch[lane] = batch
        return self.ws[lane]

    def decode_into(self, z, img, n, lane, stream):
        ws = self.workspace(n, lane)
        _lib.check(self.lib.pdm_decoder_decode(self.h, _lib.ptr(z), _lib.ptr(img), n, _lib.ptr(ws), ws.numel(),
                                               stream), "pdm_decoder_decode")

    def __del__(self):
        try:
            self.lib.pdm_decoder_destroy(self.h)
        except Exception:
            pass


class FrozenAutoencoderKL(nn.Module):
    def __init__(self, ddconfig=None, embed_dim=4, pretrained_path=None, scale_factor=0.18215, seed=0,
                 dtype=torch.bfloat16, state_dict=None, latent_size=32, chunk=32, lanes=2):
        super().__init__()
        dd = dict(DDCONFIG if ddconfig is None else ddconfig)
        self.ch = int(dd["ch"])
        self.ch_mult = tuple(dd["ch_mult"])
        self.num_res_blocks = int(dd["num_res_blocks"])
        self.z_channels = int(dd["z_channels"])
        self.out_ch = int(dd["out_ch"])
        self.scale_factor = float(scale_factor)
        self.embed_dim = embed_dim
        self.compute_dtype = dtype
        self.latent_size = int(latent_size)
        self.chunk = int(chunk)
        self.lanes = max(1, int(lanes))
        spec = W.decoder_spec(ch=self.ch, out_ch=self.out_ch, ch_mult=self.ch_mult,
                              num_res_blocks=self.num_res_blocks, z_channels=self.z_channels, embed_dim=embed_dim)
        if state_dict is not None or pretrained_path is not None:
            full = state_dict if state_dict is not None else torch.load(pretrained_path, map_location="cpu",
                                                                        weights_only=True)
            sd = {k: v for k, v in full.items() if k.startswith("decoder.") or k.startswith("post_quant_conv.")}
            missing = [k for k, _, _ in spec if k not in sd]
            if missing:
                raise RuntimeError(f"autoencoder checkpoint is missing {len(missing)} decoder keys, e.g. {missing[:3]}")
        else:
            sd = W.make_state_dict(spec, seed=seed, init="reference")
        self._names = [k for k, _, _ in spec]
        for k in self._names:
            self.register_buffer(k.replace(".", "__"), sd[k].float().clone())
        self.requires_grad_(False)
        self.eval()
        self._native = None

    def _p(self, name):
        return getattr(self, name.replace(".", "__"))

    def _apply(self, fn, *a, **kw):
        self._native = None
        return super()._apply(fn, *a, **kw)

    def _load_from_state_dict(self, *a, **kw):
        self._native = None
        return super()._load_from_state_dict(*a, **kw)

    def native(self, device):
        if self._native is None or self._native.device != device:
            self._native = _DecoderHandle(self, device)
        return self._native

    @torch.no_grad()
    def decode(self, z):
        """libs/autoencoder.py:446-450 (z / scale_factor -> post_quant_conv -> Decoder.forward 376-409)."""
        _lib.require_gpu(z)
        B, C, h, w = z.shape
        if C != self.z_channels or h != self.latent_size or w != self.latent_size:
            if h == w and C == self.z_channels:   # another latent size: a handle per size
                self.latent_size = h
                self._native = None
            else:
                raise ValueError(f"decode: expected z [B, {self.z_channels}, s, s], got {tuple(z.shape)}")
        nat = self.native(z.device)
        z = z.float().contiguous()
        up = 2 ** (len(self.ch_mult) - 1)
        img = torch.empty(B, self.out_ch, h * up, w * up, dtype=torch.float32, device=z.device)
        # at least one chunk per lane once each gets >= 8 latents (B = 32: 16 + 16 concurrently, 29.1 -> 28.3 ms at 256^2)
        nch = max(-(-B // self.chunk), min(self.lanes, B // 8))
        sizes = [B // nch + (1 if i < B % nch else 0) for i in range(nch)]   # balanced chunks of <= chunk
        starts = [sum(sizes[:i]) for i in range(nch)]
        lanes = min(self.lanes, nch)
        if lanes == 1:
            stream = _lib.stream_ptr(z.device)
            for s0, n in zip(starts, sizes):
                nat.decode_into(z[s0:s0 + n], img[s0:s0 + n], n, 0, stream)
            return img
        # chunk i on lane i % lanes: lane 0 the caller's stream, lanes 1.. the process's shared side streams (the
        # sampler's lane streams, _lib.lane_streams: no new hardware queue); the side lanes start behind everything
        # queued on the caller's stream and the caller's stream waits for them at the end
        main = torch.cuda.current_stream(z.device)
        streams = [main] + _lib.lane_streams(z.device, lanes - 1)
        for st in streams[1:]:
            st.wait_stream(main)
        for i, (s0, n) in enumerate(zip(starts, sizes)):
            lane = i % lanes
            nat.decode_into(z[s0:s0 + n], img[s0:s0 + n], n, lane, ctypes.c_void_p(streams[lane].cuda_stream))
        for st in streams[1:]:
            main.wait_stream(st)
        return img

    def forward(self, inputs, fn):
        if fn == "decode":
            return self.decode(inputs)
        raise NotImplementedError(f"{fn}: only decode is on the sampling path")


def get_model(pretrained_path=None, scale_factor=0.18215, **kw):
    """libs/autoencoder.py:471-484 (pretrained_path=None -> synthetic seeded weights)."""
    return FrozenAutoencoderKL(DDCONFIG, 4, pretrained_path, scale_factor, **kw)
