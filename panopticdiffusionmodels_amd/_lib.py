"""ctypes binding of libpdm.so (include/pdm.h).

The product path has no fallback: if the HIP library is missing, cannot be loaded, or no GPU is
present, calls raise.  Status codes map to the exception types of the reference (ValueError for bad
arguments / unsupported shapes, RuntimeError otherwise).
"""
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libpdm.so")
# A/B timing of two builds in one box session (tools/ab_build.sh): PDM_LIB_PATH names another in-tree build;
# entry points that build lacks are left unbound instead of failing the load
_AB = os.environ.get("PDM_LIB_PATH")
if _AB:
    LIB_PATH = _AB if os.path.isabs(_AB) else os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), _AB)

PDM_F32, PDM_BF16, PDM_FP8, PDM_E8M0 = 0, 1, 2, 3
EPI_BF16, EPI_GELU, EPI_F32, EPI_RES = 0, 1, 2, 3


class PdmUvitCfg(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in (
        "img_size", "patch_size", "in_chans", "embed_dim", "depth", "num_heads", "mlp_hidden", "num_classes",
        "conv", "skip", "qkv_bias", "mlp_time_embed", "t2i", "clip_dim", "num_clip_token", "separate",
        "enable_panoptic", "num_panoptic_class", "fp8", "fp8_linears", "residual_fp32")]


class PdmDecoderCfg(ctypes.Structure):
    _fields_ = [("ch", ctypes.c_int), ("ch_mult", ctypes.c_int * 4), ("num_levels", ctypes.c_int),
                ("num_res_blocks", ctypes.c_int), ("z_channels", ctypes.c_int), ("out_ch", ctypes.c_int),
                ("latent_size", ctypes.c_int), ("scale_factor", ctypes.c_float)]


class PdmClipCfg(ctypes.Structure):
    _fields_ = [("vocab", ctypes.c_int), ("width", ctypes.c_int), ("layers", ctypes.c_int), ("heads", ctypes.c_int),
                ("mlp_hidden", ctypes.c_int), ("max_position", ctypes.c_int), ("eps", ctypes.c_float)]


class PdmStageEpilogueArgs(ctypes.Structure):
    _fields_ = [
        ("pre", ctypes.c_void_p), ("conv_w", ctypes.c_void_p), ("conv_b", ctypes.c_void_p),
        ("B", ctypes.c_int), ("C", ctypes.c_int), ("H", ctypes.c_int), ("W", ctypes.c_int),
        ("has_uncond", ctypes.c_int), ("cfg_scale", ctypes.c_float), ("act_tanh", ctypes.c_int),
        ("xin", ctypes.c_void_p), ("ax", ctypes.c_float), ("ae", ctypes.c_float),
        ("m_out", ctypes.c_void_p),
        ("n_terms", ctypes.c_int), ("T", ctypes.c_void_p * 6), ("c", ctypes.c_float * 6), ("cm", ctypes.c_float),
        ("x_out", ctypes.c_void_p), ("x_out2", ctypes.c_void_p), ("x_out3", ctypes.c_void_p),
    ]


class PdmGemmArgs(ctypes.Structure):
    _fields_ = [
        ("A1", ctypes.c_void_p), ("lda1", ctypes.c_int), ("A2", ctypes.c_void_p), ("lda2", ctypes.c_int),
        ("K1", ctypes.c_int), ("W", ctypes.c_void_p), ("ldw", ctypes.c_int), ("bias", ctypes.c_void_p),
        ("M", ctypes.c_int), ("N", ctypes.c_int), ("K", ctypes.c_int),
        ("out_bf16", ctypes.c_void_p), ("ldo", ctypes.c_int), ("out_f32", ctypes.c_void_p), ("ldr", ctypes.c_int),
        ("accumulate", ctypes.c_int), ("stats_out", ctypes.c_void_p), ("ln_stats", ctypes.c_void_p),
        ("ln_colsum", ctypes.c_void_p), ("ln_eps", ctypes.c_float), ("fp8", ctypes.c_int),
        ("a_scale", ctypes.c_void_p), ("a_scale_ld", ctypes.c_int), ("w_scale", ctypes.c_void_p),
        ("w_scale_ld", ctypes.c_int), ("out_fp8", ctypes.c_void_p), ("ldo8", ctypes.c_int),
        ("out_scale", ctypes.c_void_p), ("out_scale_ld", ctypes.c_int),
        ("mx_center", ctypes.c_int), ("ln_gcol", ctypes.c_void_p),
        ("res_in", ctypes.c_void_p), ("ldri", ctypes.c_int),
        ("res_f32", ctypes.c_void_p), ("ldrf", ctypes.c_int),
        ("a_rows_per_group", ctypes.c_int), ("a_group_stride", ctypes.c_int),
        ("out2", ctypes.c_void_p), ("out2_rows_per_group", ctypes.c_int), ("out2_group_stride", ctypes.c_int),
        ("stats_out2", ctypes.c_void_p),
    ]


_SIGS = {
    "pdm_gemm_args_size": (ctypes.c_int, []),
    "pdm_last_error": (ctypes.c_char_p, []),
    "pdm_version": (ctypes.c_int, []),
    "pdm_device_arch": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_int]),
    "pdm_set_gemm_algo": (ctypes.c_int, [ctypes.c_int]),
    "pdm_set_gemm_sk": (ctypes.c_int, [ctypes.c_int]),
    "pdm_gemm_sk_launches": (ctypes.c_longlong, []),
    "pdm_gemm_sk_stats": (ctypes.c_int, [ctypes.POINTER(ctypes.c_ulonglong)]),
    "pdm_gemm_seg_stats": (ctypes.c_int, [ctypes.POINTER(ctypes.c_ulonglong)]),
    "pdm_set_attention_algo": (ctypes.c_int, [ctypes.c_int]),
    "pdm_set_gemm_tuning": (ctypes.c_int, [ctypes.c_int, ctypes.c_int]),
    "pdm_uvit_create": (ctypes.c_int, [ctypes.POINTER(PdmUvitCfg), ctypes.POINTER(ctypes.c_void_p)]),
    "pdm_uvit_destroy": (ctypes.c_int, [ctypes.c_void_p]),
    "pdm_uvit_set_param": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_void_p, ctypes.c_int,
                                          ctypes.c_longlong]),
    "pdm_uvit_param_count": (ctypes.c_int, [ctypes.c_void_p]),
    "pdm_uvit_param_info": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_int,
                                           ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_longlong)]),
    "pdm_uvit_validate": (ctypes.c_int, [ctypes.c_void_p]),
    "pdm_uvit_workspace_size": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_size_t)]),
    "pdm_uvit_forward": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t,
                                        ctypes.c_void_p]),
    "pdm_uvit_t2i_forward": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                            ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                            ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]),
    "pdm_uvit_profile": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "pdm_uvit_profile_read": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_float),
                                             ctypes.POINTER(ctypes.c_double), ctypes.c_int,
                                             ctypes.POINTER(ctypes.c_int)]),
    "pdm_stage_epilogue": (ctypes.c_int, [ctypes.POINTER(PdmStageEpilogueArgs), ctypes.c_void_p]),
    "pdm_lincomb": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p),
                                   ctypes.POINTER(ctypes.c_float), ctypes.c_longlong, ctypes.c_void_p]),
    "pdm_gemm_bf16": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                     ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                     ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
                                     ctypes.c_int, ctypes.c_void_p]),
    "pdm_gemm": (ctypes.c_int, [ctypes.POINTER(PdmGemmArgs), ctypes.c_int, ctypes.c_void_p]),
    "pdm_gemm_pair": (ctypes.c_int, [ctypes.POINTER(PdmGemmArgs), ctypes.POINTER(PdmGemmArgs), ctypes.c_int,
                                     ctypes.c_void_p]),
    "pdm_gemm_bf16_ln": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                        ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_float, ctypes.c_void_p]),
    "pdm_rowstats": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                    ctypes.c_void_p, ctypes.c_void_p]),
    "pdm_gemm_conv3x3_bf16": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                             ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                             ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]),
    "pdm_gemm_batched_bf16": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_longlong, ctypes.c_void_p,
                                             ctypes.c_int, ctypes.c_longlong, ctypes.c_void_p, ctypes.c_int,
                                             ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                             ctypes.c_int, ctypes.c_longlong, ctypes.c_void_p, ctypes.c_int,
                                             ctypes.c_longlong, ctypes.c_int, ctypes.c_void_p]),
    "pdm_layernorm": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                     ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_float,
                                     ctypes.c_void_p]),
    "pdm_attention": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                     ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_float, ctypes.c_void_p]),
    "pdm_attention_log2": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                          ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]),
    "pdm_f32_to_bf16": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_longlong, ctypes.c_void_p]),
    "pdm_mx_quantize": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                       ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]),
    "pdm_images_to_u8": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                        ctypes.c_int, ctypes.c_void_p]),
    "pdm_mask_bits_to_rgb": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                            ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]),
    "pdm_clip_create": (ctypes.c_int, [ctypes.POINTER(PdmClipCfg), ctypes.POINTER(ctypes.c_void_p)]),
    "pdm_clip_destroy": (ctypes.c_int, [ctypes.c_void_p]),
    "pdm_clip_param_count": (ctypes.c_int, [ctypes.c_void_p]),
    "pdm_clip_param_info": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_int,
                                           ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_longlong)]),
    "pdm_clip_set_param": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_void_p, ctypes.c_int,
                                          ctypes.c_longlong]),
    "pdm_clip_workspace_size": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_size_t)]),
    "pdm_clip_encode": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                       ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]),
    "pdm_decoder_create": (ctypes.c_int, [ctypes.POINTER(PdmDecoderCfg), ctypes.POINTER(ctypes.c_void_p)]),
    "pdm_decoder_destroy": (ctypes.c_int, [ctypes.c_void_p]),
    "pdm_decoder_param_count": (ctypes.c_int, [ctypes.c_void_p]),
    "pdm_decoder_param_info": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_int,
                                              ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_longlong)]),
    "pdm_decoder_set_param": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_void_p, ctypes.c_int,
                                             ctypes.c_longlong]),
    "pdm_decoder_workspace_size": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_size_t)]),
    "pdm_decoder_decode": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                          ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]),
    "pdm_decoder_set_gn_fusion": (ctypes.c_int, [ctypes.c_int]),
    # training step (include/pdm.h "training")
    "pdm_train_create": (ctypes.c_int, [ctypes.POINTER(PdmUvitCfg), ctypes.POINTER(ctypes.c_void_p)]),
    "pdm_train_destroy": (ctypes.c_int, [ctypes.c_void_p]),
    "pdm_train_param_count": (ctypes.c_int, [ctypes.c_void_p]),
    "pdm_train_param_info": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_int,
                                            ctypes.POINTER(ctypes.c_longlong), ctypes.POINTER(ctypes.c_longlong)]),
    "pdm_train_sizes": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_longlong),
                                       ctypes.POINTER(ctypes.c_longlong)]),
    "pdm_train_set_buffers": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                             ctypes.c_void_p]),
    "pdm_train_refresh": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "pdm_train_workspace_size": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_size_t)]),
    "pdm_train_step": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                      ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_void_p,
                                      ctypes.c_size_t, ctypes.c_void_p]),
    "pdm_train_step_t2i": (ctypes.c_int, [ctypes.c_void_p] + [ctypes.c_void_p] * 8 + [ctypes.c_int, ctypes.c_float,
                                                                                      ctypes.c_void_p, ctypes.c_size_t,
                                                                                      ctypes.c_void_p]),
    "pdm_train_adamw": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                       ctypes.c_void_p, ctypes.c_float, ctypes.c_float, ctypes.c_float, ctypes.c_float, ctypes.c_float,
                                       ctypes.c_int, ctypes.c_float, ctypes.c_void_p]),
    "pdm_set_wgrad_tile": (ctypes.c_int, [ctypes.c_int]),
    "pdm_wgrad": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                 ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                 ctypes.c_size_t, ctypes.c_void_p]),
    "pdm_attention_backward": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                              ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]),
    "pdm_layernorm_backward": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                              ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                              ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                              ctypes.c_size_t, ctypes.c_void_p]),
}

EXPORTED_SYMBOLS = tuple(_SIGS)

_lib = None


def load():
    """Load libpdm.so (no GPU needed to load; every compute call needs one)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"libpdm.so not found at {LIB_PATH}: build it with `python -c 'import __graft_entry__ as g; "
                           f"g.build()'` (or `make -C panopticdiffusionmodels_amd/csrc`)")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in _SIGS.items():
        if _AB and not hasattr(lib, name):
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(status, what=""):
    if status != 0:
        msg = load().pdm_last_error().decode()
        if status == 1:
            raise ValueError(f"{what}: {msg}" if what else msg)
        raise RuntimeError(f"{what}: {msg}" if what else msg)


# Priority of the lane streams.  HIP keeps one pool of hardware queues per stream priority, each capped at
# GPU_MAX_HW_QUEUES (4 by default): a normal-priority lane stream shares a queue with the caller's stream or RCCL's
# once the process has made a few streams (torchrun / accelerate), and the lanes then run one after the other.
LANE_STREAM_PRIORITY = int(os.environ.get("PDM_LANE_PRIORITY", "-1"))
_LANE_STREAMS = {}


def lane_streams(device, n):
    """The process's n side streams on `device` (LANE_STREAM_PRIORITY), shared by every multi-lane user (the
    samplers' lanes, the decoder's lanes): each extra stream a process makes can take a hardware queue the sampling
    lanes need (two decoder streams of their own cost the L/2 bench 55-60 ms of sampling per step), so lanes reuse
    these few instead of making their own.  Users run one after the other from one host thread and order their lanes
    against the caller's stream on entry and exit."""
    dev = torch.device(device)
    key = dev.index if dev.index is not None else torch.cuda.current_device()
    pool = _LANE_STREAMS.setdefault(key, [])
    while len(pool) < n:
        pool.append(torch.cuda.Stream(device=dev, priority=LANE_STREAM_PRIORITY))
    return pool[:n]


def require_gpu(t=None):
    if not torch.cuda.is_available():
        raise RuntimeError("panopticdiffusionmodels_amd runs on an MI355X (gfx950) GPU; no GPU is visible "
                           "(there is no CPU fallback in the product path)")
    if t is not None and t.device.type != "cuda":
        raise RuntimeError(f"expected a tensor on the GPU, got device {t.device}")


def stream_ptr(device=None):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


# ---- thin op wrappers (used by tests and the generic solver path) ----------------------------------

def gemm(a, w, bias=None, epi=EPI_BF16, out=None, out_f32=None, accumulate=False, a2=None):
    """C = [a | a2] @ w.T (+ bias) with the selected epilogue.  a/a2/w bf16 2-D contiguous rows."""
    lib = load()
    require_gpu(a)
    M, K1 = a.shape
    K = K1 + (a2.shape[1] if a2 is not None else 0)
    N = w.shape[0]
    assert w.shape[1] == K
    if epi in (EPI_BF16, EPI_GELU) and out is None:
        out = torch.empty(M, N, dtype=torch.bfloat16, device=a.device)
    if epi == EPI_F32 and out_f32 is None:
        out_f32 = torch.zeros(M, N, dtype=torch.float32, device=a.device)
    check(lib.pdm_gemm_bf16(ptr(a), a.stride(0), ptr(a2), a2.stride(0) if a2 is not None else 0, K1, ptr(w),
                            ptr(bias), M, N, K, epi, ptr(out), out.stride(0) if out is not None else 0,
                            ptr(out_f32), out_f32.stride(0) if out_f32 is not None else 0, int(accumulate),
                            stream_ptr(a.device)), "pdm_gemm_bf16")
    return out_f32 if epi == EPI_F32 else out


def rowstats(x, want_bf16=True):
    """(bf16 copy, LayerNorm partials [rows, ceil(D/256), 2]) of fp32 rows x [rows, D]."""
    lib = load()
    require_gpu(x)
    rows, D = x.shape
    st = torch.empty(rows, (D + 255) // 256, 2, dtype=torch.float32, device=x.device)
    xb = torch.empty(rows, D, dtype=torch.bfloat16, device=x.device) if want_bf16 else None
    check(lib.pdm_rowstats(ptr(x), x.stride(0), rows, D, ptr(xb), ptr(st), stream_ptr(x.device)), "pdm_rowstats")
    return xb, st


def gemm_ln(a, w, bias, epi, ln_stats=None, ln_colsum=None, out=None, out_f32=None, accumulate=False,
            stats_out=False, eps=1e-5):
    """GEMM with the fused-LayerNorm operands (see include/pdm.h pdm_gemm_bf16_ln).  Returns the output, plus
    the produced partials when stats_out."""
    lib = load()
    require_gpu(a)
    M, K = a.shape
    N = w.shape[0]
    if epi in (EPI_BF16, EPI_GELU) and out is None:
        out = torch.empty(M, N, dtype=torch.bfloat16, device=a.device)
    if epi == EPI_F32 and out_f32 is None:
        out_f32 = torch.zeros(M, N, dtype=torch.float32, device=a.device)
    st = torch.empty(M, (N + 255) // 256, 2, dtype=torch.float32, device=a.device) if stats_out else None
    check(lib.pdm_gemm_bf16_ln(ptr(a), a.stride(0), ptr(w), ptr(bias), M, N, K, epi, ptr(out),
                               out.stride(0) if out is not None else 0, ptr(out_f32),
                               out_f32.stride(0) if out_f32 is not None else 0, int(accumulate), ptr(st),
                               ptr(ln_stats), ptr(ln_colsum), eps, stream_ptr(a.device)), "pdm_gemm_bf16_ln")
    res = out_f32 if epi == EPI_F32 else out
    return (res, st) if stats_out else res


# ---- MXFP8 (OCP e4m3 + E8M0 per 32 elements) host reference and GEMM wrapper --------------------------

def mx_quantize(x):
    """MXFP8 of x [R, K] (K % 32 == 0) exactly as the GPU epilogue quantises (csrc/pdm_common.h mx_quant8):
    E8M0 exponent e = ceil(log2(amax/448)) + 127 per 32 consecutive elements, e4m3 = RNE(x * 2^(127 - e)).
    Returns (q [R, K] float8_e4m3fn, scale dwords [K/128, R] int32: byte j of (kt, r) = block kt*4 + j)."""
    R, K = x.shape
    xb = x.float().reshape(R, K // 32, 32)
    amax = xb.abs().amax(-1)
    bits = (amax * (1.0 / 448.0)).view(torch.int32)
    e = ((bits >> 23) & 0xFF) + ((bits & 0x7FFFFF) != 0).to(torch.int32)
    e = e.clamp(max=254)
    inv = ((254 - e) << 23).view(torch.float32)
    q = (xb * inv[..., None]).reshape(R, K).to(torch.float8_e4m3fn)
    kt = (K + 127) // 128   # K % 128 != 0: the last scale dword is zero-padded
    e8 = torch.zeros(R, kt * 4, dtype=torch.uint8, device=x.device)
    e8[:, : K // 32] = e.to(torch.uint8)
    sc = e8.reshape(R, kt, 4).permute(1, 0, 2).contiguous().view(torch.int32).reshape(kt, R)
    return q, sc


def mx_dequantize(q, sc):
    R, K = q.shape
    e = sc.contiguous().view(torch.uint8).reshape(K // 128, R, 4).permute(1, 0, 2).reshape(R, K // 32).to(torch.int32)
    scale = torch.pow(2.0, (e - 127).double()).float()
    return (q.float().reshape(R, K // 32, 32) * scale[..., None]).reshape(R, K)


def mx_quantize_gpu(x):
    """MXFP8 of fp32 / bf16 rows x [R, K] on the GPU (pdm_mx_quantize): (q float8_e4m3fn [R, K], scale dwords
    int32 [ceil(K/128), R]), bit-identical to mx_quantize."""
    lib = load()
    require_gpu(x)
    R, K = x.shape
    q = torch.empty(R, K, dtype=torch.float8_e4m3fn, device=x.device)
    s = torch.zeros((K + 127) // 128, R, dtype=torch.int32, device=x.device)
    dt = PDM_F32 if x.dtype == torch.float32 else PDM_BF16
    check(lib.pdm_mx_quantize(ptr(x), dt, x.stride(0), R, K, ptr(q), q.stride(0), ptr(s), R, stream_ptr(x.device)),
          "pdm_mx_quantize")
    return q, s


def gemm_ex(epi, a, w, bias=None, *args, **kw):
    """pdm_gemm with every option (include/pdm.h pdm_gemm_args; positional after bias: a_scale, w_scale, out, ...).
    a / w are bf16, or float8_e4m3fn with their scale dword arrays (MXFP8); a2 (bf16) continues a along K (the
    split-K skip_linear operand)."""
    g = _gemm_args(a, w, bias, *args, **kw)
    check(load().pdm_gemm(ctypes.byref(g), epi, stream_ptr(a.device)), "pdm_gemm")


def gemm_pair(epi, first, second):
    """pdm_gemm_pair: two GEMMs of one epilogue / N / K given as gemm_ex keyword dicts (a, w, bias, ...), grouped
    into one persistent launch where the kernel takes both."""
    ga, gb = _gemm_args(**first), _gemm_args(**second)
    check(load().pdm_gemm_pair(ctypes.byref(ga), ctypes.byref(gb), epi, stream_ptr(first["a"].device)),
          "pdm_gemm_pair")


def _gemm_args(a, w, bias=None, a_scale=None, w_scale=None, out=None, out_f32=None, accumulate=False,
               ln_stats=None, ln_colsum=None, stats_out=None, out_fp8=None, out_scale=None, eps=1e-5,
               mx_center=False, ln_gcol=None, res_in=None, res_f32=None, a2=None, a_gather=None, out2=None,
               out2_gather=None, stats_out2=None):
    require_gpu(a)
    M, K = a.shape
    N = w.shape[0]
    g = PdmGemmArgs()
    g.A1, g.lda1 = a.data_ptr(), a.stride(0)
    g.K1 = K
    if a2 is not None:
        g.A2, g.lda2 = a2.data_ptr(), a2.stride(0)
        K = K + a2.shape[1]
    g.W, g.ldw = w.data_ptr(), w.stride(0)
    g.bias = bias.data_ptr() if bias is not None else None
    g.M, g.N, g.K = M, N, K
    if out is not None:
        g.out_bf16, g.ldo = out.data_ptr(), out.stride(0)
    if out_f32 is not None:
        g.out_f32, g.ldr = out_f32.data_ptr(), out_f32.stride(0)
    g.accumulate = int(accumulate)
    g.stats_out = stats_out.data_ptr() if stats_out is not None else None
    g.ln_stats = ln_stats.data_ptr() if ln_stats is not None else None
    g.ln_colsum = ln_colsum.data_ptr() if ln_colsum is not None else None
    g.ln_eps = eps
    if a.dtype == torch.float8_e4m3fn:
        g.fp8 = 1
        g.a_scale, g.a_scale_ld = a_scale.data_ptr(), a_scale.shape[1]
        g.w_scale, g.w_scale_ld = w_scale.data_ptr(), w_scale.shape[1]
    if out_fp8 is not None:
        g.out_fp8, g.ldo8 = out_fp8.data_ptr(), out_fp8.stride(0)
        g.out_scale, g.out_scale_ld = out_scale.data_ptr(), out_scale.shape[1]
    g.mx_center = int(mx_center)
    g.ln_gcol = ln_gcol.data_ptr() if ln_gcol is not None else None
    if res_in is not None:
        g.res_in, g.ldri = res_in.data_ptr(), res_in.stride(0)
    if res_f32 is not None:
        g.res_f32, g.ldrf = res_f32.data_ptr(), res_f32.stride(0)
    if a_gather is not None:   # (M, rows_per_group, group_stride): row m reads a[(m // rpg) * gs + m % rpg]
        g.M, g.a_rows_per_group, g.a_group_stride = a_gather
    if out2 is not None:       # out2_gather = (rows_per_group, group_stride) of the second residual output
        g.out2 = out2.data_ptr()
        g.out2_rows_per_group, g.out2_group_stride = out2_gather
        g.stats_out2 = stats_out2.data_ptr() if stats_out2 is not None else None
    return g


def mx_quantize_centred(x, stats):
    """The group-centred MXFP8 copy a producing epilogue writes (include/pdm.h pdm_gemm_args.mx_center): x [R, K]
    minus mu_t = stats[r, t, 0] / width_t per 256-column group (fp32, as the kernel divides), quantised with
    mx_quantize."""
    R, K = x.shape
    st = stats.reshape(R, -1, 2)
    xc = x.float().clone()
    for t in range((K + 255) // 256):
        w = min(256, K - 256 * t)
        xc[:, 256 * t: 256 * t + w] -= (st[:, t, 0] / float(w))[:, None]
    return mx_quantize(xc)


def gemm_conv3x3(x, w, bias=None, epi=EPI_F32, up=0, out=None, out_f32=None, accumulate=False):
    """Implicit-GEMM conv3x3 (pad 1) on NHWC bf16 x [B, h, w, Cin]; w [N, Cin, 3, 3] bf16 (torch layout, repacked
    here to the kernel's (ky, kx, ci) K order).  up=1 convolves the nearest-x2 upsample of x."""
    lib = load()
    require_gpu(x)
    B, h, wd, C = x.shape
    H, W = h << up, wd << up
    N = w.shape[0]
    wk = w.permute(0, 2, 3, 1).reshape(N, 9 * C).contiguous()
    if epi in (EPI_BF16, EPI_GELU) and out is None:
        out = torch.empty(B * H * W, N, dtype=torch.bfloat16, device=x.device)
    if epi == EPI_F32 and out_f32 is None:
        out_f32 = torch.zeros(B * H * W, N, dtype=torch.float32, device=x.device)
    check(lib.pdm_gemm_conv3x3_bf16(ptr(x), B, H, W, C, up, ptr(wk), ptr(bias), N, epi, ptr(out), ptr(out_f32),
                                    int(accumulate), stream_ptr(x.device)), "pdm_gemm_conv3x3_bf16")
    return out_f32 if epi == EPI_F32 else out


def gemm_batched(a, w, bias=None, epi=EPI_F32):
    """out[z] = a[z] @ w[z].T (+ bias) for a [Z, M, K], w [Z, N, K] bf16 contiguous."""
    lib = load()
    require_gpu(a)
    Z, M, K = a.shape
    N = w.shape[1]
    if epi == EPI_F32:
        ob, of = None, torch.zeros(Z, M, N, dtype=torch.float32, device=a.device)
    else:
        ob, of = torch.empty(Z, M, N, dtype=torch.bfloat16, device=a.device), None
    check(lib.pdm_gemm_batched_bf16(ptr(a), K, M * K, ptr(w), K, N * K, ptr(bias), M, N, K, Z, epi, ptr(ob), N, M * N,
                                    ptr(of), N, M * N, 0, stream_ptr(a.device)), "pdm_gemm_batched_bf16")
    return of if epi == EPI_F32 else ob


def layernorm(x, gamma, beta, eps=1e-5):
    lib = load()
    require_gpu(x)
    rows, D = x.shape
    y = torch.empty(rows, D, dtype=torch.bfloat16, device=x.device)
    check(lib.pdm_layernorm(ptr(x), x.stride(0), ptr(gamma), ptr(beta), ptr(y), y.stride(0), rows, D, eps,
                            stream_ptr(x.device)), "pdm_layernorm")
    return y


def attention(qkv, B, L, H, Dh, scale=None, q_log2=False):
    """q_log2: q already carries Dh^-0.5 * log2(e) (pdm_attention_log2, the U-ViT forward's layout)."""
    lib = load()
    require_gpu(qkv)
    out = torch.empty(B * L, H * Dh, dtype=torch.bfloat16, device=qkv.device)
    if q_log2:
        check(lib.pdm_attention_log2(ptr(qkv), qkv.stride(0), ptr(out), out.stride(0), B, L, H, Dh,
                                     stream_ptr(qkv.device)), "pdm_attention_log2")
        return out
    scale = Dh ** -0.5 if scale is None else scale
    check(lib.pdm_attention(ptr(qkv), qkv.stride(0), ptr(out), out.stride(0), B, L, H, Dh, scale,
                            stream_ptr(qkv.device)), "pdm_attention")
    return out


def lincomb(terms, coeffs, out=None):
    """out = sum_i coeffs[i] * terms[i] (fp32, same shape, contiguous)."""
    lib = load()
    t0 = terms[0]
    require_gpu(t0)
    n = len(terms)
    if n > 8:
        raise ValueError("lincomb supports at most 8 terms")
    if out is None:
        out = torch.empty_like(t0)
    arr = (ctypes.c_void_p * max(n, 1))(*[t.data_ptr() for t in terms])
    cs = (ctypes.c_float * max(n, 1))(*[float(c) for c in coeffs])
    check(lib.pdm_lincomb(ptr(out), n, arr, cs, t0.numel(), stream_ptr(t0.device)), "pdm_lincomb")
    return out


def stage_epilogue(pre, B, conv_w=None, conv_b=None, cfg_scale=None, act_tanh=False, xin=None, ax=0.0, ae=1.0,
                   m_out=None, terms=(), coeffs=(), cm=0.0, x_out=None, x_out2=None, x_out3=None):
    """See pdm_stage_epilogue in include/pdm.h.  pre [B or 2B, C, H, W] fp32 contiguous."""
    lib = load()
    require_gpu(pre)
    _, C, H, W = pre.shape
    a = PdmStageEpilogueArgs()
    a.pre = pre.data_ptr()
    a.conv_w = conv_w.data_ptr() if conv_w is not None else None
    a.conv_b = conv_b.data_ptr() if conv_b is not None else None
    a.B, a.C, a.H, a.W = B, C, H, W
    a.has_uncond = int(cfg_scale is not None)
    a.cfg_scale = float(cfg_scale or 0.0)
    a.act_tanh = int(act_tanh)
    a.xin = xin.data_ptr() if xin is not None else None
    a.ax, a.ae = float(ax), float(ae)
    a.m_out = m_out.data_ptr() if m_out is not None else None
    if len(terms) > 6:
        raise ValueError("stage_epilogue supports at most 6 terms")
    a.n_terms = len(terms)
    for i, (t, c) in enumerate(zip(terms, coeffs)):
        a.T[i] = t.data_ptr()
        a.c[i] = float(c)
    a.cm = float(cm)
    a.x_out = x_out.data_ptr() if x_out is not None else None
    a.x_out2 = x_out2.data_ptr() if x_out2 is not None else None
    a.x_out3 = x_out3.data_ptr() if x_out3 is not None else None
    check(lib.pdm_stage_epilogue(ctypes.byref(a), stream_ptr(pre.device)), "pdm_stage_epilogue")


def wgrad(dy, x, out=None, accumulate=False, scratch_mb=64):
    """Weight gradient dW = dy^T @ x (fp32 [N, K]) of bf16 rows dy [M, N], x [M, K] (pdm_wgrad)."""
    lib = load()
    require_gpu(dy)
    M, N = dy.shape
    K = x.shape[1]
    if out is None:
        out = torch.zeros(N, K, dtype=torch.float32, device=dy.device)
    scratch = torch.empty(scratch_mb << 18, dtype=torch.float32, device=dy.device) if scratch_mb else None
    check(lib.pdm_wgrad(ptr(dy), dy.stride(0), ptr(x), x.stride(0), ptr(out), out.stride(0), M, N, K, int(accumulate),
                        ptr(scratch), scratch.numel() * 4 if scratch is not None else 0, stream_ptr(dy.device)),
          "pdm_wgrad")
    return out


def attention_backward(qkv, o, dout, B, L, H, Dh=64):
    """d qkv (bf16 [B*L, 3*H*Dh]) of softmax attention (scale Dh^-0.5) from the forward's packed qkv, its output o
    and the output gradient dout (pdm_attention_backward)."""
    lib = load()
    require_gpu(qkv)
    dqkv = torch.empty_like(qkv)
    check(lib.pdm_attention_backward(ptr(qkv), ptr(o), ptr(dout), ptr(dqkv), B, L, H, Dh, stream_ptr(qkv.device)),
          "pdm_attention_backward")
    return dqkv


def layernorm_backward(x, dh, gamma, dx=None, accumulate=False):
    """(dx fp32, dx bf16, dgamma, dbeta) of nn.LayerNorm(D) over fp32 rows x with output gradient dh (fp32 / bf16)."""
    lib = load()
    require_gpu(x)
    rows, D = x.shape
    if dx is None:
        dx = torch.zeros(rows, D, dtype=torch.float32, device=x.device)
    dxb = torch.empty(rows, D, dtype=torch.bfloat16, device=x.device)
    dg = torch.empty(D, dtype=torch.float32, device=x.device)
    db = torch.empty(D, dtype=torch.float32, device=x.device)
    scratch = torch.empty((4 * ((rows + 3) // 4) + 8) * 2 * D, dtype=torch.float32, device=x.device)
    check(lib.pdm_layernorm_backward(ptr(x), ptr(dh), int(dh.dtype == torch.bfloat16), ptr(gamma), ptr(dx), ptr(dxb),
                                     ptr(dg), ptr(db), rows, D, int(accumulate), ptr(scratch), scratch.numel() * 4,
                                     stream_ptr(x.device)), "pdm_layernorm_backward")
    return dx, dxb, dg, db


class GemmProfiler:
    """HIP-event timing of every GEMM launch of a forward (pdm_uvit_profile)."""

    def __init__(self, native, max_launches=512):
        self.nat = native
        self.cap = max_launches

    def enable(self):
        check(self.nat.lib.pdm_uvit_profile(self.nat.h, self.cap), "pdm_uvit_profile")

    def disable(self):
        check(self.nat.lib.pdm_uvit_profile(self.nat.h, 0), "pdm_uvit_profile")

    def read(self):
        ms = (ctypes.c_float * self.cap)()
        fl = (ctypes.c_double * self.cap)()
        n = ctypes.c_int()
        check(self.nat.lib.pdm_uvit_profile_read(self.nat.h, ms, fl, self.cap, ctypes.byref(n)), "pdm_uvit_profile_read")
        k = min(n.value, self.cap)
        return [ms[i] for i in range(k)], [fl[i] for i in range(k)]
