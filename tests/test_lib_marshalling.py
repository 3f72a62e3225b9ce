"""CPU checks of the ctypes binding's argument marshalling (panopticdiffusionmodels_amd/_lib.py), so that a signature
change breaks the CPU suite instead of a GPU run (round 4: a gemm_ex signature change failed 20 fp8 GPU tests).

1. every prototype in include/pdm.h has the parameter count of its _SIGS entry, and every _SIGS entry is declared;
2. every call of a C entry point (`<x>.pdm_NAME(...)`) anywhere in the package, tests, tools and bench.py passes as
   many positional arguments as _SIGS declares;
3. every call of a _lib wrapper through `lib.` / `_lib.` binds to the wrapper's Python signature;
4. the wrappers run end to end against a recording fake of the library (CPU tensors, no GPU): every argument
   converts to its declared ctypes type and the argument counts match."""
import ast
import ctypes
import inspect
import os
import re

import pytest
import torch

from panopticdiffusionmodels_amd import _lib

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _py_files():
    roots = [os.path.join(REPO, d) for d in ("panopticdiffusionmodels_amd", "tests", "tools")]
    files = [os.path.join(REPO, f) for f in ("bench.py", "__graft_entry__.py")]
    for r in roots:
        for dp, _, fs in os.walk(r):
            files += [os.path.join(dp, f) for f in fs if f.endswith(".py")]
    return files


def _header_prototypes():
    src = open(os.path.join(REPO, "include", "pdm.h")).read()
    src = re.sub(r"/\*.*?\*/", " ", src, flags=re.S)
    src = re.sub(r"//[^\n]*", " ", src)
    protos = {}
    for m in re.finditer(r"\b(pdm_\w+)\s*\(([^;{]*?)\)\s*;", src):
        params = m.group(2).strip()
        n = 0 if params in ("", "void") else params.count(",") + 1
        protos[m.group(1)] = n
    return protos


def test_header_matches_sigs():
    protos = _header_prototypes()
    for name, (_, args) in _lib._SIGS.items():
        assert name in protos, f"{name} bound in _lib but not declared in include/pdm.h"
        assert protos[name] == len(args), f"{name}: pdm.h has {protos[name]} parameters, _SIGS {len(args)}"


def test_c_entry_call_sites_match_sigs():
    bad = []
    for f in _py_files():
        tree = ast.parse(open(f).read(), f)
        for node in ast.walk(tree):
            if not (isinstance(node, ast.Call) and isinstance(node.func, ast.Attribute)):
                continue
            name = node.func.attr
            if not name.startswith("pdm_") or name not in _lib._SIGS:
                continue
            if any(isinstance(a, ast.Starred) for a in node.args) or node.keywords:
                continue
            want = len(_lib._SIGS[name][1])
            if len(node.args) != want:
                bad.append(f"{os.path.relpath(f, REPO)}:{node.lineno} {name}: {len(node.args)} args, expects {want}")
    assert not bad, "\n".join(bad)


WRAPPERS = {n: getattr(_lib, n) for n in ("gemm", "rowstats", "gemm_ln", "mx_quantize_gpu", "gemm_ex", "gemm_pair",
                                          "gemm_conv3x3", "gemm_batched", "layernorm", "attention", "lincomb",
                                          "stage_epilogue", "wgrad", "attention_backward", "layernorm_backward",
                                          "mx_quantize", "mx_dequantize", "mx_quantize_centred", "_gemm_args")}


def test_wrapper_call_sites_bind():
    bad = []
    for f in _py_files():
        tree = ast.parse(open(f).read(), f)
        for node in ast.walk(tree):
            if not (isinstance(node, ast.Call) and isinstance(node.func, ast.Attribute)):
                continue
            recv = node.func.value
            if not (isinstance(recv, ast.Name) and recv.id in ("lib", "_lib")) or node.func.attr not in WRAPPERS:
                continue
            if any(isinstance(a, ast.Starred) for a in node.args) or any(k.arg is None for k in node.keywords):
                continue
            sig = inspect.signature(WRAPPERS[node.func.attr])
            try:
                sig.bind(*[None] * len(node.args), **{k.arg: None for k in node.keywords})
            except TypeError as e:
                bad.append(f"{os.path.relpath(f, REPO)}:{node.lineno} {node.func.attr}: {e}")
    assert not bad, "\n".join(bad)


class _FakeFn:
    def __init__(self, name, calls):
        self.name, self.calls = name, calls
        self.argtypes, self.restype = None, None

    def __call__(self, *args):
        assert self.argtypes is not None, f"{self.name} called before its argtypes were bound"
        assert len(args) == len(self.argtypes), f"{self.name}: {len(args)} args, argtypes {len(self.argtypes)}"
        for i, (t, a) in enumerate(zip(self.argtypes, args)):
            try:
                t.from_param(a)
            except Exception as e:   # noqa: BLE001
                raise AssertionError(f"{self.name} arg {i}: {a!r} does not convert to {t}: {e}")
        self.calls.append(self.name)
        return b"" if self.restype is ctypes.c_char_p else 0


class _FakeLib:
    def __init__(self):
        self.calls = []
        self._fns = {}

    def __getattr__(self, name):
        if name.startswith("_") or name == "calls":
            raise AttributeError(name)
        if name not in self._fns:
            self._fns[name] = _FakeFn(name, self.calls)
        return self._fns[name]


@pytest.fixture()
def fake(monkeypatch):
    fl = _FakeLib()
    monkeypatch.setattr(_lib, "_lib", None)
    monkeypatch.setattr(_lib.os.path, "exists", lambda p: True)
    monkeypatch.setattr(_lib.ctypes, "CDLL", lambda path: fl)
    monkeypatch.setattr(_lib, "require_gpu", lambda t=None: None)
    monkeypatch.setattr(_lib, "stream_ptr", lambda device=None: ctypes.c_void_p(0))
    assert _lib.load() is fl
    yield fl
    _lib._lib = None


def test_wrappers_marshal_against_fake_library(fake):
    bf = torch.bfloat16
    a = torch.randn(64, 128).to(bf)
    w = torch.randn(32, 128).to(bf)
    bias = torch.randn(32)
    _lib.gemm(a, w, bias)
    _lib.gemm(a[:, :64], w, bias, _lib.EPI_F32, a2=a[:, 64:])
    _lib.rowstats(torch.randn(64, 128))
    st = torch.zeros(64, 1, 2)
    _lib.gemm_ln(a, w, bias, _lib.EPI_BF16, ln_stats=st, ln_colsum=torch.zeros(32), stats_out=True)
    q, s = _lib.mx_quantize(torch.randn(64, 128))
    wq, ws = _lib.mx_quantize(torch.randn(32, 128))
    _lib.mx_quantize_gpu(torch.randn(64, 128))
    out = torch.empty(64, 32, dtype=bf)
    _lib.gemm_ex(_lib.EPI_BF16, a, w, bias, out=out)
    _lib.gemm_ex(_lib.EPI_BF16, q, wq, bias, s, ws, out)            # MXFP8 operands, scales positional
    _lib.gemm_ex(_lib.EPI_RES, a, w, bias, out=out, res_in=out, accumulate=True, stats_out=st)
    _lib.gemm_ex(_lib.EPI_F32, a[:, :64], w, bias, out_f32=torch.zeros(64, 32), a2=a[:, 64:])
    _lib.gemm_pair(_lib.EPI_BF16, dict(a=a, w=w, bias=bias, out=out), dict(a=a, w=w, bias=bias, out=out.clone()))
    _lib.gemm_conv3x3(torch.randn(1, 4, 4, 16).to(bf), torch.randn(8, 16, 3, 3).to(bf), torch.randn(8))
    _lib.gemm_batched(torch.randn(2, 16, 32).to(bf), torch.randn(2, 8, 32).to(bf))
    _lib.layernorm(torch.randn(16, 64), torch.ones(64), torch.zeros(64))
    qkv = torch.randn(2 * 17, 3 * 64).to(bf)
    _lib.attention(qkv, 2, 17, 1, 64)
    _lib.attention(qkv, 2, 17, 1, 64, q_log2=True)
    _lib.lincomb([torch.randn(8), torch.randn(8)], [1.0, 0.5])
    pre = torch.randn(4, 4, 8, 8)
    _lib.stage_epilogue(pre, 2, conv_w=torch.randn(4, 4, 3, 3), conv_b=torch.randn(4), cfg_scale=0.4,
                        xin=torch.randn(2, 4, 8, 8), terms=(torch.randn(2, 4, 8, 8),), coeffs=(1.0,),
                        x_out=torch.empty(2, 4, 8, 8))
    _lib.wgrad(torch.randn(16, 8).to(bf), torch.randn(16, 4).to(bf), scratch_mb=1)
    _lib.attention_backward(qkv, torch.randn(34, 64).to(bf), torch.randn(34, 64).to(bf), 2, 17, 1)
    _lib.layernorm_backward(torch.randn(16, 64), torch.randn(16, 64), torch.ones(64))

    class _Native:
        lib, h = fake, ctypes.c_void_p(1)
    p = _lib.GemmProfiler(_Native(), max_launches=4)
    p.enable()
    p.read()
    p.disable()
    for name in ("pdm_gemm_bf16", "pdm_rowstats", "pdm_gemm_bf16_ln", "pdm_mx_quantize", "pdm_gemm", "pdm_gemm_pair",
                 "pdm_gemm_conv3x3_bf16", "pdm_gemm_batched_bf16", "pdm_layernorm", "pdm_attention",
                 "pdm_attention_log2", "pdm_lincomb", "pdm_stage_epilogue", "pdm_wgrad", "pdm_attention_backward",
                 "pdm_layernorm_backward", "pdm_uvit_profile", "pdm_uvit_profile_read"):
        assert name in fake.calls, name


def test_gemm_args_struct_matches_library():
    """sizeof(pdm_gemm_args) of the built library equals the ctypes mirror (the library loads without a GPU)."""
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libpdm.so not built")
    lib = ctypes.CDLL(_lib.LIB_PATH)
    lib.pdm_gemm_args_size.restype = ctypes.c_int
    assert lib.pdm_gemm_args_size() == ctypes.sizeof(_lib.PdmGemmArgs)
