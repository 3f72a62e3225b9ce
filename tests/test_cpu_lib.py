"""CPU-only checks of the native boundary: libpdm.so loads without a GPU and exports every symbol that
include/pdm.h declares; host-side helpers mirror the reference."""
import os
import re

import numpy as np
import pytest
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_symbols():
    src = open(os.path.join(REPO, "include", "pdm.h")).read()
    return sorted(set(re.findall(r"\b(pdm_[a-z0-9_]+)\s*\(", src)))


def test_lib_exports_header_symbols():
    from panopticdiffusionmodels_amd import _lib
    lib = _lib.load()
    for name in _declared_symbols():
        assert hasattr(lib, name), f"libpdm.so does not export {name}"
    assert set(_declared_symbols()) == set(_lib.EXPORTED_SYMBOLS)
    assert lib.pdm_version() >= 1


def test_gemm_args_layout_matches_binding():
    """The ctypes mirror of pdm_gemm_args has the size the library was compiled with (no field drift)."""
    import ctypes
    from panopticdiffusionmodels_amd import _lib
    assert _lib.load().pdm_gemm_args_size() == ctypes.sizeof(_lib.PdmGemmArgs)


def test_create_and_param_table_without_gpu():
    """Handle creation / parameter table / workspace sizing are pure host logic (no GPU call)."""
    import ctypes

    from panopticdiffusionmodels_amd import _lib, configs, native, weights
    lib = _lib.load()
    for name in ["imagenet256_uvit_large", "imagenet256_uvit_huge", "imagenet512_uvit_huge", "cifar10_uvit_small",
                 "mscoco_uvit_small", "tiny_uvit_cond", "tiny_t2i"]:
        kw = configs.nnet_kwargs(name)
        t2i = kw.pop("name") == "uvit_t2i"
        h = ctypes.c_void_p()
        _lib.check(lib.pdm_uvit_create(ctypes.byref(native.cfg_struct(kw, t2i)), ctypes.byref(h)))
        n = lib.pdm_uvit_param_count(h)
        spec = weights.uvit_t2i_spec(**kw) if t2i else weights.uvit_spec(**kw)
        shapes = {k: int(np.prod(s)) for k, s, _ in spec}
        buf = ctypes.create_string_buffer(256)
        for i in range(n):
            dt, ne = ctypes.c_int(), ctypes.c_longlong()
            _lib.check(lib.pdm_uvit_param_info(h, i, buf, 256, ctypes.byref(dt), ctypes.byref(ne)))
            key = buf.value.decode()
            if key.endswith((".ln_colsum", ".ln_bias")):   # fused-LayerNorm terms: one per output feature
                wkey = key.rsplit(".", 1)[0] + ".weight"
                assert ne.value == shapes[wkey] // shapes[key.split(".attn.")[0].split(".mlp.")[0] + ".norm1.weight"]
                continue
            assert key in shapes, key
            if key.startswith("decoder_pred"):
                assert ne.value >= shapes[key]
            else:
                assert ne.value == shapes[key], key
        ws = ctypes.c_size_t()
        _lib.check(lib.pdm_uvit_workspace_size(h, 100, ctypes.byref(ws)))
        assert ws.value > 0
        # forward without registered weights must fail with a state error (no GPU call happens)
        if not t2i:
            yp = ctypes.c_void_p(16) if kw.get("num_classes", -1) > 0 else None
            st = lib.pdm_uvit_forward(h, ctypes.c_void_p(16), ctypes.c_void_p(16), yp, ctypes.c_void_p(16), 1,
                                      ctypes.c_void_p(16), 1 << 40, None)
            assert st == 3 and b"not registered" in lib.pdm_last_error()
        lib.pdm_uvit_destroy(h)


def test_create_rejects_unsupported():
    import ctypes

    from panopticdiffusionmodels_amd import _lib, configs, native
    lib = _lib.load()
    kw = configs.nnet_kwargs("imagenet256_uvit_large")
    kw.pop("name")
    kw["mlp_time_embed"] = True
    h = ctypes.c_void_p()
    with pytest.raises(ValueError):
        _lib.check(lib.pdm_uvit_create(ctypes.byref(native.cfg_struct(kw, False)), ctypes.byref(h)))


def test_product_refuses_cpu():
    from panopticdiffusionmodels_amd.utils import get_nnet
    from panopticdiffusionmodels_amd import configs
    net = get_nnet(**configs.nnet_kwargs("tiny_uvit_cond"))
    x = torch.zeros(1, 4, 16, 16)
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(RuntimeError):
        net(x, torch.ones(1), torch.zeros(1, dtype=torch.long))


def test_state_dict_keys_match_reference_spec():
    from panopticdiffusionmodels_amd import configs, weights
    from panopticdiffusionmodels_amd.utils import get_nnet
    for name in ["tiny_uvit_cond", "tiny_uvit_h", "tiny_uvit_uncond", "cifar10_uvit_small"]:
        kw = configs.nnet_kwargs(name)
        net = get_nnet(**kw)
        sd = weights.nnet_state_dict(kw, seed=0)
        assert list(net.state_dict().keys()) == list(sd.keys()) or set(net.state_dict()) == set(sd)
        net.load_state_dict(sd)


def test_int2bits_roundtrip(golden):
    from panopticdiffusionmodels_amd import utils
    ids = torch.from_numpy(golden["utils/ids"])
    bits = utils.int2bits(ids, out_dtype=torch.float)
    np.testing.assert_array_equal(bits.numpy(), golden["utils/bits"])
    back = utils.bits2int(bits > 0)
    np.testing.assert_array_equal(back.numpy(), golden["utils/bits2int"])
    assert utils.amortize(103, 25) == [25, 25, 25, 25, 3]


def test_fp8_param_table_without_gpu():
    """MXFP8 handle (BASELINE configs[4]): every block Linear is an e4m3 [N][K] byte weight with an E8M0
    [K/128][N] scale companion; the rest of the table is the bf16 one; t2i and non-128 widths are rejected."""
    import ctypes

    from panopticdiffusionmodels_amd import _lib, configs, native
    lib = _lib.load()
    kw = configs.nnet_kwargs("imagenet512_uvit_huge")
    kw.pop("name")
    kw["fp8"] = True
    h = ctypes.c_void_p()
    _lib.check(lib.pdm_uvit_create(ctypes.byref(native.cfg_struct(kw, False)), ctypes.byref(h)))
    table = {}
    buf = ctypes.create_string_buffer(256)
    for i in range(lib.pdm_uvit_param_count(h)):
        dt, ne = ctypes.c_int(), ctypes.c_longlong()
        _lib.check(lib.pdm_uvit_param_info(h, i, buf, 256, ctypes.byref(dt), ctypes.byref(ne)))
        table[buf.value.decode()] = (dt.value, ne.value)
    D, Hd = 1152, 4608
    for key, (N, K) in {"out_blocks.3.attn.qkv.weight": (3 * D, D), "mid_block.attn.proj.weight": (D, D),
                        "in_blocks.0.mlp.fc1.weight": (Hd, D), "in_blocks.13.mlp.fc2.weight": (D, Hd)}.items():
        assert table[key] == (_lib.PDM_FP8, N * K), key
        assert table[key + "_scale"] == (_lib.PDM_E8M0, K // 128 * N), key
    assert table["decoder_pred.weight"][0] == _lib.PDM_BF16
    assert table["out_blocks.0.skip_linear.weight"] == (_lib.PDM_BF16, 2 * D * D)
    ws8, ws16 = ctypes.c_size_t(), ctypes.c_size_t()
    _lib.check(lib.pdm_uvit_workspace_size(h, 100, ctypes.byref(ws8)))
    lib.pdm_uvit_destroy(h)
    kw["fp8"] = False
    _lib.check(lib.pdm_uvit_create(ctypes.byref(native.cfg_struct(kw, False)), ctypes.byref(h)))
    _lib.check(lib.pdm_uvit_workspace_size(h, 100, ctypes.byref(ws16)))
    lib.pdm_uvit_destroy(h)
    assert 0 < ws8.value < ws16.value   # MXFP8 operands replace the bf16 copies
    for name, t2i in (("tiny_uvit_h", False), ("tiny_t2i", True)):   # D = 576; t2i
        k2 = configs.nnet_kwargs(name)
        k2.pop("name")
        k2["fp8"] = True
        with pytest.raises(ValueError):
            _lib.check(lib.pdm_uvit_create(ctypes.byref(native.cfg_struct(k2, t2i)), ctypes.byref(h)))


def test_no_inflight_load_register_touched_before_its_wait():
    """in the SHIPPED code object (libpdm.so's gfx950 bundles, disassembled), no instruction on any
    control-flow path from a vector-memory load to its first vmcnt wait reads or writes the load's destination VGPRs
    -- the guard for the attention kernels' inline-asm Q loads, whose waits hipcc does not know about
    (tools/check_asm_loads.py; attention.hip PDM_WAIT_Q)."""
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    lib = os.path.join(repo, "panopticdiffusionmodels_amd", "libpdm.so")
    if not os.path.exists("/opt/rocm/lib/llvm/bin/llvm-objdump") or not os.path.exists(lib):
        pytest.skip("llvm-objdump or libpdm.so missing")
    r = subprocess.run([sys.executable, os.path.join(repo, "tools", "check_asm_loads.py"), lib],
                       capture_output=True, text=True, timeout=300)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    m = re.search(r"checked (\d+) VGPR-destination VMEM loads in (\d+) kernels \((\d+) plain", r.stdout)
    assert m and int(m.group(1)) > 1000 and int(m.group(3)) > 0   # the walk saw the attention kernels' asm loads
