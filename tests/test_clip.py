"""t2i conditioning producer: libs/clip.py FrozenCLIPEmbedder on the HIP CLIP encoder.

CPU: the oracle (oracle/clip_ref.py) against transformers' CLIPTextModel outputs (tests/golden/clip_golden.npz,
made by tests/golden/make_clip_golden.py), state_dict keys, the C-ABI parameter table.
GPU: pdm_clip_encode against the golden outputs (tiny configs, head dim 32 / 64) and against the oracle at the
ViT-L/14 text shape (12 x 768, 77 tokens).  Tolerance: bf16 GEMM operands, rel-L2 <= 2e-2 (as the U-ViT
forward).
"""
import ctypes
import os

import numpy as np
import pytest
import torch

from oracle import clip_ref

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOL = 2e-2


@pytest.fixture(scope="module")
def cg():
    return np.load(os.path.join(REPO, "tests", "golden", "clip_golden.npz"))


def _case(cg, name):
    sd = {k.split("/sd/")[1]: torch.from_numpy(cg[k]) for k in cg.files if k.startswith(name + "/sd/")}
    return sd, torch.from_numpy(cg[name + "/ids"]), int(cg[name + "/heads"]), torch.from_numpy(cg[name + "/out"])


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm())


def _encoder(sd, heads):
    from panopticdiffusionmodels_amd.libs.clip import CLIPTextEncoder
    D = sd["final_layer_norm.weight"].numel()
    n = len({k.split(".")[2] for k in sd if k.startswith("encoder.layers.")})
    m = CLIPTextEncoder(vocab_size=sd["embeddings.token_embedding.weight"].shape[0], hidden_size=D,
                        intermediate_size=sd["encoder.layers.0.mlp.fc1.weight"].shape[0], num_hidden_layers=n,
                        num_attention_heads=heads,
                        max_position_embeddings=sd["embeddings.position_embedding.weight"].shape[0])
    m.load_state_dict(sd)
    return m


@pytest.mark.parametrize("name", ["clip_dh32", "clip_dh64"])
def test_oracle_vs_clip_golden(cg, name):
    sd, ids, heads, out = _case(cg, name)
    assert _rel(clip_ref.clip_text_forward(sd, ids, heads), out) < 1e-5


def test_state_dict_keys_and_prefixes(cg):
    sd, _, heads, _ = _case(cg, "clip_dh64")
    m = _encoder(sd, heads)
    assert set(m.state_dict()) == set(sd)
    # the reference module tree (FrozenCLIPEmbedder.transformer = CLIPTextModel, transformers 4.x keys)
    m.load_state_dict({"transformer.text_model." + k: v for k, v in sd.items()})
    for k, v in m.state_dict().items():
        assert torch.equal(v, sd[k])


def test_clip_param_table_without_gpu():
    from panopticdiffusionmodels_amd import _lib
    lib = _lib.load()
    cfg = _lib.PdmClipCfg(49408, 768, 12, 12, 3072, 77, 1e-5)
    h = ctypes.c_void_p()
    _lib.check(lib.pdm_clip_create(ctypes.byref(cfg), ctypes.byref(h)))
    n = lib.pdm_clip_param_count(h)
    assert n == 2 + 12 * 10 + 2
    buf = ctypes.create_string_buffer(256)
    total = 0
    for i in range(n):
        dt, ne = ctypes.c_int(), ctypes.c_longlong()
        _lib.check(lib.pdm_clip_param_info(h, i, buf, 256, ctypes.byref(dt), ctypes.byref(ne)))
        total += ne.value
    assert total > 123_000_000 - 1_000_000   # ViT-L/14 text tower: 123.06 M parameters (+ folded terms)
    ws = ctypes.c_size_t()
    _lib.check(lib.pdm_clip_workspace_size(h, 32, ctypes.byref(ws)))
    assert ws.value > 32 * 77 * 768 * 4
    st = lib.pdm_clip_encode(h, ctypes.c_void_p(16), 1, 77, ctypes.c_void_p(16), ctypes.c_void_p(16), 1 << 40, None)
    assert st == 3 and b"not registered" in lib.pdm_last_error()
    assert lib.pdm_clip_encode(h, ctypes.c_void_p(16), 1, 78, ctypes.c_void_p(16), None, 0, None) == 1
    lib.pdm_clip_destroy(h)
    bad = _lib.PdmClipCfg(49408, 768, 12, 10, 3072, 77, 1e-5)   # head dim 76.8
    assert lib.pdm_clip_create(ctypes.byref(bad), ctypes.byref(h)) == 1


def test_embedder_without_tokenizer_raises():
    from panopticdiffusionmodels_amd.libs.clip import FrozenCLIPEmbedder
    e = FrozenCLIPEmbedder(config=dict(vocab_size=64, hidden_size=64, intermediate_size=128, num_hidden_layers=1,
                                       num_attention_heads=2))
    with pytest.raises(RuntimeError, match="tokenizer"):
        e.encode(["a photo of a cat"])
    with pytest.raises(FileNotFoundError):
        FrozenCLIPEmbedder(version="openai/clip-vit-large-patch14")


def test_embedder_refuses_unloaded_weights(tmp_path):
    """The default-initialised encoder is not silently used; a local checkpoint loads strictly."""
    from panopticdiffusionmodels_amd.libs.clip import FrozenCLIPEmbedder
    cfg = dict(vocab_size=64, hidden_size=64, intermediate_size=128, num_hidden_layers=1, num_attention_heads=2)
    e = FrozenCLIPEmbedder(config=cfg)
    with pytest.raises(RuntimeError, match="no weights loaded"):
        e.encode_tokens(torch.zeros(1, 4, dtype=torch.int64))
    # a checkpoint directory with a key missing fails at construction (strict loading)
    import json
    from safetensors.torch import save_file
    sd = {"text_model." + k: v.contiguous() for k, v in e.transformer.state_dict().items()}
    sd.pop("text_model.final_layer_norm.bias")
    (tmp_path / "config.json").write_text(json.dumps(cfg))
    save_file(sd, str(tmp_path / "model.safetensors"))
    with pytest.raises(RuntimeError, match="final_layer_norm.bias"):
        FrozenCLIPEmbedder(version=str(tmp_path), tokenizer=lambda *a, **k: None, config=cfg)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["clip_dh32", "clip_dh64"])
def test_hip_clip_vs_transformers_golden(cg, name):
    sd, ids, heads, out = _case(cg, name)
    m = _encoder(sd, heads).cuda()
    z = m(ids.cuda()).cpu()
    assert z.shape == out.shape
    assert _rel(z, out) < TOL, _rel(z, out)
    # prefix of the sequence (L < max_position): causal, so it equals the prefix of the full output
    z20 = m(ids[:, :20].cuda()).cpu()
    assert _rel(z20, out[:, :20]) < TOL


@pytest.mark.gpu
def test_hip_clip_full_vit_l14_vs_oracle():
    from panopticdiffusionmodels_amd.libs.clip import FrozenCLIPEmbedder
    torch.manual_seed(0)
    e = FrozenCLIPEmbedder(synthetic=True)   # ViT-L/14 text shape, random weights (no checkpoint offline)
    sd = e.transformer.state_dict()
    with torch.no_grad():
        for k, v in sd.items():
            if k.endswith(".weight") and v.dim() == 2:
                v.normal_(0, 0.02)
            elif "norm" in k and k.endswith(".weight"):
                v.copy_(1 + 0.2 * torch.randn_like(v))
            else:
                v.normal_(0, 0.05)
    e = e.cuda()
    g = torch.Generator().manual_seed(3)
    ids = torch.randint(0, 49408, (4, 77), generator=g)
    ids[:, 0] = 49406
    ids[1, 9:] = 49407   # padded prompt (eos / pad tail)
    z = e.encode_tokens(ids.cuda()).cpu()
    ref = clip_ref.clip_text_forward({k: v.float() for k, v in sd.items()}, ids, 12)
    assert _rel(z, ref) < TOL, _rel(z, ref)
    # batch invariance: row 1 alone equals row 1 of the batch
    z1 = e.encode_tokens(ids[1:2].cuda()).cpu()
    assert _rel(z1, z[1:2]) < 1e-5
    with pytest.raises(IndexError):
        e.encode_tokens(torch.tensor([[49408]]).cuda())
