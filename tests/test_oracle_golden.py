"""Pin the CPU oracle against vectors produced by the reference itself (tests/golden/make_golden.py).

Tolerance for the fp32 restatement vs the reference: rel-L2 <= 1e-5, per-element
abs 1e-5 on O(1) data.
"""
import numpy as np
import pytest
import torch

from oracle import autoencoder_ref, solver_ref, utils_ref, uvit_ref
from panopticdiffusionmodels_amd import configs as C
from panopticdiffusionmodels_amd import weights as W


def rel_l2(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def _sd(name, golden):
    cfg = C.nnet_kwargs(name)
    sd = W.nnet_state_dict(cfg, seed=11, init="random")
    chk = np.array([float(v.double().sum()) for v in sd.values()] + [float(v.double().abs().sum()) for v in sd.values()])
    np.testing.assert_allclose(chk, golden[f"{name}/sd_checksum"], rtol=1e-12, atol=1e-9)
    return cfg, sd


@pytest.mark.parametrize("name", ["tiny_uvit_cond", "tiny_uvit_h", "tiny_uvit_uncond"])
def test_uvit_forward(golden, name):
    cfg, sd = _sd(name, golden)
    x = torch.from_numpy(golden[f"{name}/in_x"])
    t = torch.from_numpy(golden[f"{name}/in_t"])
    y = torch.from_numpy(golden[f"{name}/in_y"]) if f"{name}/in_y" in golden else None
    eps = uvit_ref.uvit_forward(sd, cfg, x, t, y)
    assert rel_l2(eps, golden[f"{name}/eps"]) < 1e-5


def test_uvit_t2i_forward(golden):
    name = "tiny_t2i"
    cfg, sd = _sd(name, golden)
    g = {k: torch.from_numpy(golden[f"{name}/in_{k}"]) for k in ("x", "t", "context", "mask_token")}
    eps, pm = uvit_ref.uvit_t2i_forward(sd, cfg, g["x"], g["t"], g["context"], mask_token=g["mask_token"])
    assert rel_l2(eps, golden[f"{name}/eps_mask"]) < 1e-5
    assert rel_l2(pm, golden[f"{name}/pred_mask"]) < 1e-5
    eps = uvit_ref.uvit_t2i_forward(sd, cfg, g["x"], g["t"], g["context"])
    assert rel_l2(eps, golden[f"{name}/eps_nomask"]) < 1e-5
    eps, _ = uvit_ref.uvit_t2i_forward(sd, cfg, g["x"], g["t"], g["context"], mask_token=g["mask_token"],
                                       use_ground_truth=True)
    assert rel_l2(eps, golden[f"{name}/eps_gt"]) < 1e-5


def test_ops(golden):
    t = torch.from_numpy(golden["ops/temb_t"])
    for dim in (64, 144, 1024, 1152, 7):
        np.testing.assert_allclose(uvit_ref.timestep_embedding(t, dim).numpy(), golden[f"ops/temb_{dim}"], atol=2e-6)
    for p, c in ((2, 4), (4, 4), (2, 8)):
        x = torch.from_numpy(golden[f"ops/unpatch_in_{p}_{c}"])
        np.testing.assert_array_equal(uvit_ref.unpatchify(x, c).numpy(), golden[f"ops/unpatch_out_{p}_{c}"])
    for L in (257, 258, 334, 590):
        for Dh in (64, 72):
            D = 2 * Dh
            gg = torch.Generator().manual_seed(1000 + L * 100 + Dh)
            x = torch.randn(1, L, D, generator=gg)
            sd = {"a.qkv.weight": torch.randn(3 * D, D, generator=gg) * D ** -0.5,
                  "a.proj.weight": torch.randn(D, D, generator=gg) * D ** -0.5,
                  "a.proj.bias": torch.randn(D, generator=gg) * 0.1}
            o = uvit_ref.attention(sd, "a", x, 2)
            assert rel_l2(o[0, ::7, :], golden[f"ops/attn_{L}_{Dh}"]) < 1e-5


def test_schedules(golden):
    ns = solver_ref.DiscreteSchedule(golden["solver/betas"])
    tg = torch.from_numpy(golden["solver/pp_grid_t"])
    np.testing.assert_allclose(ns.log_mean(tg), golden["solver/pp_log_mean"], rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(ns.std(tg), golden["solver/pp_std"], rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(ns.lam(tg), golden["solver/pp_lambda"], rtol=1e-6, atol=1e-6)
    lam = torch.from_numpy(golden["solver/pp_inv_lambda_in"])
    np.testing.assert_allclose(ns.inv_lam(lam), golden["solver/pp_inv_lambda"], rtol=1e-6, atol=1e-7)
    nl = solver_ref.LinearSchedule()
    tl = torch.from_numpy(golden["solver/lin_t"])
    np.testing.assert_allclose(nl.log_mean(tl), golden["solver/lin_log_mean"], rtol=1e-6, atol=1e-8)
    np.testing.assert_allclose(nl.lam(tl), golden["solver/lin_lambda"], rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(nl.inv_lam(nl.lam(tl)), golden["solver/lin_inv_lambda"], rtol=1e-5, atol=1e-7)


def _eps_fn(x, t):
    return torch.tanh(x) * (0.3 + 0.5 * t.reshape(-1, 1, 1, 1)) + 0.1 * torch.roll(x, 1, dims=-1)


def _mask_fn(m, t):
    return torch.tanh(0.7 * m + t.reshape(-1, 1, 1, 1))


def test_pp_solver_analytic(golden):
    betas = golden["solver/betas"]
    x0 = torch.from_numpy(golden["solver/x_init"])
    m0 = torch.from_numpy(golden["solver/mask_init"])
    calls = []

    def model(x, t, m):
        calls.append(t.numpy().copy())
        return _eps_fn(x, t), None
    x, _ = solver_ref.pp_sample(model, betas, x0.clone(), steps=50)
    np.testing.assert_allclose(np.stack(calls), golden["solver/pp_calls_t"], rtol=2e-6, atol=1e-7)
    assert rel_l2(x, golden["solver/pp_final"]) < 1e-5

    def model_m(x, t, m):
        return _eps_fn(x, t) + 0.05 * m[:, :4], _mask_fn(m, t)
    x, pm = solver_ref.pp_sample(model_m, betas, x0.clone(), steps=50, mask_token=m0.clone(), enable_mask_opt=True)
    assert rel_l2(x, golden["solver/ppm_final"]) < 1e-5
    assert rel_l2(pm, golden["solver/ppm_pred_mask"]) < 1e-5
    x, pm = solver_ref.pp_sample(model_m, betas, x0.clone(), steps=50, mask_token=m0.clone(), enable_mask_opt=False)
    assert rel_l2(x, golden["solver/ppm_noopt_final"]) < 1e-5
    assert rel_l2(pm, golden["solver/ppm_noopt_pred_mask"]) < 1e-5
    for steps in (10, 12, 20, 21):
        x, _ = solver_ref.pp_sample(model, betas, x0.clone(), steps=steps, eps=1e-3)
        assert rel_l2(x, golden[f"solver/pp_final_steps{steps}"]) < 1e-5


def test_pytorch_solver_analytic(golden):
    x0 = torch.from_numpy(golden["solver/x_init"])
    calls = []

    def model(x, t):
        calls.append((t * 999).numpy().copy())
        return _eps_fn(x, t * 999 / 999.0)
    x = solver_ref.pytorch_sample(model, x0.clone(), steps=50, eps=1e-4)
    np.testing.assert_allclose(np.stack(calls), golden["solver/pt_calls_t999"], rtol=2e-6, atol=1e-4)
    assert rel_l2(x, golden["solver/pt_final"]) < 1e-5
    for steps in (10, 12, 20, 21):
        x = solver_ref.pytorch_sample(lambda a, t: _eps_fn(a, t * 999 / 999.0), x0.clone(), steps=steps, eps=1e-4)
        assert rel_l2(x, golden[f"solver/pt_final_steps{steps}"]) < 1e-5


@pytest.mark.parametrize("name", ["tiny_uvit_cond", "tiny_uvit_h", "tiny_t2i"])
def test_tiny_sample(golden, name):
    cfg, sd = _sd(name, golden)
    full = C.get_config(name)
    z0 = torch.from_numpy(golden[f"sample/{name}/z_init"])
    if name == "tiny_uvit_cond":
        y = torch.from_numpy(golden[f"sample/{name}/y"])
        net = lambda x, t, yy: uvit_ref.uvit_forward(sd, cfg, x, t, yy)  # noqa: E731
        fn = solver_ref.cfg_class_closure(net, y, full["cfg_scale"], cfg["num_classes"] - 1, 999)
        z = solver_ref.pytorch_sample(fn, z0.clone(), steps=50, eps=1e-4)
        assert rel_l2(z, golden[f"sample/{name}/z"]) < 1e-5
    elif name == "tiny_uvit_h":
        y = torch.from_numpy(golden[f"sample/{name}/y"])
        net = lambda x, t, yy: uvit_ref.uvit_forward(sd, cfg, x, t, yy)  # noqa: E731
        fn = solver_ref.cfg_class_closure(net, y, full["cfg_scale"], cfg["num_classes"] - 1, 1000)
        z, _ = solver_ref.pp_sample(lambda x, t, m: (fn(x, t), None), golden["solver/betas"], z0.clone(), steps=50)
        assert rel_l2(z, golden[f"sample/{name}/z"]) < 1e-5
    else:
        ctx = torch.from_numpy(golden[f"sample/{name}/context"])
        empty = torch.from_numpy(golden[f"sample/{name}/empty_context"])
        m0 = torch.from_numpy(golden[f"sample/{name}/mask_init"])

        def net(x, t, c, m=None):
            return uvit_ref.uvit_t2i_forward(sd, cfg, x, t, c, mask_token=m)
        fn = solver_ref.cfg_t2i_closure(net, ctx, empty, full["cfg_scale"])
        z, pm = solver_ref.pp_sample(fn, golden["solver/betas"], z0.clone(), steps=50, mask_token=m0.clone(),
                                     enable_mask_opt=True)
        assert rel_l2(z, golden[f"sample/{name}/z"]) < 1e-5
        assert rel_l2(pm, golden[f"sample/{name}/pred_mask"]) < 1e-5


def test_decoder(golden):
    sd = W.make_state_dict(W.decoder_spec(ch=32, ch_mult=(1, 2), num_res_blocks=1), seed=13, init="random")
    chk = np.array([float(v.double().sum()) for v in sd.values()] + [float(v.double().abs().sum()) for v in sd.values()])
    np.testing.assert_allclose(chk, golden["decoder/sd_checksum"], rtol=1e-12, atol=1e-9)
    z = torch.from_numpy(golden["decoder/z"])
    img = autoencoder_ref.decode(sd, z, ch_mult=(1, 2), num_res_blocks=1)
    assert rel_l2(img, golden["decoder/img"]) < 1e-5


@pytest.mark.parametrize("key,ch,mult,nrb,seed,init", [
    ("decoder64", 64, (1, 2), 1, 7, "random"),
    ("decoder_full", 128, (1, 2, 4, 4), 2, 1, "reference"),
])
def test_decoder_sizes(golden, key, ch, mult, nrb, seed, init):
    sd = W.make_state_dict(W.decoder_spec(ch=ch, ch_mult=mult, num_res_blocks=nrb), seed=seed, init=init)
    chk = np.array([float(v.double().sum()) for v in sd.values()] + [float(v.double().abs().sum()) for v in sd.values()])
    np.testing.assert_allclose(chk, golden[f"{key}/sd_checksum"], rtol=1e-12, atol=1e-9)
    img = autoencoder_ref.decode(sd, torch.from_numpy(golden[f"{key}/z"]), ch_mult=mult, num_res_blocks=nrb)
    assert rel_l2(img, golden[f"{key}/img"]) < 1e-5


def test_utils(golden):
    ids = golden["utils/ids"]
    np.testing.assert_array_equal(utils_ref.int2bits(ids), golden["utils/bits"].astype(np.int64))
    np.testing.assert_array_equal(utils_ref.bits2int(golden["utils/bits"] > 0), golden["utils/bits2int"].astype(np.int64))
    am = list(golden["utils/amortize"])
    k = am.index(-1)
    assert utils_ref.amortize(103, 25) == am[:k] and utils_ref.amortize(100, 25) == am[k + 1:]
