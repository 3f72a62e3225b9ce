"""CPU checks of the training step: the oracle (oracle/train_ref.py) against the reference's own
training loop (tests/golden/train_golden.npz, tests/golden/make_train_golden.py), the host-side noise draws / LR
schedule of panopticdiffusionmodels_amd.train against the same fixtures, and the pdm_train parameter table (pure host
logic, no GPU call) against the reference state_dict keys."""
import ctypes
import os

import numpy as np
import pytest
import torch

from oracle import train_ref
from panopticdiffusionmodels_amd import configs, weights

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NAMES = ["tiny_uvit_train", "tiny_uvit_train_uncond"]


@pytest.fixture(scope="module")
def tg():
    return np.load(os.path.join(REPO, "tests", "golden", "train_golden.npz"))


def rel(a, b):
    a, b = torch.as_tensor(a).double(), torch.as_tensor(b).double()
    return float((a - b).norm() / max(float(b.norm()), 1e-30))


def _setup(name, tg):
    full = configs.get_config(name)
    cfg = full["nnet"]
    sd = weights.nnet_state_dict(cfg, seed=11, init="random")
    kw = dict(cfg)
    kw.pop("name")
    x0 = torch.from_numpy(tg[f"{name}/x0"])
    y = torch.from_numpy(tg[f"{name}/y"]) if f"{name}/y" in tg.files else None
    return full, kw, sd, x0, y


@pytest.mark.parametrize("name", NAMES)
def test_noise_draws_match_reference(name, tg):
    """Schedule.sample / VPSDE sample restated (oracle and product host code) reproduce the reference's draws."""
    from panopticdiffusionmodels_amd import train
    full, kw, sd, x0, y = _setup(name, tg)
    for i in range(3):
        nps, ts = 100 + i, 200 + i
        if full["train"]["objective"] == "discrete":
            n, eps, xt = train_ref.discrete_sample(x0, nps, ts)
            t_in = n.float()
            np.random.seed(nps)
            torch.manual_seed(ts)
            n2, eps2, xt2 = train.Schedule(train.stable_diffusion_beta_schedule()).sample(x0)
            assert torch.equal(n2.float(), t_in) and torch.equal(eps2, eps)
            assert rel(xt2, xt) < 1e-6
        else:
            t, eps, xt = train_ref.sde_sample(x0, ts)
            t_in = t * 999
            torch.manual_seed(ts)
            t2, eps2, xt2 = train.LSimple_sde_sample(train.VPSDE(), x0)
            assert torch.equal(t2, t) and torch.equal(eps2, eps)
            assert rel(xt2, xt) < 1e-6
        assert rel(t_in, tg[f"{name}/it{i}_t"]) < 1e-7
        assert torch.equal(eps, torch.from_numpy(tg[f"{name}/it{i}_eps"]))
        assert rel(xt, tg[f"{name}/it{i}_xt"]) < 1e-6
        opt = full["optimizer"]
        lr = train.customized_lr(opt["lr"], i, full["lr_scheduler"]["warmup_steps"])
        assert abs(lr - float(tg[f"{name}/it{i}_lr"])) <= 1e-12


@pytest.mark.parametrize("name", NAMES)
def test_oracle_training_loop_vs_reference(name, tg):
    """Three reference train_step iterations: losses, first-iteration gradients, final parameters and EMA."""
    full, kw, sd, x0, y = _setup(name, tg)
    draws = [(100 + i, 200 + i) for i in range(3)]
    losses, g0, p, e = train_ref.train_steps(sd, kw, x0, y, draws, full["train"]["objective"], full["optimizer"],
                                             full["lr_scheduler"]["warmup_steps"], full["train"]["ema_rate"])
    for i in range(3):
        assert rel(losses[i], tg[f"{name}/it{i}_loss"]) < 1e-5, i
    worst = max(rel(g0[k], tg[f"{name}/grad/{k}"]) for k in sd if float(np.abs(tg[f"{name}/grad/{k}"]).sum()) > 0)
    assert worst < 1e-4, worst
    for k in sd:
        d_ref = torch.from_numpy(tg[f"{name}/param/{k}"]).double() - sd[k].double()
        d = p[k].double() - sd[k].double()
        assert float((d - d_ref).norm()) <= 1e-3 * float(d_ref.norm()) + 1e-7, k
        assert rel(e[k], tg[f"{name}/ema/{k}"]) < 1e-6, k


def test_train_param_table_without_gpu():
    """pdm_train_create's flat parameter table covers exactly the reference state_dict keys with their sizes, 64-element
    aligned, in backward order (head first, embeddings last)."""
    from panopticdiffusionmodels_amd import _lib, native
    lib = _lib.load()
    for name in ["imagenet256_uvit_large", "cifar10_uvit_small", "tiny_uvit_train", "tiny_uvit_train_uncond"]:
        kw = configs.nnet_kwargs(name)
        kw.pop("name")
        h = ctypes.c_void_p()
        _lib.check(lib.pdm_train_create(ctypes.byref(native.cfg_struct(kw, False)), ctypes.byref(h)))
        spec = {k: int(np.prod(s)) for k, s, _ in weights.uvit_spec(**kw)}
        buf = ctypes.create_string_buffer(256)
        seen, offs = {}, []
        for i in range(lib.pdm_train_param_count(h)):
            off, ne = ctypes.c_longlong(), ctypes.c_longlong()
            _lib.check(lib.pdm_train_param_info(h, i, buf, 256, ctypes.byref(off), ctypes.byref(ne)))
            seen[buf.value.decode()] = ne.value
            offs.append(off.value)
            assert off.value % 64 == 0
        assert seen == spec, name
        assert offs == sorted(offs)
        keys = list(seen)
        assert keys[-1] == "patch_embed.proj.bias" and "decoder_pred.weight" in keys[:4]
        n, nwt = ctypes.c_longlong(), ctypes.c_longlong()
        _lib.check(lib.pdm_train_sizes(h, ctypes.byref(n), ctypes.byref(nwt)))
        assert n.value >= sum(spec.values())
        ws = ctypes.c_size_t()
        _lib.check(lib.pdm_train_workspace_size(h, 4, ctypes.byref(ws)))
        assert ws.value > 0
        with pytest.raises(RuntimeError):   # no buffers registered: a state error, no GPU call
            _lib.check(lib.pdm_train_refresh(h, None))
        lib.pdm_train_destroy(h)
    # unsupported nets are rejected up front
    kw = configs.nnet_kwargs("tiny_uvit_cond")   # head dim 32
    kw.pop("name")
    h = ctypes.c_void_p()
    with pytest.raises(ValueError):
        _lib.check(lib.pdm_train_create(ctypes.byref(native.cfg_struct(kw, False)), ctypes.byref(h)))


def test_gradient_average_gloo():
    """average_gradients (the DDP step between backward and AdamW) over a world-2 gloo group."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29600 + os.getpid() % 200
    ps = [ctx.Process(target=_avg_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = [q.get(timeout=120) for _ in ps]
    for p in ps:
        p.join(timeout=60)
    for r, v in out:
        assert np.allclose(v, np.arange(6, dtype=np.float32) * 1.5), (r, v)


def _avg_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from panopticdiffusionmodels_amd.train import average_gradients
    g = torch.arange(6, dtype=torch.float32) * (rank + 1)
    average_gradients(g)
    q.put((rank, g.numpy()))
    dist.destroy_process_group()


# ---- the panoptic t2i step (train_t2i_discrete.py:148-224, 446-473) ----------------------------------------------
T2I = "tiny_t2i_train"


@pytest.fixture(scope="module")
def t2g():
    return np.load(os.path.join(REPO, "tests", "golden", "t2i_train_golden.npz"))


def _t2i_setup(t2g):
    full = configs.get_config(T2I)
    cfg = full["nnet"]
    sd = weights.nnet_state_dict(cfg, seed=11, init="random")
    kw = dict(cfg)
    kw.pop("name")
    x0, ctx, pan = (torch.from_numpy(t2g[k]) for k in ("x0", "context", "panoptic"))
    return full, kw, sd, x0, ctx, pan


def test_t2i_draws_match_reference(t2g):
    """int2bits analog bits and the t2i Schedule.sample (n, eps, xn, mask_n) under the recorded seeds, from the oracle
    and from the host-side train.Schedule / train.int2bits, equal the reference's draws."""
    from panopticdiffusionmodels_amd import train
    full, kw, sd, x0, ctx, pan = _t2i_setup(t2g)
    scaled = train_ref.int2bits(pan) * 2.0 - 1.0
    assert torch.equal(scaled, torch.from_numpy(t2g["scaled"]))
    assert torch.equal(train.int2bits(pan) * 2.0 - 1.0, scaled)
    sched = train.Schedule(train.stable_diffusion_beta_schedule())
    for i, (nps, ts) in enumerate([(300, 400), (301, 401)]):
        n, eps, xn, eps_m, mask_n = train_ref.t2i_sample(x0, scaled, nps, ts)
        assert np.array_equal(n.float().numpy(), t2g[f"it{i}_t"])
        assert np.allclose(xn.numpy(), t2g[f"it{i}_xt"], atol=1e-6)
        assert np.allclose(mask_n.numpy(), t2g[f"it{i}_mask_n"], atol=1e-6)
        np.random.seed(nps)
        torch.manual_seed(ts)
        n2, eps2, xn2, eps_m2, mask_n2 = sched.sample(x0, panoptic=scaled)
        assert np.array_equal(n2.float().numpy(), t2g[f"it{i}_t"])
        assert np.allclose(mask_n2.numpy(), t2g[f"it{i}_mask_n"], atol=1e-6)


def test_t2i_oracle_loss_and_grads_vs_reference(t2g):
    """The oracle's fp32 autograd of the separate-stream panoptic net (oracle/uvit_ref.uvit_t2i_forward) against the
    reference's own first iteration: both losses and every used parameter's gradient; the parameters without a
    gradient are exactly the ones the reference leaves without one."""
    full, kw, sd, x0, ctx, pan = _t2i_setup(t2g)
    scaled = torch.from_numpy(t2g["scaled"])
    le, lm, g, used = train_ref.lsimple_t2i_grads(sd, kw, torch.from_numpy(t2g["it0_xt"]),
                                                  torch.from_numpy(t2g["it0_t"]), ctx,
                                                  torch.from_numpy(t2g["it0_mask_n"]), torch.from_numpy(t2g["it0_eps"]),
                                                  scaled)
    assert rel(le, t2g["it0_loss"]) < 1e-5 and rel(lm, t2g["it0_loss_mask"]) < 1e-5
    ref_used = {k[5:] for k in t2g.files if k.startswith("grad/")}
    assert used == ref_used
    assert {k for k in sd if k.startswith("zero_convs.")} - used == {f"zero_convs.{i}.conv.{w}" for i in range(0, 6, 2)
                                                                      for w in ("weight", "bias")}
    worst = max(rel(g[k], t2g[f"grad/{k}"]) for k in used)
    assert worst < 1e-4, worst


def test_t2i_param_table_without_gpu():
    """The t2i trainer's parameter table covers exactly the reference state_dict keys; the parameters the forward never
    uses (zero_convs.{even}, mask_embed_0) come last, after every used one."""
    from panopticdiffusionmodels_amd import _lib, native
    lib = _lib.load()
    for name in (T2I, "mscoco_uvit_small"):
        kw = configs.nnet_kwargs(name)
        kw.pop("name")
        h = ctypes.c_void_p()
        _lib.check(lib.pdm_train_create(ctypes.byref(native.cfg_struct(kw, True)), ctypes.byref(h)))
        spec = {k: int(np.prod(s)) for k, s, _ in weights.uvit_t2i_spec(**kw)}
        buf = ctypes.create_string_buffer(256)
        seen = {}
        for i in range(lib.pdm_train_param_count(h)):
            off, ne = ctypes.c_longlong(), ctypes.c_longlong()
            _lib.check(lib.pdm_train_param_info(h, i, buf, 256, ctypes.byref(off), ctypes.byref(ne)))
            seen[buf.value.decode()] = ne.value
        assert seen == spec, name
        keys = list(seen)
        unused = [k for k in keys if k.startswith("mask_embed_0.") or
                  (k.startswith("zero_convs.") and int(k.split(".")[1]) % 2 == 0)]
        assert keys[-len(unused):] == unused
        ws = ctypes.c_size_t()
        _lib.check(lib.pdm_train_workspace_size(h, 2, ctypes.byref(ws)))
        assert ws.value > 0
        lib.pdm_train_destroy(h)


# ---- head dim 72 (U-ViT-H): sketches of the reference's gradients / displacements (tests/golden/make_train_h_golden.py)
H72 = "tiny_uvit_train_h"


def sketch(key, v, S=8):
    """(norm, S projections on N(0, 1) vectors seeded crc32(key) + i) -- make_train_h_golden.sketch."""
    import zlib
    v = torch.as_tensor(v).detach().double().flatten().cpu()
    pr = [float(torch.randn(v.numel(), generator=torch.Generator().manual_seed(zlib.crc32(key.encode()) + i),
                            dtype=torch.float64) @ v) for i in range(S)]
    return np.array([float(v.norm())] + pr)


def sketch_rel(key, v, ref_sk):
    sk = sketch(key, v)
    return float(np.linalg.norm(sk[1:] - ref_sk[1:]) / max(np.linalg.norm(ref_sk[1:]), 1e-30))


@pytest.fixture(scope="module")
def thg():
    return np.load(os.path.join(REPO, "tests", "golden", "train_h_golden.npz"))


def test_h72_oracle_vs_reference(thg):
    """The oracle's fp32 autograd at head dim 72 against the reference's first iteration (loss, every gradient's
    sketch, the small tensors whole) and its three-iteration loop (losses, the displacement sketches)."""
    full = configs.get_config(H72)
    cfg = full["nnet"]
    sd = weights.nnet_state_dict(cfg, seed=11, init="random")
    kw = dict(cfg)
    kw.pop("name")
    x0, y = torch.from_numpy(thg["x0"]), torch.from_numpy(thg["y"])
    loss, g = train_ref.lsimple_grads(sd, kw, torch.from_numpy(thg["it0_xt"]), torch.from_numpy(thg["it0_t"]), y,
                                      torch.from_numpy(thg["it0_eps"]))
    assert rel(loss, thg["it0_loss"]) < 1e-5
    worst = max(sketch_rel(k, g[k], thg[f"gsk/{k}"]) for k in sd if float(thg[f"gsk/{k}"][0]) > 0)
    assert worst < 1e-4, worst
    for k in sd:
        if f"grad/{k}" in thg.files:
            assert rel(g[k], thg[f"grad/{k}"]) < 1e-4, k
    draws = [(100 + i, 200 + i) for i in range(3)]
    losses, _, p, _ = train_ref.train_steps(sd, kw, x0, y, draws, "discrete", full["optimizer"],
                                            full["lr_scheduler"]["warmup_steps"], full["train"]["ema_rate"])
    for i in range(3):
        assert rel(losses[i], thg[f"it{i}_loss"]) < 1e-5, i
    worst = max(sketch_rel(k, p[k] - sd[k].float(), thg[f"dsk/{k}"]) for k in sd if float(thg[f"dsk/{k}"][0]) > 0)
    assert worst < 1e-3, worst
