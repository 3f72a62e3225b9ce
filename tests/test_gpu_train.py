"""GPU parity of the LSimple training step through the C-ABI: each backward kernel against
fp32 torch autograd, the whole step against the oracle (itself pinned to the reference's training loop,
tests/test_train_oracle.py) and against the reference's own three-iteration loop (tests/golden/train_golden.npz).

Tolerances (bf16 GEMM operands, fp32 accumulation, as the reference's autocast run): per-kernel outputs rel-L2 <= 1e-2;
loss <= 1e-2; gradients per tensor rel-L2 <= 3e-2 (tiny nets) / 5e-2 (full U-ViT-L/2 shape); the optimizer in fp32
(fed the reference's own gradients) within 2 ulp per element."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEV = "cuda"


def rel(a, b):
    a, b = torch.as_tensor(a).double().cpu(), torch.as_tensor(b).double().cpu()
    return float((a - b).norm() / max(float(b.norm()), 1e-30))


@pytest.fixture(scope="module")
def tg():
    return np.load(os.path.join(REPO, "tests", "golden", "train_golden.npz"))


@pytest.mark.parametrize("tile", [0, 128, 256])
@pytest.mark.parametrize("M,N,K", [(1000, 192, 320), (33, 64, 16), (66 * 4, 64, 256), (8256, 1024, 4096),
                                   (8256, 3072, 1024), (517, 16, 1024), (300, 520, 136)])
def test_wgrad_vs_torch(M, N, K, tile):
    from panopticdiffusionmodels_amd import _lib
    _lib.check(_lib.load().pdm_set_wgrad_tile(tile))
    g = torch.Generator().manual_seed(M + N + K)
    dy = torch.randn(M, N, generator=g).bfloat16()
    x = torch.randn(M, K, generator=g).bfloat16()
    ref = dy.double().t() @ x.double()
    out = _lib.wgrad(dy.to(DEV), x.to(DEV))
    assert rel(out, ref) < 1e-5
    acc = torch.randn(N, K, generator=g)
    out2 = _lib.wgrad(dy.to(DEV), x.to(DEV), out=acc.to(DEV).clone(), accumulate=True)
    assert rel(out2, ref + acc.double()) < 1e-5
    out3 = _lib.wgrad(dy.to(DEV), x.to(DEV), scratch_mb=0)   # no scratch: one pass over the whole reduction
    _lib.check(_lib.load().pdm_set_wgrad_tile(0))
    assert rel(out3, ref) < 1e-5


@pytest.mark.parametrize("B,L,H", [(2, 66, 1), (2, 258, 2), (3, 17, 2), (1, 288, 3), (2, 257, 1), (2, 289, 1),
                                   (2, 334, 2), (2, 590, 2), (1, 608, 1), (3, 301, 1)])
def test_attention_backward_vs_autograd(B, L, H):
    """L <= 288: Q, K, V, dO resident in LDS; 288 < L <= 608 (the t2i streams: 334 image, 590 mask tokens): the
    two-images-at-a-time kernel."""
    from panopticdiffusionmodels_amd import _lib
    Dh = 64
    g = torch.Generator().manual_seed(B * 1000 + L + H)
    qkv = (torch.randn(B * L, 3 * H * Dh, generator=g) * 1.5).bfloat16()
    dout = torch.randn(B * L, H * Dh, generator=g).bfloat16()
    q = qkv.float().reshape(B, L, 3, H, Dh).permute(2, 0, 3, 1, 4).clone().requires_grad_(True)
    att = torch.softmax(q[0] @ q[1].transpose(-1, -2) * Dh ** -0.5, -1) @ q[2]
    o = att.permute(0, 2, 1, 3).reshape(B * L, H * Dh)
    o.backward(dout.float())
    ref = q.grad.permute(1, 3, 0, 2, 4).reshape(B * L, 3 * H * Dh)
    o_gpu = _lib.attention(qkv.to(DEV), B, L, H, Dh)
    dq = _lib.attention_backward(qkv.to(DEV), o_gpu, dout.to(DEV), B, L, H, Dh)
    D = H * Dh
    for part, sl in (("q", slice(0, D)), ("k", slice(D, 2 * D)), ("v", slice(2 * D, 3 * D))):
        assert rel(dq[:, sl].float(), ref[:, sl]) < 1e-2, part


@pytest.mark.parametrize("rows,D,bf", [(100, 64, True), (517, 1024, True), (300, 1152, False), (7, 512, False)])
def test_layernorm_backward_vs_autograd(rows, D, bf):
    from panopticdiffusionmodels_amd import _lib
    g = torch.Generator().manual_seed(rows + D)
    x = torch.randn(rows, D, generator=g) * 2 + 0.5
    gamma = torch.randn(D, generator=g) * 0.2 + 1
    beta = torch.randn(D, generator=g) * 0.1
    dh = torch.randn(rows, D, generator=g)
    if bf:
        dh = dh.bfloat16()
    xr = x.clone().requires_grad_(True)
    gr = gamma.clone().requires_grad_(True)
    br = beta.clone().requires_grad_(True)
    torch.nn.functional.layer_norm(xr, (D,), gr, br, 1e-5).backward(dh.float())
    acc = torch.randn(rows, D, generator=g)
    dx, dxb, dgm, dbt = _lib.layernorm_backward(x.to(DEV), dh.to(DEV), gamma.to(DEV), dx=acc.to(DEV).clone(),
                                                accumulate=True)
    assert rel(dx, xr.grad + acc) < 1e-5
    assert rel(dxb.float(), xr.grad + acc) < 5e-3
    assert rel(dgm, gr.grad) < 1e-5 and rel(dbt, br.grad) < 1e-5


def _state(name, seed=11, init="random"):
    from panopticdiffusionmodels_amd import configs, weights
    from panopticdiffusionmodels_amd.train import HipTrainState
    full = configs.get_config(name)
    sd = weights.nnet_state_dict(full["nnet"], seed=seed, init=init)
    st = HipTrainState(full["nnet"], DEV, optimizer=full.get("optimizer"), lr_scheduler=full.get("lr_scheduler"),
                       ema_rate=full.get("train", {}).get("ema_rate", 0.9999))
    st.load_state_dict(sd)
    kw = dict(full["nnet"])
    kw.pop("name")
    return full, kw, sd, st


@pytest.mark.parametrize("name", ["tiny_uvit_train", "tiny_uvit_train_uncond"])
def test_train_step_grads_vs_reference(name, tg):
    """First iteration of the reference's loop: per-sample loss and every parameter's gradient."""
    full, kw, sd, st = _state(name)
    y = torch.from_numpy(tg[f"{name}/y"]) if f"{name}/y" in tg.files else None
    loss = st.forward_backward(torch.from_numpy(tg[f"{name}/it0_xt"]), torch.from_numpy(tg[f"{name}/it0_t"]), y,
                               torch.from_numpy(tg[f"{name}/it0_eps"]))
    assert rel(loss, tg[f"{name}/it0_loss"]) < 1e-2
    grads = st.grads()
    bad = {k: rel(grads[k], tg[f"{name}/grad/{k}"]) for k in grads}
    worst = max(bad.values())
    assert worst < 3e-2, sorted(bad.items(), key=lambda kv: -kv[1])[:5]


@pytest.mark.parametrize("name", ["tiny_uvit_train", "tiny_uvit_train_uncond"])
def test_adamw_ema_vs_reference(name, tg):
    """The optimizer + EMA kernel fed the reference's own first-iteration gradients: parameters after one AdamW
    step at lr 2e-4 (and the EMA) against torch.optim.AdamW semantics (oracle.train_ref.adamw_step)."""
    from oracle import train_ref
    full, kw, sd, st = _state(name)
    opt = full["optimizer"]
    g = {k: torch.from_numpy(tg[f"{name}/grad/{k}"]) for k in sd}
    with torch.no_grad():
        for k, v in g.items():
            st._view(st.G, k).copy_(v.to(DEV).view(st._view(st.G, k).shape))
    st.lr_scheduler["warmup_steps"] = -1
    st.optimizer_step()
    p, e = st.state_dict(), st.ema_state_dict()
    for k in sd:
        pr, _, _ = train_ref.adamw_step(sd[k].float(), g[k], torch.zeros_like(g[k]), torch.zeros_like(g[k]), 1,
                                        opt["lr"], opt["betas"], 1e-8, opt["weight_decay"])
        er = train_ref.ema(sd[k].float(), pr, full["train"]["ema_rate"])
        # fp32 update of both: within 2 ulp of each element (the displacement itself is ~1e-3 of a parameter)
        assert bool(((p[k].cpu() - pr).abs() <= 2.5e-7 * pr.abs() + 1e-9).all()), k
        assert bool(((e[k].cpu() - er).abs() <= 2.5e-7 * er.abs() + 1e-9).all()), k
    # the bf16 working copy follows the parameters
    off, n = st.index["mid_block.mlp.fc1.weight"]
    assert torch.equal(st.WB[off:off + n], st.P[off:off + n].bfloat16())


@pytest.mark.parametrize("name", ["tiny_uvit_train", "tiny_uvit_train_uncond"])
def test_three_iterations_vs_reference(name, tg):
    """The reference's three-iteration loop (warm-up LR 0, 0.2 lr, 0.4 lr; EMA): losses per iteration and the final
    parameters' displacement from the initial ones."""
    full, kw, sd, st = _state(name)
    y = torch.from_numpy(tg[f"{name}/y"]) if f"{name}/y" in tg.files else None
    for i in range(3):
        loss = st.forward_backward(torch.from_numpy(tg[f"{name}/it{i}_xt"]), torch.from_numpy(tg[f"{name}/it{i}_t"]),
                                   y, torch.from_numpy(tg[f"{name}/it{i}_eps"]))
        assert rel(loss, tg[f"{name}/it{i}_loss"]) < 1e-2, i
        lr = st.optimizer_step()
        assert abs(lr - float(tg[f"{name}/it{i}_lr"])) < 1e-12
    p, e = st.state_dict(), st.ema_state_dict()
    num = den = 0.0
    for k in sd:
        d_ref = torch.from_numpy(tg[f"{name}/param/{k}"]).double() - sd[k].double()
        d = p[k].cpu().double() - sd[k].double()
        num += float((d - d_ref).norm() ** 2)
        den += float(d_ref.norm() ** 2)
        assert rel(e[k], tg[f"{name}/ema/{k}"]) < 1e-3, k
    # Adam normalises each element's step, so elements whose gradient is near zero move by a bf16-noise-driven
    # amount; the displacement as a whole must still follow the reference's
    assert (num / den) ** 0.5 < 0.25, (num / den) ** 0.5


def test_train_step_full_L2_shape_vs_oracle():
    """U-ViT-L/2 at full width / depth / token count (D 1024, 21 blocks, L 258), 2 images: loss and gradients vs the
    oracle's fp32 autograd."""
    from oracle import train_ref
    full, kw, sd, st = _state("imagenet256_uvit_large", seed=3, init="random")
    g = torch.Generator().manual_seed(8)
    B = 2
    xt = torch.randn(B, 4, 32, 32, generator=g)
    t = torch.rand(B, generator=g) * 999
    y = torch.tensor([5, 1000])
    eps = torch.randn(B, 4, 32, 32, generator=g)
    loss = st.forward_backward(xt, t, y, eps)
    lref, gref = train_ref.lsimple_grads(sd, kw, xt, t, y, eps)
    assert rel(loss, lref) < 1e-2
    grads = st.grads()
    bad = {k: rel(grads[k], gref[k]) for k in grads if float(gref[k].norm()) > 0}
    worst = max(bad.values())
    assert worst < 5e-2, sorted(bad.items(), key=lambda kv: -kv[1])[:5]


def test_train_step_batch_invariance():
    """Per-sample losses do not depend on the batch they are computed in; gradients of a duplicated batch equal those
    of the single copy (gscale = 1 / B)."""
    full, kw, sd, st = _state("tiny_uvit_train")
    g = torch.Generator().manual_seed(2)
    xt = torch.randn(3, 4, 16, 16, generator=g)
    t = torch.rand(3, generator=g) * 999
    y = torch.tensor([1, 4, 10])
    eps = torch.randn(3, 4, 16, 16, generator=g)
    l1 = st.forward_backward(xt, t, y, eps).cpu()
    g1 = {k: v.cpu() for k, v in st.grads().items()}
    l2 = st.forward_backward(torch.cat([xt, xt]), torch.cat([t, t]), torch.cat([y, y]), torch.cat([eps, eps])).cpu()
    g2 = st.grads()
    assert torch.allclose(l2[:3], l1, rtol=1e-5, atol=1e-7) and torch.allclose(l2[3:], l1, rtol=1e-5, atol=1e-7)
    for k in g1:
        assert rel(g2[k], g1[k]) < 1e-3 or float(g1[k].norm()) == 0, k


def test_train_lanes_equal_single():
    """Two concurrent half-batch lanes (HipTrainState lanes=2) give the single-lane losses and gradients (only the
    fp32 summation order of the token reduction differs), and the same parameters after an AdamW step."""
    from panopticdiffusionmodels_amd import configs, weights
    from panopticdiffusionmodels_amd.train import HipTrainState
    full = configs.get_config("tiny_uvit_train")
    sd = weights.nnet_state_dict(full["nnet"], seed=11, init="random")
    sts = []
    for lanes in (1, 2):
        st = HipTrainState(full["nnet"], DEV, optimizer=full["optimizer"], lr_scheduler=dict(warmup_steps=-1),
                           ema_rate=0.9, lanes=lanes)
        st.load_state_dict(sd)
        sts.append(st)
    g = torch.Generator().manual_seed(4)
    xt = torch.randn(5, 4, 16, 16, generator=g)
    t = torch.rand(5, generator=g) * 999
    y = torch.tensor([1, 4, 10, 0, 7])
    eps = torch.randn(5, 4, 16, 16, generator=g)
    losses = [st.forward_backward(xt, t, y, eps).cpu() for st in sts]
    assert torch.allclose(losses[0], losses[1], rtol=1e-5, atol=1e-7)
    g1, g2 = sts[0].grads(), sts[1].grads()
    for k in g1:
        assert rel(g2[k], g1[k]) < 1e-4 or float(g1[k].norm()) == 0, k
    for st in sts:
        st.optimizer_step()
    p1, p2 = sts[0].state_dict(), sts[1].state_dict()
    num = sum(float((p2[k].double() - p1[k].double()).norm() ** 2) for k in p1)
    den = sum(float((p1[k].double() - sd[k].double().to(p1[k].device)).norm() ** 2) for k in p1)
    assert (num / den) ** 0.5 < 0.05


def test_train_label_out_of_range_raises():
    """An out-of-range label raises IndexError (the reference's nn.Embedding does) instead of reading the
    neighbouring parameter as the embedding; train_step reports the NEXT step's LR as the reference logs it
    (optimizer.param_groups[0]['lr'] after lr_scheduler.step(), train_ldm_discrete.py:174-177)."""
    full, kw, sd, st = _state("tiny_uvit_train")
    nc = kw["num_classes"]
    g = torch.Generator().manual_seed(5)
    xt = torch.randn(2, 4, 16, 16, generator=g)
    t = torch.rand(2, generator=g) * 999
    eps = torch.randn(2, 4, 16, 16, generator=g)
    for bad in (nc, -1):
        with pytest.raises(IndexError):
            st.forward_backward(xt, t, torch.tensor([0, bad]), eps)
    # device-resident labels: clamped on the stream (no read outside label_emb), the error raised without a per-step
    # synchronisation -- by check_labels(), or by the next step once the offending one has finished
    loss = st.forward_backward(xt, t, torch.tensor([0, nc + 3]).cuda(), eps)
    assert torch.isfinite(loss).all()
    with pytest.raises(IndexError):
        st.check_labels()
    st.check_labels()   # reported once
    st.forward_backward(xt, t, torch.tensor([-2, 1]).cuda(), eps)
    torch.cuda.synchronize()
    with pytest.raises(IndexError):
        st.forward_backward(xt, t, torch.tensor([0, 1]).cuda(), eps)
    st.forward_backward(xt, t, torch.tensor([0, 1]).cuda(), eps)
    st.check_labels()
    st.G.zero_()
    st.lr_scheduler["warmup_steps"] = 4
    out = st.train_step(torch.randn(2, 4, 16, 16, generator=g), torch.tensor([1, nc - 1]))
    assert st.step == 1 and abs(out["lr"] - st.optimizer["lr"] * 0.25) < 1e-15


@pytest.mark.parametrize("B,L,H", [(2, 258, 2), (1, 66, 3), (2, 17, 1), (1, 415, 1), (3, 130, 1)])
def test_attention_backward_dh72_vs_autograd(B, L, H):
    """Head dim 72 (U-ViT-H/2, H/4): rows padded to 96 in LDS, five 16-wide output tiles, against fp32 autograd."""
    from panopticdiffusionmodels_amd import _lib
    Dh = 72
    g = torch.Generator().manual_seed(B * 100 + L + H)
    qkv = (torch.randn(B * L, 3 * H * Dh, generator=g) * 1.5).bfloat16()
    dout = torch.randn(B * L, H * Dh, generator=g).bfloat16()
    q = qkv.float().reshape(B, L, 3, H, Dh).permute(2, 0, 3, 1, 4).clone().requires_grad_(True)
    att = torch.softmax(q[0] @ q[1].transpose(-1, -2) * Dh ** -0.5, -1) @ q[2]
    att.permute(0, 2, 1, 3).reshape(B * L, H * Dh).backward(dout.float())
    ref = q.grad.permute(1, 3, 0, 2, 4).reshape(B * L, 3 * H * Dh)
    o_gpu = _lib.attention(qkv.to(DEV), B, L, H, Dh)
    dq = _lib.attention_backward(qkv.to(DEV), o_gpu, dout.to(DEV), B, L, H, Dh)
    D = H * Dh
    for part, sl in (("q", slice(0, D)), ("k", slice(D, 2 * D)), ("v", slice(2 * D, 3 * D))):
        assert rel(dq[:, sl].float(), ref[:, sl]) < 1e-2, part


def test_attention_backward_long_repeatable():
    """The long-sequence kernel (L = 590, the t2i mask stream) gives the same bits on every call (no atomics, fixed
    reduction order)."""
    from panopticdiffusionmodels_amd import _lib
    B, L, H, Dh = 2, 590, 2, 64
    g = torch.Generator().manual_seed(7)
    qkv = (torch.randn(B * L, 3 * H * Dh, generator=g) * 1.5).bfloat16().to(DEV)
    dout = torch.randn(B * L, H * Dh, generator=g).bfloat16().to(DEV)
    o = _lib.attention(qkv, B, L, H, Dh)
    d1 = _lib.attention_backward(qkv, o, dout, B, L, H, Dh)
    d2 = _lib.attention_backward(qkv, o, dout, B, L, H, Dh)
    assert torch.equal(d1, d2)



# ---- the panoptic t2i step (train_t2i_discrete.py:148-224, 446-473; libs/uvit_t2i.py separate streams) -----------
@pytest.fixture(scope="module")
def t2g():
    return np.load(os.path.join(REPO, "tests", "golden", "t2i_train_golden.npz"))


def _t2i_inputs(t2g, i):
    return tuple(torch.from_numpy(t2g[k]) for k in (f"it{i}_xt", f"it{i}_t", "context", f"it{i}_mask_n", f"it{i}_eps",
                                                    "scaled"))


def test_t2i_train_step_grads_vs_reference(t2g):
    """First iteration of the reference's t2i loop (tiny_t2i_train: the full token counts, Lx 334 / Lm 590, so both
    attention-backward kernels' long form runs): loss_eps, loss_mask and every gradient; parameters the forward never
    uses get none."""
    full, kw, sd, st = _state("tiny_t2i_train")
    loss, loss_m = st.forward_backward_t2i(*_t2i_inputs(t2g, 0))
    assert rel(loss, t2g["it0_loss"]) < 1e-2 and rel(loss_m, t2g["it0_loss_mask"]) < 1e-2
    grads = st.grads()
    used = {k[5:] for k in t2g.files if k.startswith("grad/")}
    bad = {k: rel(grads[k], t2g[f"grad/{k}"]) for k in used}
    worst = max(bad.values())
    assert worst < 3e-2, sorted(bad.items(), key=lambda kv: -kv[1])[:5]
    for k in set(grads) - used:
        assert float(grads[k].abs().max()) == 0.0, k


def test_t2i_two_iterations_vs_reference(t2g):
    """The reference's two-iteration t2i loop: losses and LR per iteration, the parameters' displacement; AdamW leaves
    the unused parameters (zero_convs.{even}, mask_embed_0) exactly where they were, as torch.optim does."""
    full, kw, sd, st = _state("tiny_t2i_train")
    for i in range(2):
        loss, loss_m = st.forward_backward_t2i(*_t2i_inputs(t2g, i))
        assert rel(loss, t2g[f"it{i}_loss"]) < 1e-2 and rel(loss_m, t2g[f"it{i}_loss_mask"]) < 1e-2, i
        lr = st.optimizer_step()
        assert abs(lr - float(t2g[f"it{i}_lr"])) < 1e-12
    p = st.state_dict()
    used = {k[5:] for k in t2g.files if k.startswith("grad/")}
    num = den = 0.0
    for k in sd:
        d = p[k].cpu().double() - sd[k].double()
        if k not in used:
            assert float(d.abs().max()) == 0.0, k
            continue
        d_ref = torch.from_numpy(t2g[f"delta/{k}"].astype(np.float64))
        num += float((d - d_ref).norm() ** 2)
        den += float(d_ref.norm() ** 2)
    assert (num / den) ** 0.5 < 0.25, (num / den) ** 0.5


def test_t2i_train_step_full_size_vs_oracle():
    """MSCOCO U-ViT-S/2 t2i + panoptic mask at full width / depth / token counts (D 512, 13 blocks per stream, Lx 334,
    Lm 590), 2 images: both losses and the gradients vs the oracle's fp32 autograd."""
    from oracle import train_ref
    full, kw, sd, st = _state("mscoco_uvit_small", seed=3, init="random")
    g = torch.Generator().manual_seed(8)
    B = 2
    xt = torch.randn(B, 4, 32, 32, generator=g)
    t = torch.rand(B, generator=g) * 999
    ctx = torch.randn(B, 77, 768, generator=g)
    scaled = train_ref.int2bits(torch.randint(0, 201, (B, 1, 32, 32), generator=g)) * 2 - 1
    mask_n = scaled * 0.5 + torch.randn(B, 8, 32, 32, generator=g)
    eps = torch.randn(B, 4, 32, 32, generator=g)
    loss, loss_m = st.forward_backward_t2i(xt, t, ctx, mask_n, eps, scaled)
    le, lm, gref, used = train_ref.lsimple_t2i_grads(sd, kw, xt, t, ctx, mask_n, eps, scaled)
    assert rel(loss, le) < 1e-2 and rel(loss_m, lm) < 1e-2
    grads = st.grads()
    bad = {k: rel(grads[k], gref[k]) for k in used if float(gref[k].norm()) > 0}
    worst = max(bad.values())
    assert worst < 5e-2, sorted(bad.items(), key=lambda kv: -kv[1])[:5]


# ---- head dim 72 (U-ViT-H): sketches of the reference's gradients / displacements ----------------------------------
@pytest.fixture(scope="module")
def thg():
    return np.load(os.path.join(REPO, "tests", "golden", "train_h_golden.npz"))


def _sketch_rel(key, v, ref_sk, S=8):
    """relative error of v's sketch (tests/golden/make_train_h_golden.sketch: inner products with N(0, 1) vectors seeded
    crc32(key) + i) against the reference's"""
    import zlib
    v = v.detach().double().flatten().cpu()
    sk = np.array([float(torch.randn(v.numel(), generator=torch.Generator().manual_seed(zlib.crc32(key.encode()) + i),
                                     dtype=torch.float64) @ v) for i in range(S)])
    return float(np.linalg.norm(sk - ref_sk[1:]) / max(np.linalg.norm(ref_sk[1:]), 1e-30))


def test_train_h72_grads_vs_reference(thg):
    """Head dim 72 (8 x 72, the U-ViT-H head; tiny_uvit_train_h): the reference's first-iteration loss and every
    gradient (sketch; tensors <= 4096 elements whole)."""
    full, kw, sd, st = _state("tiny_uvit_train_h")
    y = torch.from_numpy(thg["y"])
    loss = st.forward_backward(torch.from_numpy(thg["it0_xt"]), torch.from_numpy(thg["it0_t"]), y,
                               torch.from_numpy(thg["it0_eps"]))
    assert rel(loss, thg["it0_loss"]) < 1e-2
    grads = st.grads()
    bad = {k: _sketch_rel(k, grads[k], thg[f"gsk/{k}"]) for k in grads if float(thg[f"gsk/{k}"][0]) > 0}
    worst = max(bad.values())
    assert worst < 3e-2, sorted(bad.items(), key=lambda kv: -kv[1])[:5]
    for k in grads:
        if f"grad/{k}" in thg.files and float(np.linalg.norm(thg[f"grad/{k}"])) > 0:
            assert rel(grads[k], thg[f"grad/{k}"]) < 3e-2, k


def test_train_h72_three_iterations_vs_reference(thg):
    """The reference's three-iteration loop at head dim 72: losses and LR per iteration, the parameters' displacement
    (sketches, aggregated as the head-dim-64 loop test does)."""
    full, kw, sd, st = _state("tiny_uvit_train_h")
    y = torch.from_numpy(thg["y"])
    for i in range(3):
        loss = st.forward_backward(torch.from_numpy(thg[f"it{i}_xt"]), torch.from_numpy(thg[f"it{i}_t"]), y,
                                   torch.from_numpy(thg[f"it{i}_eps"]))
        assert rel(loss, thg[f"it{i}_loss"]) < 1e-2, i
        lr = st.optimizer_step()
        assert abs(lr - float(thg[f"it{i}_lr"])) < 1e-12
    p = st.state_dict()
    num = den = 0.0
    for k in sd:
        ref = thg[f"dsk/{k}"]
        e = _sketch_rel(k, p[k].cpu().double() - sd[k].double(), ref) * np.linalg.norm(ref[1:])
        num += e ** 2
        den += float(np.linalg.norm(ref[1:]) ** 2)
    assert (num / den) ** 0.5 < 0.25, (num / den) ** 0.5


def test_train_step_full_H2_shape_vs_oracle():
    """U-ViT-H/2 at full width / depth / token count (D 1152, 16 heads x 72, 29 blocks, L 258), 1 image: loss and
    gradients vs the oracle's fp32 autograd."""
    from oracle import train_ref
    full, kw, sd, st = _state("imagenet256_uvit_huge", seed=3, init="random")
    g = torch.Generator().manual_seed(9)
    xt = torch.randn(1, 4, 32, 32, generator=g)
    t = torch.rand(1, generator=g) * 999
    y = torch.tensor([7])
    eps = torch.randn(1, 4, 32, 32, generator=g)
    loss = st.forward_backward(xt, t, y, eps)
    lref, gref = train_ref.lsimple_grads(sd, kw, xt, t, y, eps)
    assert rel(loss, lref) < 1e-2
    grads = st.grads()
    bad = {k: rel(grads[k], gref[k]) for k in grads if float(gref[k].norm()) > 0}
    worst = max(bad.values())
    assert worst < 5e-2, sorted(bad.items(), key=lambda kv: -kv[1])[:5]


def test_t2i_train_lanes_equal_single(t2g):
    """The t2i step on two concurrent half-batch lanes gives the single-lane losses and gradients (fp32 summation order
    of the token reductions aside); the unused parameters stay gradient-free on both lanes."""
    from panopticdiffusionmodels_amd import configs, weights
    from panopticdiffusionmodels_amd.train import HipTrainState
    full = configs.get_config("tiny_t2i_train")
    sd = weights.nnet_state_dict(full["nnet"], seed=11, init="random")
    sts = []
    for lanes in (1, 2):
        st = HipTrainState(full["nnet"], DEV, optimizer=full["optimizer"], lr_scheduler=dict(warmup_steps=-1),
                           ema_rate=0.9, lanes=lanes)
        st.load_state_dict(sd)
        sts.append(st)
    xt, t, ctx, mask_n, eps, scaled = _t2i_inputs(t2g, 0)
    xt, t, ctx, mask_n, eps, scaled = (torch.cat([v, v.flip(0)], 0)[:3] for v in (xt, t, ctx, mask_n, eps, scaled))
    outs = [tuple(v.cpu() for v in st.forward_backward_t2i(xt, t, ctx, mask_n, eps, scaled)) for st in sts]
    for a, b in zip(outs[0], outs[1]):
        assert torch.allclose(a, b, rtol=1e-5, atol=1e-7)
    g1, g2 = sts[0].grads(), sts[1].grads()
    used = {k[5:] for k in t2g.files if k.startswith("grad/")}
    for k in g1:
        if k in used:
            assert rel(g2[k], g1[k]) < 1e-4 or float(g1[k].norm()) == 0, k
        else:
            assert float(g2[k].abs().max()) == 0.0, k
