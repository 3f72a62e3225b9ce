"""Throughput of the HIP LSimple training step on one GPU.

    python tools/train_bench.py [--config imagenet256_uvit_large] [--batch 64] [--steps 5] [--warmup 2]

One step = the reference's train_step (train_ldm_discrete.py:159-175 / train_ldm.py): noise draw, forward with
saved activations, LSimple loss, backward, AdamW + EMA, on a fixed synthetic latent batch (seeded random-init
weights).  Prints one JSON line: images/s, ms per step split into forward+backward and optimizer (HIP events on the
launch stream), and the algorithmic rate: 3 x the forward's GEMM + attention FLOPs per image (dX and dW GEMMs each
cost one forward GEMM; the attention backward recomputes the scores: 7 / 2 of the forward's attention FLOPs are
counted as 2 + ... only the textbook 2.5x is counted).
"""
import argparse
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from panopticdiffusionmodels_amd import configs, weights  # noqa: E402
from panopticdiffusionmodels_amd.train import HipTrainState, Schedule, stable_diffusion_beta_schedule  # noqa: E402


def train_flops_per_image(cfg):
    D, depth = cfg["embed_dim"], cfg["depth"]
    Hd = int(D * cfg.get("mlp_ratio", 4))
    n = (cfg["img_size"] // cfg["patch_size"]) ** 2
    nb = 2 * (depth // 2) + 1

    def stream(L):
        gemm = nb * 2 * L * (3 * D * D + D * D + 2 * D * Hd) + (depth // 2) * 2 * L * 2 * D * D
        return gemm, nb * 4 * L * L * D

    if cfg["name"] == "uvit_t2i":   # image stream [time, context, patches], mask stream cat(x, m), the injections
        Lx = n + 1 + cfg.get("num_clip_token", 77)
        gi, ai = stream(Lx)
        gm, am = stream(Lx + n)
        gemm, attn = gi + gm + nb * 2 * Lx * D * D, ai + am
    else:
        gemm, attn = stream(n + (2 if cfg.get("num_classes", -1) > 0 else 1))
    return 3 * gemm + 2.5 * attn   # fwd + dX + dW GEMMs; attention fwd + the 1.5x backward (dS, dQ/dK/dV)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="imagenet256_uvit_large")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--wgrad-tile", type=int, default=0, help="dW GEMM n-tile: 0 auto, 128, 256 (A/B timing)")
    ap.add_argument("--lanes", type=int, default=2, help="concurrent half-batch lanes (HipTrainState lanes)")
    args = ap.parse_args()
    from panopticdiffusionmodels_amd import _lib
    _lib.check(_lib.load().pdm_set_wgrad_tile(args.wgrad_tile))
    full = configs.get_config(args.config)
    dev = torch.device("cuda")
    sd = weights.nnet_state_dict(full["nnet"], seed=0, init="reference")
    t2i = full["nnet"]["name"] == "uvit_t2i"
    st = HipTrainState(full["nnet"], dev, optimizer=full.get("optimizer"), lr_scheduler=full.get("lr_scheduler"),
                       ema_rate=full.get("train", {}).get("ema_rate", 0.9999), lanes=args.lanes)
    st.load_state_dict(sd)
    del sd
    g = torch.Generator().manual_seed(0)
    B = args.batch
    x0 = torch.randn(B, *full["z_shape"], generator=g).to(dev)
    ncls = full["nnet"].get("num_classes", -1)
    y = torch.randint(0, ncls, (B,), generator=g).to(dev) if ncls > 0 and not t2i else None
    if t2i:   # synthetic CLIP contexts and panoptic category masks (train_t2i_discrete.py's batch[1], batch[2])
        from panopticdiffusionmodels_amd.train import int2bits
        nn_ = full["nnet"]
        ctx = torch.randn(B, nn_.get("num_clip_token", 77), nn_.get("clip_dim", 768), generator=g).to(dev)
        pan = torch.randint(0, 201, (B, 1, nn_["img_size"], nn_["img_size"]), generator=g)
        scaled = (int2bits(pan) * 2.0 - 1.0).to(dev)
    sched = Schedule(stable_diffusion_beta_schedule())
    import numpy as np
    rng = np.random.RandomState(0)

    def step(timed):
        e = [torch.cuda.Event(enable_timing=True) for _ in range(3)] if timed else None
        if t2i:
            n, eps, xn, eps_m, mask_n = sched.sample(x0, rng, panoptic=scaled)
            if timed:
                e[0].record()
            loss, loss_m = st.forward_backward_t2i(xn, n.float(), ctx, mask_n, eps, scaled)
            loss = loss + loss_m
        else:
            n, eps, xn = sched.sample(x0, rng)
            if timed:
                e[0].record()
            loss = st.forward_backward(xn, n.float(), y, eps)
        if timed:
            e[1].record()
        st.optimizer_step()
        if timed:
            e[2].record()
        return loss, e

    for _ in range(args.warmup):
        step(False)
    torch.cuda.synchronize()
    evs = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss, e = step(True)
        evs.append(e)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.steps
    fb = sum(e[0].elapsed_time(e[1]) for e in evs) / len(evs)
    opt = sum(e[1].elapsed_time(e[2]) for e in evs) / len(evs)
    fl = train_flops_per_image(full["nnet"])
    ips = B / dt
    print(json.dumps({
        "metric": f"training images/s, {args.config} LSimple step{' (panoptic: loss_eps + loss_mask)' if t2i else ''} "
                  f"(fwd + bwd + AdamW + EMA), 1 GPU",
        "value": round(ips, 2), "unit": "images/sec", "batch": B, "steps": args.steps, "ms_per_step": round(dt * 1e3, 2),
        "fwd_bwd_ms": round(fb, 2), "adamw_ema_ms": round(opt, 2), "params": sum(v[1] for v in st.index.values()),
        "algorithmic_tflop_per_image": round(fl / 1e12, 4), "achieved_tflops": round(ips * fl / 1e12, 1),
        "frac_of_bf16_peak": round(ips * fl / 2.5e15, 4), "loss": float(loss.mean()),
        "workspace_gb": round(st.ws.numel() / 1e9, 2), "wgrad_tile": args.wgrad_tile or "auto",
        "lanes": st.lanes}), flush=True)


if __name__ == "__main__":
    main()
