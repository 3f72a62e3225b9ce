#!/usr/bin/env python3
"""Throughput benchmark of the sampling hot path (BASELINE.json metric).

Workload (BASELINE.json configs[1]): configs/imagenet256_uvit_large.py — U-ViT-L/2, 50-step DPM-Solver
(dpm_solver_pytorch fast, eval_ldm.py:93-108), classifier-free guidance 0.4, KL-f8 decode to 256x256,
bf16 compute, synthetic seeded weights and inputs.  One "step" = one batch of B images per GPU:
z_T -> 50 NFE (each = one 2B-row U-ViT forward + fused CFG/solver epilogue) -> all-gather of the final
latents over RCCL (N > 1) -> decode of the rank's own B latents.

  python bench.py [--gpus N --steps K --warmup W --batch B]
  torchrun --nproc-per-node N bench.py --gpus N ...   (one process per GPU, RCCL over xGMI)

Rank 0 prints one JSON line.  `value` = images/sec of the whole job = N*B*K / max-over-ranks wall time.
The CPU baseline (rank 0, N = 1 only, after the GPU timing) times the fp32 CPU oracle on a bounded sample of the
same workload: one full 50-NFE CFG sample of 2 images + their decode.
"""
import argparse
import json
import os
import sys
import time

# HIP hardware queues: the environment's (the box's default of 4).  The sampling lanes run on high-priority streams
# of their own queue pool (sampler.py), so they stay concurrent beside the launch stream and RCCL's.

import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

from panopticdiffusionmodels_amd import configs, parallel, weights  # noqa: E402
from panopticdiffusionmodels_amd.libs.autoencoder import get_model  # noqa: E402
from panopticdiffusionmodels_amd.sampler import ClassCondSampler  # noqa: E402
from panopticdiffusionmodels_amd.utils import get_nnet  # noqa: E402

PEAK_BF16 = 2.5e15   # dense bf16 MFMA, MI355X_MICROARCH.md chip table
PEAK_FP8 = 5.0e15    # dense MX-fp8 (block-scaled 16x16x128 f8f6f4) MFMA, same table
MODEL_NAMES = {"imagenet256_uvit_large": "U-ViT-L/2", "imagenet256_uvit_huge": "U-ViT-H/2",
               "imagenet512_uvit_huge": "U-ViT-H/4", "cifar10_uvit_small": "U-ViT-S/2 (pixel)",
               "mscoco_uvit_small": "U-ViT-S/2 t2i + panoptic mask (CLIP ViT-L/14 text encoder)"}
# algorithmic TFLOP per image (50 NFE x CFG forward + decode; t2i adds the CLIP encoder, 13.1 GF)
TF_PER_IMAGE = {"imagenet256_uvit_large": 15.913, "imagenet256_uvit_huge": 27.261, "imagenet512_uvit_huge": 29.160,
                "mscoco_uvit_small": 10.221 + 0.0131, "cifar10_uvit_small": 1.220}
CLIP_BOS, CLIP_EOS = 49406, 49407
FP8_SET = {"fp8": "qkv/proj/fc2", "fp8-all": "qkv/proj/fc1/fc2"}   # libs/uvit.py UViT.set_precision


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=None,
                    help="images per GPU per step (default: the config's mini_batch_size -- the reference's 50 "
                         "for ImageNet, configs/imagenet256_uvit_large.py:66; 32 for MSCOCO; BASELINE's 4 for "
                         "CIFAR-10)")
    ap.add_argument("--config", default="imagenet256_uvit_large")
    ap.add_argument("--lanes", type=int, default=2,
                    help="sample the batch as this many concurrent sub-batches on their own streams (fills the "
                         "partly idle last GEMM wave of batches whose rows tile the 256-row GEMM unevenly)")
    ap.add_argument("--no-decode", action="store_true")
    ap.add_argument("--decode-lanes", type=int, default=2, help="concurrent decode chunks (libs/autoencoder.py)")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--cpu-baseline", choices=["auto", "off"], default="auto")
    ap.add_argument("--precision", choices=["bf16", "fp8", "fp8-all"], default=None,
                    help="override the config's block-Linear precision (configs[4] default: fp8)")
    return ap.parse_args()


def gemm_flops_per_forward(cfg, rows):
    D, depth = cfg["embed_dim"], cfg["depth"]
    Hd = int(D * cfg.get("mlp_ratio", 4))
    L = (cfg["img_size"] // cfg["patch_size"]) ** 2 + (2 if cfg.get("num_classes", -1) > 0 else 1)
    M = rows * L
    per_block = 2 * M * (3 * D * D + D * D + 2 * D * Hd)
    return (depth + 1) * per_block + (depth // 2) * 2 * M * 2 * D * D


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1:
            raise SystemExit("for --gpus > 1 launch with torch.distributed.run (one process per GPU)")
        raise SystemExit(f"WORLD_SIZE={world} but --gpus {args.gpus}: launch one process per GPU with "
                         f"--nproc-per-node equal to --gpus")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    # any launch through torch.distributed.run (RANK/MASTER_ADDR set) joins an RCCL group, world size 1 included,
    # so the barrier / all_reduce(MAX) / all-gather legs run exactly as at N > 1
    distributed = "RANK" in os.environ and "MASTER_ADDR" in os.environ
    if distributed:
        dist.init_process_group("nccl", device_id=dev)

    full = configs.get_config(args.config)
    ncfg = dict(full["nnet"])
    B = args.batch if args.batch is not None else int(full.get("mini_batch_size", 50))
    # weights: seeded synthetic (no checkpoints offline); identical on every rank
    sd = weights.nnet_state_dict(ncfg, seed=0, init="reference", device=dev)
    net = get_nnet(**ncfg).to(dev).eval()
    net.load_state_dict(sd)
    del sd
    precision = args.precision or full.get("precision", "bf16")   # configs[4]: MXFP8 (UViT.set_precision)
    if hasattr(net, "set_precision"):
        net.set_precision(precision)
    t2i = ncfg["name"] == "uvit_t2i"
    null_label = ncfg["num_classes"] - 1 if ncfg.get("num_classes", -1) > 0 else None
    if t2i:   # configs[3]: prompts -> CLIP contexts (sample_t2i_discrete.py:49-53) -> panoptic co-generation
        from panopticdiffusionmodels_amd.libs.clip import FrozenCLIPEmbedder
        from panopticdiffusionmodels_amd.sampler import T2ISampler
        clip = FrozenCLIPEmbedder(synthetic=True)
        with torch.no_grad():   # seeded synthetic ViT-L/14 text weights (no checkpoint offline)
            g = torch.Generator().manual_seed(5)
            for k, v in clip.transformer.state_dict().items():
                if "norm" in k and k.endswith(".weight"):
                    v.fill_(1.0)
                elif v.dim() == 2:
                    v.copy_(torch.randn(v.shape, generator=g) * 0.02)
                else:
                    v.zero_()
        clip = clip.to(dev)
        sampler = T2ISampler(net, cfg_scale=full["cfg_scale"], steps=full["sample_steps"],
                             use_graph=not args.no_graph, lanes=args.lanes)
        empty_ids = torch.full((1, 77), CLIP_EOS, dtype=torch.int64)
        empty_ids[0, 0] = CLIP_BOS
        empty_ctx = clip.encode_tokens(empty_ids.to(dev))[0]   # the dataset's empty_context (datasets.py:629)
    else:
        sampler = ClassCondSampler(net, front_end=full["front_end"], cfg_scale=full["cfg_scale"],
                                   null_label=null_label, steps=full["sample_steps"], eps=full.get("eps"),
                                   use_graph=not args.no_graph, lanes=args.lanes)
    # configs[0] (CIFAR-10) samples pixels: no autoencoder (eval.py:56-86)
    decode = full.get("decode", True) and not args.no_decode
    ae = get_model(None, scale_factor=full.get("scale_factor", 0.18215), seed=1,
                   lanes=args.decode_lanes).to(dev) if decode else None

    # inputs for every (warmup + timed) step, generated per GLOBAL sample index and resident in HBM
    nsteps = args.warmup + args.steps
    zs, ys = [], []
    zshape = full["z_shape"]
    for s in range(nsteps):   # step s covers global samples [s*world*B, (s+1)*world*B), this rank its shard
        idx = [s * world * B + i for i in parallel.shard(world * B, world, rank)]
        z, y = parallel.sample_inputs(idx, zshape, num_classes=1000 if null_label is not None else None)
        zs.append(z.to(dev))
        if t2i:   # synthetic tokenised prompts (BOS, 5..60 body tokens, EOS padding) + mask tokens, per global index
            ids = torch.full((len(idx), 77), CLIP_EOS, dtype=torch.int64)
            mts = []
            for r, i in enumerate(idx):
                gi = torch.Generator().manual_seed(4321 * 1_000_003 + i)
                n = int(torch.randint(5, 61, (1,), generator=gi))
                ids[r, 0] = CLIP_BOS
                ids[r, 1:1 + n] = torch.randint(0, CLIP_BOS, (n,), generator=gi)
                mts.append(torch.randn(1, ncfg["num_panoptic_class"], *zshape[1:], generator=gi))
            ys.append((ids.to(dev), torch.cat(mts).to(dev)))
        else:
            ys.append(y.to(dev) if y is not None else None)

    from panopticdiffusionmodels_amd import _lib
    prof = _lib.GemmProfiler(net.native(), max_launches=512)

    ev = []   # (start, after sampling, after decode) HIP events per timed step, on the launch stream

    def one_step(s, timed=False):
        if timed:
            e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            e[0].record()
        if t2i:
            ids, mt = ys[s]
            z, _pred_mask = sampler.sample(zs[s], clip.encode_tokens(ids), empty_ctx, mt)
        else:
            z = sampler.sample(zs[s], ys[s])
        if distributed:
            z = parallel.gather_latents(z)[rank * B:(rank + 1) * B]
        if timed:
            e[1].record()
        out = ae.decode(z) if ae is not None else z
        if timed:
            e[2].record()
            ev.append(e)
        return out

    for s in range(args.warmup):
        one_step(s)
    torch.cuda.synchronize(dev)
    if distributed:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for s in range(args.warmup, nsteps):
        out = one_step(s, timed=True)
    torch.cuda.synchronize(dev)
    if distributed:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    if distributed:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    assert torch.isfinite(out).all()

    # ---- roofline of the dominant kernel (the bf16 GEMM family), after the timed region: the last step's inputs
    # sampled once more eagerly with libpdm's HIP events around every GEMM launch (recorded on the launch stream);
    # the last forward's launches are read back -- the kernels and shapes of the timed steps
    prof.enable()
    if t2i:
        ids, mt = ys[-1]
        T2ISampler(net, cfg_scale=full["cfg_scale"], steps=full["sample_steps"], use_graph=False).sample(
            zs[-1], clip.encode_tokens(ids), empty_ctx, mt)
    else:
        sampler.sample(zs[-1], ys[-1], eager=True)
    prof.disable()
    torch.cuda.synchronize(dev)
    roof = gemm_roofline(prof, ncfg, 2 * B if t2i or sampler.cfg else B, precision, config=args.config)
    samp_ms = sum(e[0].elapsed_time(e[1]) for e in ev) / len(ev)
    dec_ms = sum(e[1].elapsed_time(e[2]) for e in ev) / len(ev)
    if roof and roof.get("flops_per_forward"):
        # the timed configuration itself (two concurrent lanes of half the rows, graph replay) has overlapping
        # kernels whose durations are not rates; this bounds the GEMM family's rate there from below
        gemm_tf = roof["flops_per_forward"] * sampler.nfe / 1e12
        rate = gemm_tf / (samp_ms / 1e3)
        roof["timed_config"] = {
            "lanes": sampler.lanes, "gemm_tflop_per_step": round(gemm_tf, 2), "sample_ms_per_step": round(samp_ms, 2),
            "gemm_rate_lower_bound_tflops": round(rate, 1), "frac_lower_bound": round(rate / roof["peak"], 4),
            "note": "every GEMM FLOP of one timed step's sampling / that step's whole sampling time (attention, small "
                    "kernels and launch gaps counted as GEMM time): a lower bound on the GEMM family's rate in the "
                    "timed lanes configuration"}

    images = world * B * args.steps
    value = images / elapsed
    tf_img = TF_PER_IMAGE.get(args.config)
    res = {
        "metric": metric_name(args.config, zshape, ae is not None),
        "value": round(value, 3),
        "unit": "images/sec",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16" if precision == "bf16" else f"mxfp8-e4m3 ({FP8_SET[precision]}) + bf16",
        "data": f"synthetic (seeded random-init {MODEL_NAMES.get(args.config, args.config)} + KL-f8 weights, "
                + ("z_T ~ N(0,1), token ids of 5-60-token prompts, mask tokens ~ N(0,1))" if t2i
                   else "z_T ~ N(0,1), labels U{0..999})"),
        "config": {"workload": f"{args.config}: 50-step DPM-Solver (fast, order 3), CFG {full['cfg_scale']}, "
                               f"{f'+ KL-f8 decode {8 * zshape[-1]}x{8 * zshape[-1]}' if ae is not None else 'no decode'}",
                   "model": MODEL_NAMES.get(args.config, args.config), "per_gpu_batch": B, "global_batch": world * B,
                   "nfe": sampler.nfe, "hip_graph": not args.no_graph, "parallelism": f"dp{world} (batch-sharded)",
                   "lanes": sampler.lanes},
        "roofline": roof,
        "end_to_end": None if tf_img is None or (ae is None and decode_expected(full)) else
        end_to_end(value, world, tf_img, ncfg, full, precision, sampler.nfe),
        "breakdown_ms_per_step": {"sample_50nfe": round(samp_ms, 2), "decode": round(dec_ms, 2),
                                  "note": "HIP events on the launch stream around each timed step (graph replay)"},
    }
    if rank == 0 and world == 1 and args.cpu_baseline == "auto":
        res["cpu_baseline"] = cpu_baseline(full, ncfg, ae is not None)
    if rank == 0:
        print(json.dumps(res), flush=True)
    if distributed:
        dist.destroy_process_group()


def decode_expected(full):
    return bool(full.get("decode", True))


def end_to_end(value, world, tf_img, ncfg, full, precision, nfe):
    """images/s x algorithmic FLOPs per image against the roofline time of one image: every
    FLOP at its dense MFMA peak -- bf16, or for the MXFP8 configs[4] the block Linears the precision mode runs in
    fp8 at the fp8 peak and everything else (skip_linear, fc1 in 'fp8', attention, decode) at the bf16 peak."""
    peak_s = tf_img * 1e12 / PEAK_BF16
    note = "whole job: images/s x algorithmic FLOPs per image (SURVEY.md §8d) vs N x the dense bf16 peak"
    if precision != "bf16":
        D, depth = ncfg["embed_dim"], ncfg["depth"]
        Hd = int(D * ncfg.get("mlp_ratio", 4))
        L = (ncfg["img_size"] // ncfg["patch_size"]) ** 2 + 2
        lin = {"qkv": 3 * D * D, "proj": D * D, "fc1": D * Hd, "fc2": Hd * D}
        fp8 = ("qkv", "proj", "fc2") if precision == "fp8" else ("qkv", "proj", "fc1", "fc2")
        rows_per_img = nfe * (2 if full.get("cfg_scale", 0) > 0 else 1)
        f8 = rows_per_img * (depth + 1) * 2.0 * L * sum(lin[k] for k in fp8)
        peak_s = (tf_img * 1e12 - f8) / PEAK_BF16 + f8 / PEAK_FP8
        note = (f"whole job vs the FLOP-weighted dense peak: {f8 / 1e12:.2f} of {tf_img} TF per image "
                f"({'/'.join(fp8)}) at the MXFP8 peak, the rest at bf16")
    return {"algorithmic_tflop_per_image": tf_img, "achieved_tflops": round(value * tf_img, 1),
            "frac_of_peak": round(value * peak_s / world, 4),
            "roofline_images_per_sec": round(world / peak_s, 1), "note": note}


def metric_name(config, zshape, with_decode):
    """BASELINE.json's metric for the headline config; the same wording with the model / resolution of the
    other configs (their lines are extra evidence, not the headline)."""
    if config == "imagenet256_uvit_large" and with_decode:
        return "images/sec (whole node), ImageNet256 U-ViT-L 50-step DPM-Solver, 1/2/4/8 GPU"
    data = {"imagenet256_uvit_huge": "ImageNet256", "imagenet512_uvit_huge": "ImageNet512",
            "mscoco_uvit_small": "MSCOCO256 t2i + panoptic", "cifar10_uvit_small": "CIFAR10"}.get(config, config)
    if config == "cifar10_uvit_small":   # pixel-space net: the sample IS the image (eval.py:56-86)
        return (f"images/sec (whole node), {data} {MODEL_NAMES.get(config, config)} 50-step DPM-Solver, "
                f"{zshape[-1]}x{zshape[-1]} pixels (no decoder)")
    res = 8 * zshape[-1]
    return (f"images/sec (whole node), {data} {MODEL_NAMES.get(config, config)} 50-step DPM-Solver"
            f"{f', {res}x{res} decode' if with_decode else ', latents only (no decode)'}")


def measured_traffic(config, rows, precision):
    """HBM bytes per GEMM launch from the newest committed PMC summary of this config / batch / precision
    (tools/profile_bench.sh + tools/summarize_prof.py: FETCH_SIZE x 2 + WRITE_SIZE, separate rocprofv3 passes),
    or None when no summary was collected for these shapes."""
    import glob
    for f in sorted(glob.glob(os.path.join(REPO, "profiles", "*_traffic.json")), reverse=True):
        d = json.load(open(f))
        key = (d.get("config", "imagenet256_uvit_large"), d.get("rows", 190), d.get("precision", "bf16"))
        if key == (config, rows, precision) and d.get("gemm_family"):
            return d["gemm_family"]["hbm_bytes_per_launch"], os.path.basename(f)
    return None, None


def gemm_roofline(prof, ncfg, rows, precision="bf16", config="imagenet256_uvit_large"):
    """GEMM-family roofline; `traffic` from the committed PMC summary of these shapes (config, rows,
    precision), null when none was collected."""
    times_ms, flops = prof.read()
    n = len(times_ms)
    tot_t = sum(times_ms) / 1e3
    tot_f = sum(flops)
    achieved = tot_f / tot_t
    traffic, tsrc = measured_traffic(config, rows, precision)
    kernel = "bf16 GEMM family (all U-ViT linear layers: qkv, proj, fc1, fc2, skip_linear" + \
        (", context_embed, zero_convs)" if ncfg["name"] == "uvit_t2i" else ")")
    peak = PEAK_BF16
    if precision != "bf16":
        # mixed family: MXFP8 qkv/proj/fc2 (+ fc1 for 'fp8-all'), bf16 skip_linear (K = 2D) and fc1 ('fp8');
        # peak = the FLOP-weighted harmonic mean of the two dense peaks
        D, L = ncfg["embed_dim"], (ncfg["img_size"] // ncfg["patch_size"]) ** 2 + 2
        Hd = int(D * ncfg.get("mlp_ratio", 4))
        f_bf16 = (ncfg["depth"] // 2) * 2.0 * rows * L * D * 2 * D
        if precision == "fp8":
            f_bf16 += (ncfg["depth"] + 1) * 2.0 * rows * L * D * Hd
        peak = tot_f / ((tot_f - f_bf16) / PEAK_FP8 + f_bf16 / PEAK_BF16)
        kernel = (f"GEMM family: MXFP8 {FP8_SET[precision]} + bf16 skip_linear"
                  f"{' and fc1' if precision == 'fp8' else ''} (FLOP-weighted fp8/bf16 peak)")
    return {"bound": "mfma", "kernel": kernel,
            "achieved": round(achieved / 1e12, 1), "peak": round(peak / 1e12, 1), "unit": "TFLOP/s",
            "frac": round(achieved / peak, 4), "traffic": traffic,
            "traffic_source": tsrc,
            "measured": "HIP events on the launch stream around each GEMM of the last CFG forward of one eager "
                        "sample of the last step's batch, after the timed region",
            "launches_per_forward": n, "avg_launch_ms": round(tot_t / n * 1e3, 4),
            "flops_per_launch": round(tot_f / n),
            "flops_per_forward": gemm_flops_per_forward(ncfg, rows) if ncfg["name"] == "uvit" else round(tot_f)}


def cpu_model():
    try:
        return [ln for ln in open("/proc/cpuinfo") if ln.startswith("model name")][0].split(":", 1)[1].strip()
    except Exception:
        return "unknown"


def cpu_baseline_t2i(full, ncfg, kw, sd, cores, with_decode):
    """configs[3] on the host: one full 50-NFE panoptic co-generation of B = 2 images through the oracle's
    dpm_solver_pp front end with the t2i CFG closure (train_t2i_discrete.py:387-439, 504-546: cond and uncond as
    two B-row forwards per NFE, mask co-update, enable_mask_opt) + decode; contexts are random (the CLIP encoder,
    0.13 % of the FLOPs, is left out)."""
    from oracle import autoencoder_ref, solver_ref, uvit_ref
    B = 2
    g = torch.Generator().manual_seed(0)
    z = torch.randn(B, *full["z_shape"], generator=g)
    ctx = torch.randn(B, 77, 768, generator=g)
    empty = torch.randn(77, 768, generator=g)
    mt = torch.randn(B, ncfg["num_panoptic_class"], *full["z_shape"][1:], generator=g)

    def nnet(x, t, c, m=None):
        return uvit_ref.uvit_t2i_forward(sd, kw, x, t, c, mask_token=m, enable_panoptic=m is not None)
    with torch.no_grad():
        nnet(z, torch.full((B,), 500.0), ctx, mt)   # warm-up
        fn = solver_ref.cfg_t2i_closure(nnet, ctx, empty, full["cfg_scale"])
        t0 = time.perf_counter()
        lat, _ = solver_ref.pp_sample(fn, solver_ref.sd_betas(), z, steps=full["sample_steps"], mask_token=mt,
                                      enable_mask_opt=True)
        t_sample = time.perf_counter() - t0
        t_dec = 0.0
        if with_decode:
            dsd = weights.decoder_state_dict(seed=1)
            t0 = time.perf_counter()
            autoencoder_ref.decode(dsd, lat)
            t_dec = time.perf_counter() - t0
    assert torch.isfinite(lat).all()
    return {"value": round(B / (t_sample + t_dec), 5), "unit": "images/sec", "cores": cores, "kind": "port",
            "cpu": cpu_model(),
            "sample": f"one full 50-NFE panoptic dpm_solver_pp sample of B={B} (CFG {full['cfg_scale']}: cond + "
                      f"uncond forwards of {B} rows per NFE, mask co-update) = {t_sample:.1f} s, + KL-f8 decode of "
                      f"{B} images = {t_dec:.1f} s; random contexts (CLIP encoder excluded)"}


def cpu_baseline(full, ncfg, with_decode):
    """The reference path timed on the host cores with the fp32 CPU oracle (oracle/uvit_ref.py, solver_ref.py,
    autoencoder_ref.py), SURVEY.md §8d: one FULL 50-NFE sample of B = 2 images through the reference's own
    solver front end and CFG closure (eval_ldm.py:66-108: cond and uncond as two B-row forwards per NFE), then
    the KL-f8 decode of both images.  Threads: the process's CPU affinity, capped by OMP_NUM_THREADS (the GPU
    box sets 16 = this job's CPU share; os.cpu_count() there reports the whole machine)."""
    from oracle import autoencoder_ref, solver_ref, uvit_ref
    cores = len(os.sched_getaffinity(0))
    if os.environ.get("OMP_NUM_THREADS", "").isdigit():
        cores = min(cores, int(os.environ["OMP_NUM_THREADS"]))
    torch.set_num_threads(cores)
    kw = dict(ncfg)
    kw.pop("name")
    sd = weights.nnet_state_dict(ncfg, seed=0, init="reference")
    if ncfg["name"] == "uvit_t2i":
        return cpu_baseline_t2i(full, ncfg, kw, sd, cores, with_decode)
    # configs[0] (CIFAR-10, unconditional, no CFG): BASELINE's batch of 4; the latent configs: 2 images
    B = 4 if ncfg.get("num_classes", -1) <= 0 else 2
    g = torch.Generator().manual_seed(0)
    z = torch.randn(B, *full["z_shape"], generator=g)
    null = ncfg["num_classes"] - 1 if ncfg.get("num_classes", -1) > 0 else None
    y = torch.randint(0, null, (B,), generator=g) if null is not None else None

    def nnet(x, t, yy):
        return uvit_ref.uvit_forward(sd, kw, x, t, yy)
    nfe = [0]

    def counted(fn):
        def f(*a):
            nfe[0] += 1
            return fn(*a)
        return f
    with torch.no_grad():
        nnet(z, torch.full((B,), 500.0), y)   # warm-up (allocator, thread pool)
        if full["front_end"] == "dpm_solver_pytorch":
            model = counted(solver_ref.cfg_class_closure(nnet, y, full["cfg_scale"], null, 999))
            t0 = time.perf_counter()
            lat = solver_ref.pytorch_sample(model, z, steps=full["sample_steps"], eps=full.get("eps", 1e-4))
        else:
            fn = counted(solver_ref.cfg_class_closure(nnet, y, full["cfg_scale"], null, 1000))
            t0 = time.perf_counter()
            lat, _ = solver_ref.pp_sample(lambda x, t, mt: (fn(x, t), None), solver_ref.sd_betas(), z,
                                          steps=full["sample_steps"])
        t_sample = time.perf_counter() - t0
        t_dec = 0.0
        if with_decode:
            dsd = weights.decoder_state_dict(seed=1)
            t0 = time.perf_counter()
            autoencoder_ref.decode(dsd, lat)
            t_dec = time.perf_counter() - t0
    assert torch.isfinite(lat).all()
    return {"value": round(B / (t_sample + t_dec), 5), "unit": "images/sec", "cores": cores, "kind": "port",
            "cpu": cpu_model(),
            "sample": f"one full {nfe[0]}-NFE {full['front_end']} sample of B={B} images ("
                      + (f"CFG {full['cfg_scale']}: cond + uncond forwards of {B} rows per NFE"
                         if full["cfg_scale"] > 0 else f"no guidance: one forward of {B} rows per NFE")
                      + f") = {t_sample:.1f} s"
                      + (f", + KL-f8 decode of {B} images = {t_dec:.1f} s" if with_decode else ", no decode (pixels)")
                      + f"; images/sec = {B} / total"}


if __name__ == "__main__":
    main()
