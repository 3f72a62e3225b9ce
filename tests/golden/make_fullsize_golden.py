"""Generate tests/golden/fullsize.npz: the REFERENCE's own outputs at every BASELINE config's full size (build
container only; SURVEY.md §8c "full-size configs").

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_fullsize_golden.py [/root/reference] [--only sample:<config>,...]

`--only` regenerates just the named entries (fwd:<config> / sample:<config>) and merges them into the existing
fullsize.npz (every entry is deterministic, so the others are unchanged by a full run).

Weights and inputs come from this repo's seeded generators (panopticdiffusionmodels_amd.weights,
make_golden._inputs), so only outputs and checksums are stored:
  fwd/<config>/*      one forward of the reference UViT / UViT-t2i at B = 2 (weights init="random", seed 3 -- the
                      nets of tests/test_gpu_configs.py), inputs _inputs(config, 2, seed=5)
  sample/<config>/*   a full 50-NFE CFG sample of one image through the reference solver front end the config
                      names (eval_ldm.py:66-108 for dpm_solver_pytorch, eval_ldm_discrete.py:72-102 for
                      dpm_solver_pp, train_t2i_discrete.py:387-546 for the panoptic t2i), weights init="reference"
                      seed 0 (the bench nets), z_T / labels / contexts from parallel.sample_inputs-style seeds;
                      CIFAR-10 (configs[0]): 4 images, unconditional, no CFG, pixel space, eval.py:47-86
                      (ScoreModel(nnet, 'noise_pred', VPSDE) -> dpm_solver_pytorch model_wrapper, time_input_type '0')
Nothing here is imported by the product or run on the GPU box; the .npz is data.
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import C, W, _import_reference, _inputs, _np, _sd_checksum  # noqa: E402

CONFIGS = ["cifar10_uvit_small", "imagenet256_uvit_large", "imagenet256_uvit_huge", "imagenet512_uvit_huge",
           "mscoco_uvit_small"]
SAMPLE_CONFIGS = ["cifar10_uvit_small", "imagenet256_uvit_large", "imagenet256_uvit_huge", "imagenet512_uvit_huge",
                  "mscoco_uvit_small"]
BETAS = (torch.linspace(0.00085 ** 0.5, 0.0120 ** 0.5, 1000, dtype=torch.float64) ** 2).numpy()


def sample_inputs(name, seed=99):
    """One image's sampling inputs: z_T, label (class-conditional), context / empty context / mask token (t2i).
    configs[0] (CIFAR-10, pixel space, no CFG) samples the BASELINE batch of 4 images."""
    full = C.get_config(name)
    n = full["nnet"]
    g = torch.Generator().manual_seed(seed)
    nb = 4 if name == "cifar10_uvit_small" else 1
    out = {"z": torch.randn(nb, *full["z_shape"], generator=g)}
    if n.get("num_classes", -1) > 0:
        out["y"] = torch.randint(0, n["num_classes"] - 1, (1,), generator=g)
    if n["name"] == "uvit_t2i":
        out["context"] = torch.randn(1, n["num_clip_token"], n["clip_dim"], generator=g)
        out["empty_context"] = torch.randn(n["num_clip_token"], n["clip_dim"], generator=g)
        out["mask_token"] = torch.randn(1, n["num_panoptic_class"], *full["z_shape"][1:], generator=g)
    return out


def _net(mods, name, seed, init):
    uvit, uvit_t2i = mods[0], mods[1]
    cfg = C.nnet_kwargs(name)
    sd = W.nnet_state_dict(cfg, seed=seed, init=init)
    kw = dict(cfg)
    kind = kw.pop("name")
    net = (uvit_t2i if kind == "uvit_t2i" else uvit).UViT(**kw)
    net.load_state_dict(sd)
    return net.eval(), sd


def gen_forward(mods, out, names=CONFIGS):
    for name in names:
        net, sd = _net(mods, name, 3, "random")
        inp = _inputs(name, 2, seed=5)
        with torch.no_grad():
            if "context" in inp:
                eps, pm = net(inp["x"], inp["t"], inp["context"], mask_token=inp["mask_token"])
                out[f"fwd/{name}/pred_mask"] = _np(pm)
            else:
                eps = net(inp["x"], inp["t"], inp.get("y"))
        out[f"fwd/{name}/sd_checksum"] = _sd_checksum(sd)
        out[f"fwd/{name}/in_checksum"] = np.array([float(v.double().sum()) for v in inp.values()])
        out[f"fwd/{name}/eps"] = _np(eps)
        print("fwd", name, tuple(eps.shape), flush=True)


def gen_sample(mods, out, names=SAMPLE_CONFIGS):
    _, _, _, pp, dpt, sde = mods
    for name in names:
        full = C.get_config(name)
        net, sd = _net(mods, name, 0, "reference")
        inp = sample_inputs(name)
        scale = full["cfg_scale"]
        with torch.no_grad():
            if full["nnet"]["name"] == "uvit_t2i":   # train_t2i_discrete.py:387-439, 504-546
                ns = pp.NoiseScheduleVP(schedule="discrete", betas=torch.tensor(BETAS).float())
                ec = inp["empty_context"].unsqueeze(0)

                def model_fn(x, t_continuous, panoptic=None, mask_token=None, use_ground_truth=False,
                             enable_panoptic=False):
                    t = t_continuous * 1000
                    c, pm = net(x, t, context=inp["context"], mask_token=mask_token, mask_0=panoptic,
                                use_ground_truth=use_ground_truth, enable_panoptic=enable_panoptic)
                    u, pmu = net(x, t, context=ec, mask_token=mask_token, mask_0=panoptic,
                                 use_ground_truth=use_ground_truth, enable_panoptic=enable_panoptic)
                    return c + scale * (c - u), pm + scale * (pm - pmu)
                z, pm = pp.DPM_Solver(model_fn, ns, predict_x0=True, thresholding=False).sample(
                    inp["z"].clone(), steps=50, eps=1.0 / 1000, T=1.0, order=3, mask_token=inp["mask_token"].clone(),
                    enable_mask_opt=True, use_ground_truth=False, enable_panoptic=True)
                out[f"sample/{name}/pred_mask"] = _np(pm)
            elif full["front_end"] == "dpm_solver_pp":   # eval_ldm_discrete.py:72-102
                ns = pp.NoiseScheduleVP(schedule="discrete", betas=torch.tensor(BETAS).float())
                null = full["nnet"]["num_classes"] - 1

                def model_fn(x, t_continuous, panoptic=None, mask_token=None, use_ground_truth=False,
                             enable_panoptic=False):
                    t = t_continuous * 1000
                    c = net(x, t, y=inp["y"])
                    u = net(x, t, y=torch.tensor([null] * x.size(0)))
                    return c + scale * (c - u), None
                z, _ = pp.DPM_Solver(model_fn, ns, predict_x0=True, thresholding=False).sample(
                    inp["z"].clone(), steps=50, eps=1.0 / 1000, T=1.0)
            elif not (scale and scale > 0):   # eval.py:47-49, 56-86: unconditional, no CFG, pixel space
                score = sde.ScoreModel(net, pred="noise_pred", sde=sde.VPSDE())
                ns = dpt.NoiseScheduleVP(schedule="linear")
                mf = dpt.model_wrapper(score.noise_pred, ns, time_input_type="0", model_kwargs=dict())
                z = dpt.DPM_Solver(mf, ns).sample(inp["z"].clone(), steps=50, eps=1e-4,
                                                  adaptive_step_size=False, fast_version=True)
            else:   # eval_ldm.py:66-108
                null = full["nnet"]["num_classes"] - 1

                def cfg_nnet(x, timesteps, y):
                    c = net(x, timesteps, y=y)
                    u = net(x, timesteps, y=torch.tensor([null] * x.size(0)))
                    return c + scale * (c - u)
                score = sde.ScoreModel(cfg_nnet, pred="noise_pred", sde=sde.VPSDE())
                ns = dpt.NoiseScheduleVP(schedule="linear")
                mf = dpt.model_wrapper(score.noise_pred, ns, time_input_type="0", model_kwargs=dict(y=inp["y"]))
                z = dpt.DPM_Solver(mf, ns).sample(inp["z"].clone(), steps=50, eps=full.get("eps", 1e-4),
                                                  adaptive_step_size=False, fast_version=True)
        out[f"sample/{name}/sd_checksum"] = _sd_checksum(sd)
        out[f"sample/{name}/z"] = _np(z)
        print("sample", name, tuple(z.shape), flush=True)


def main():
    argv = list(sys.argv[1:])
    only = None
    if "--only" in argv:
        i = argv.index("--only")
        only = argv[i + 1].split(",")
        del argv[i:i + 2]
    ref = argv[0] if argv else "/root/reference"
    mods = _import_reference(ref)
    torch.set_num_threads(8)
    path = os.path.join(HERE, "fullsize.npz")
    if only is None:
        out = {}
        gen_forward(mods, out)
        gen_sample(mods, out)
    else:
        with np.load(path) as f:
            out = {k: f[k] for k in f.files}
        gen_forward(mods, out, [e.split(":", 1)[1] for e in only if e.startswith("fwd:")])
        gen_sample(mods, out, [e.split(":", 1)[1] for e in only if e.startswith("sample:")])
    np.savez_compressed(path, **{k: np.asarray(v) for k, v in out.items()})
    print(f"wrote {path}: {len(out)} arrays, {os.path.getsize(path) / 1e6:.2f} MB")


if __name__ == "__main__":
    main()
