#!/usr/bin/env python3
"""CPU ablation of the MXFP8 forward error (BASELINE configs[4], U-ViT-H/4): the fp32 oracle forward
(oracle/uvit_ref.py, libs/uvit.py:115-120) with the block Linears fake-quantised exactly as the HIP fp8 path
computes them (csrc/capi.hip run_block8):

  qkv, fc1   operand MX(x) of the RAW residual row (optionally centred per 256-column group, --center), weight
             MX(W * gamma), LayerNorm applied to the accumulator: rstd * (acc - mean * colsum) + (W beta + b)
  proj       MX(bf16(attention output)) x MX(W)
  fc2        MX(bf16(GELU(fc1))) x MX(W)
  skip_linear stays bf16 in the product (run_block8); it can be quantised here for the record (--skip8)

Prints the forward rel-L2 vs the unquantised oracle for: all four in MXFP8, each one alone in MXFP8, and
each one kept in bf16 with the other three in MXFP8.  Test infrastructure only (imports oracle/).

  python tools/fp8_ablation.py [--init random|reference] [--seed 3] [--B 2] [--center]
"""
import argparse
import os
import sys

import torch
import torch.nn.functional as F

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from oracle import uvit_ref  # noqa: E402
from panopticdiffusionmodels_amd import _lib, configs, weights  # noqa: E402

LINEARS = ("qkv", "proj", "fc1", "fc2")


def mxr(x):
    """x -> dequantised MXFP8 (the GPU quantiser, _lib.mx_quantize), any leading shape, last dim % 32 == 0."""
    sh = x.shape
    q, s = _lib.mx_quantize(x.reshape(-1, sh[-1]).float())
    return _lib.mx_dequantize(q, s).reshape(sh)


def bf(x):
    return x.bfloat16().float()


def ln_consumer(x, gamma, beta, w, b, fp8, center):
    """LN(x) W^T + b as the fused-LN consumer computes it (native.py _ln_fold, gemm.hip epilogue256)."""
    if not fp8:
        return F.linear(F.layer_norm(x, (x.shape[-1],), gamma, beta, eps=1e-5), w, b)
    D = x.shape[-1]
    xd = x.double()
    mean = xd.mean(-1, keepdim=True)
    rstd = 1.0 / torch.sqrt(xd.var(-1, unbiased=False, keepdim=True) + 1e-5)
    wq = mxr(w * gamma[None]).double()
    bias = w.double() @ beta.double() + (b.double() if b is not None else 0.0)
    if center:
        G = (D + 255) // 256
        xc = xd.clone()
        corr = 0.0
        for g in range(G):
            sl = slice(256 * g, min(D, 256 * (g + 1)))
            gm = xd[..., sl].mean(-1, keepdim=True)
            xc[..., sl] -= gm
            corr = corr + (gm - mean) * wq[:, sl].sum(1)
        acc = mxr(xc.float()).double() @ wq.t() + corr
        return (acc * rstd + bias).float()
    acc = mxr(x).double() @ wq.t()
    return (rstd * (acc - mean * wq.sum(1)) + bias).float()


def block(sd, pre, x, heads, q8, center, skip=None, skip8=False):
    if skip is not None:
        cat = torch.cat([x, skip], -1)
        w = sd[f"{pre}.skip_linear.weight"]
        x = F.linear(mxr(cat) if skip8 else cat, mxr(w) if skip8 else w, sd[f"{pre}.skip_linear.bias"])
    B, L, D = x.shape
    qkv = ln_consumer(x, sd[f"{pre}.norm1.weight"], sd[f"{pre}.norm1.bias"], sd[f"{pre}.attn.qkv.weight"],
                      sd.get(f"{pre}.attn.qkv.bias"), "qkv" in q8, center)
    qkv = qkv.reshape(B, L, 3, heads, D // heads).permute(2, 0, 3, 1, 4)
    s = (qkv[0] @ qkv[1].transpose(-2, -1)) * (D // heads) ** -0.5
    o = (torch.softmax(s, -1) @ qkv[2]).permute(0, 2, 1, 3).reshape(B, L, D)
    w = sd[f"{pre}.attn.proj.weight"]
    if "proj" in q8:
        x = x + F.linear(mxr(bf(o)), mxr(w), sd[f"{pre}.attn.proj.bias"])
    else:
        x = x + F.linear(o, w, sd[f"{pre}.attn.proj.bias"])
    h = F.gelu(ln_consumer(x, sd[f"{pre}.norm2.weight"], sd[f"{pre}.norm2.bias"], sd[f"{pre}.mlp.fc1.weight"],
                           sd[f"{pre}.mlp.fc1.bias"], "fc1" in q8, center))
    w = sd[f"{pre}.mlp.fc2.weight"]
    if "fc2" in q8:
        return x + F.linear(mxr(bf(h)), mxr(w), sd[f"{pre}.mlp.fc2.bias"])
    return x + F.linear(h, w, sd[f"{pre}.mlp.fc2.bias"])


def forward(sd, cfg, x, t, y, q8=(), center=False, skip8=False):
    D, p, C, depth, heads = cfg["embed_dim"], cfg["patch_size"], cfg["in_chans"], cfg["depth"], cfg["num_heads"]
    h = uvit_ref.patch_embed(sd, "patch_embed", x, p)
    tt = uvit_ref.timestep_embedding(t, D).unsqueeze(1)
    h = torch.cat([sd["label_emb.weight"][y].unsqueeze(1), tt, h], 1) + sd["pos_embed"]
    skips = []
    for i in range(depth // 2):
        h = block(sd, f"in_blocks.{i}", h, heads, q8, center)
        skips.append(h)
    h = block(sd, "mid_block", h, heads, q8, center)
    for i in range(depth // 2):
        h = block(sd, f"out_blocks.{i}", h, heads, q8, center, skip=skips.pop(), skip8=skip8)
    h = F.layer_norm(h, (D,), sd["norm.weight"], sd["norm.bias"], eps=1e-5)
    h = F.linear(h, sd["decoder_pred.weight"], sd["decoder_pred.bias"])
    h = uvit_ref.unpatchify(h[:, 2:, :], C)
    if cfg.get("conv", True):
        h = F.conv2d(h, sd["final_layer.weight"], sd["final_layer.bias"], padding=1)
    return h


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="imagenet512_uvit_huge")
    ap.add_argument("--init", default="random")
    ap.add_argument("--seed", type=int, default=3)
    ap.add_argument("--B", type=int, default=2)
    ap.add_argument("--center", action="store_true")
    ap.add_argument("--quick", action="store_true", help="only all-four and the fc1-bf16 mix")
    ap.add_argument("--offset", type=float, default=0.0,
                    help="add this constant to every pos_embed entry: a per-token offset of the residual rows that "
                         "the LayerNorms remove (stress test of the raw-row vs group-centred MXFP8 operand)")
    args = ap.parse_args()
    torch.set_num_threads(min(8, os.cpu_count() or 8))
    cfg = configs.nnet_kwargs(args.config)
    sd = weights.nnet_state_dict(cfg, seed=args.seed, init=args.init)
    sd["pos_embed"] = sd["pos_embed"] + args.offset
    g = torch.Generator().manual_seed(1)   # = tests/test_gpu_fp8.py test_fp8_forward_vs_oracle
    x = torch.randn(args.B, *configs.get_config(args.config)["z_shape"], generator=g)
    t = torch.rand(args.B, generator=g) * 999
    y = torch.randint(0, 1001, (args.B,), generator=g)
    with torch.no_grad():
        ref = forward(sd, cfg, x, t, y)
        r = lambda o: float((o - ref).norm() / ref.norm())  # noqa: E731
        print(f"{args.config} init={args.init} seed={args.seed} B={args.B} center={args.center} offset={args.offset}")
        print(f"  all four MXFP8            : {r(forward(sd, cfg, x, t, y, LINEARS, args.center)):.4e}")
        if args.quick:
            print(f"  fc1   bf16, rest MXFP8  : {r(forward(sd, cfg, x, t, y, ('qkv', 'proj', 'fc2'), args.center)):.4e}")
            return
        for lin in LINEARS:
            print(f"  only {lin:5s} MXFP8         : {r(forward(sd, cfg, x, t, y, (lin,), args.center)):.4e}")
        for lin in LINEARS:
            rest = tuple(v for v in LINEARS if v != lin)
            print(f"  {lin:5s} bf16, rest MXFP8  : {r(forward(sd, cfg, x, t, y, rest, args.center)):.4e}")
        print(f"  all four + skip_linear MXFP8: "
              f"{r(forward(sd, cfg, x, t, y, LINEARS, args.center, skip8=True)):.4e}")


if __name__ == "__main__":
    main()
