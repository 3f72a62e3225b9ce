#!/usr/bin/env python3
"""What a bf16 residual stream would cost the KL-f8 decoder (dev tool, CPU, imports oracle/): the fp32 oracle
decode (oracle/autoencoder_ref.py, libs/autoencoder.py:75-134,376-409) with x rounded to bf16 after every
residual add, nin_shortcut, upsample conv and conv_in -- the roundings a bf16 stream would add -- vs the plain
fp32 oracle.  Measured 1.25e-2 rel-L2 on the full decoder at latent 16 (reference init), against the 2e-2
decoder tolerance, so the HIP decoder keeps its fp32 stream.   python tools/decoder_bf16_residual_sim.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import autoencoder_ref as A  # noqa: E402
from panopticdiffusionmodels_amd import weights as W  # noqa: E402

torch.manual_seed(0)
sd = W.make_state_dict(W.decoder_spec(ch=128, ch_mult=(1, 2, 4, 4), num_res_blocks=2), seed=1, init="reference")
z = torch.randn(1, 4, 16, 16)
ref = A.decode(sd, z)


def rb(x):
    return x.to(torch.bfloat16).float()


orig_attn, orig_conv = A.attn_block, A._conv


def resnet_block(sd, p, x):
    h = A._conv(sd, f"{p}.conv1", A._swish(A._gn(sd, f"{p}.norm1", x)), 1)
    h = A._conv(sd, f"{p}.conv2", A._swish(A._gn(sd, f"{p}.norm2", h)), 1)
    if f"{p}.nin_shortcut.weight" in sd:
        x = rb(A._conv(sd, f"{p}.nin_shortcut", x, 0))
    return rb(x + h)


def conv(sd, p, x, pad):
    y = orig_conv(sd, p, x, pad)
    return rb(y) if (p.endswith("conv_in") or "upsample" in p) else y


A.resnet_block = resnet_block
A.attn_block = lambda sd, p, x: rb(orig_attn(sd, p, x))
A._conv = conv
out = A.decode(sd, z)
print("bf16 residual stream vs fp32: rel-L2 %.3e" % float((out - ref).norm() / ref.norm()))
