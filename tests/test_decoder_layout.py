"""Host-logic check of the HIP decoder's data layout (no GPU): the weights exactly as
`libs/autoencoder.py` packs them for `pdm_decoder_*` (3x3 convs -> [Cout][ky][kx][Cin], q/k/v -> one
[3C, C] matrix, conv_out padded to 4 rows) are run through a torch-CPU emulation of the driver sequence in
csrc/decoder.hip (NHWC activations; every GEMM is out = A W^T + b; conv3x3 as the implicit GEMM of
gemm.hip's `conv_row_ptr`: k = (ky*3 + kx)*Cin + ci, zero page for padded taps, nearest-x2 upsample folded
into the source index; GroupNorm over NHWC channel groups; attention as S = Q K^T, row softmax, V^T, P V)
and compared with the oracle decode.  Weights are pre-rounded to bf16 so the packing is exact and the
comparison is fp32 vs fp32 (rel-L2 <= 1e-5)."""
import torch
import torch.nn.functional as F

from oracle import autoencoder_ref
from panopticdiffusionmodels_amd import _lib
from panopticdiffusionmodels_amd import weights as W
from panopticdiffusionmodels_amd.libs.autoencoder import FrozenAutoencoderKL, _DecoderHandle

CH, MULT, NRB = 64, (1, 2), 1


def _param_list(ch, mult, nrb):
    """(name, dtype) in the order pdm_decoder_create registers them (csrc/decoder.hip)."""
    T = ch * mult[-1]
    out = [("post_quant_conv.weight", 0), ("post_quant_conv.bias", 0), ("decoder.conv_in.weight", 0),
           ("decoder.conv_in.bias", 0)]

    def res(p, cin, cout):
        r = [(f"{p}.norm1.weight", 0), (f"{p}.norm1.bias", 0), (f"{p}.conv1.weight", 1), (f"{p}.conv1.bias", 0),
             (f"{p}.norm2.weight", 0), (f"{p}.norm2.bias", 0), (f"{p}.conv2.weight", 1), (f"{p}.conv2.bias", 0)]
        if cin != cout:
            r += [(f"{p}.nin_shortcut.weight", 1), (f"{p}.nin_shortcut.bias", 0)]
        return r
    out += res("decoder.mid.block_1", T, T)
    a = "decoder.mid.attn_1"
    out += [(f"{a}.norm.weight", 0), (f"{a}.norm.bias", 0), (f"{a}.qkv.weight", 1), (f"{a}.qkv.bias", 0),
            (f"{a}.proj_out.weight", 1), (f"{a}.proj_out.bias", 0)]
    out += res("decoder.mid.block_2", T, T)
    cin = T
    for lvl in reversed(range(len(mult))):
        cout = ch * mult[lvl]
        for b in range(nrb + 1):
            out += res(f"decoder.up.{lvl}.block.{b}", cin, cout)
            cin = cout
        if lvl:
            out += [(f"decoder.up.{lvl}.upsample.conv.weight", 1), (f"decoder.up.{lvl}.upsample.conv.bias", 0)]
    out += [("decoder.norm_out.weight", 0), ("decoder.norm_out.bias", 0), ("decoder.conv_out.weight", 1),
            ("decoder.conv_out.bias", 0)]
    return out


def _conv_gemm(a, B, res, cin, w, b, up=0):
    """Implicit GEMM of gemm.hip conv mode: a NHWC [B, res>>up, res>>up, cin] -> [B*res*res, cout]."""
    src = a.reshape(B, res >> up, res >> up, cin)
    if up:
        src = src.repeat_interleave(2, dim=1).repeat_interleave(2, dim=2)
    pad = F.pad(src, (0, 0, 1, 1, 1, 1))                  # zero page for taps outside the grid
    cols = [pad[:, ky:ky + res, kx:kx + res, :] for ky in range(3) for kx in range(3)]
    A = torch.cat(cols, dim=-1).reshape(B * res * res, 9 * cin)   # k = (ky*3 + kx)*cin + ci
    return A @ w.t() + b


def _gn_nhwc(x, B, P, C, gamma, beta, swish):
    g = x.reshape(B, P, 32, C // 32)
    mean = g.mean(dim=(1, 3), keepdim=True)
    var = g.var(dim=(1, 3), unbiased=False, keepdim=True)
    y = ((g - mean) / torch.sqrt(var + 1e-6)).reshape(B, P, C) * gamma + beta
    return y * torch.sigmoid(y) if swish else y


def _emulate(pk, z, ch, mult, nrb, scale):
    """csrc/decoder.hip pdm_decoder_decode, step for step, in fp32 on the packed weights."""
    f = {k: v.float() for k, v in pk.items()}
    B, _, h, _ = z.shape
    T = ch * mult[-1]
    # conv_in_kernel: post_quant folded into the row load, then the 4->T 3x3 conv (fp32, [co][ci][ky][kx])
    zz = z / scale
    q = torch.einsum("oc,bchw->bohw", f["post_quant_conv.weight"].reshape(4, 4), zz) + f["post_quant_conv.bias"].view(1, 4, 1, 1)
    x = F.conv2d(q, f["decoder.conv_in.weight"].reshape(T, 4, 3, 3), f["decoder.conv_in.bias"], padding=1)
    X = x.permute(0, 2, 3, 1).reshape(B, h * h, T)
    res = h

    def resblock(X, res, cin, cout, p):
        P = res * res
        G = _gn_nhwc(X, B, P, cin, f[f"{p}.norm1.weight"], f[f"{p}.norm1.bias"], True)
        H = _conv_gemm(G, B, res, cin, f[f"{p}.conv1.weight"], f[f"{p}.conv1.bias"]).reshape(B, P, cout)
        G = _gn_nhwc(H, B, P, cout, f[f"{p}.norm2.weight"], f[f"{p}.norm2.bias"], True)
        if cin != cout:
            X = (X.reshape(B * P, cin) @ f[f"{p}.nin_shortcut.weight"].t() + f[f"{p}.nin_shortcut.bias"]).reshape(B, P, cout)
        return X + _conv_gemm(G, B, res, cout, f[f"{p}.conv2.weight"], f[f"{p}.conv2.bias"]).reshape(B, P, cout)

    X = resblock(X, res, T, T, "decoder.mid.block_1")
    a = "decoder.mid.attn_1"
    hw = res * res
    G = _gn_nhwc(X, B, hw, T, f[f"{a}.norm.weight"], f[f"{a}.norm.bias"], False)
    QKV = (G.reshape(B * hw, T) @ f[f"{a}.qkv.weight"].t() + f[f"{a}.qkv.bias"]).reshape(B, hw, 3 * T)
    Q, K, V = QKV[..., :T], QKV[..., T:2 * T], QKV[..., 2 * T:]
    S = Q @ K.transpose(1, 2)                                  # batched GEMM, W operand = K rows (ldw = 3C)
    P = torch.softmax(S * T ** -0.5, dim=-1)                   # softmax_rows_kernel
    VT = V.transpose(1, 2)                                     # transpose_kernel -> [B, C, hw]
    O = P @ VT.transpose(1, 2)                                 # batched GEMM with W = V^T rows
    X = X + (O.reshape(B * hw, T) @ f[f"{a}.proj_out.weight"].t() + f[f"{a}.proj_out.bias"]).reshape(B, hw, T)
    X = resblock(X, res, T, T, "decoder.mid.block_2")
    cin = T
    for lvl in reversed(range(len(mult))):
        cout = ch * mult[lvl]
        for b in range(nrb + 1):
            X = resblock(X, res, cin, cout, f"decoder.up.{lvl}.block.{b}")
            cin = cout
        if lvl:
            p = f"decoder.up.{lvl}.upsample.conv"
            X = _conv_gemm(X.reshape(B * res * res, cin), B, res * 2, cin, f[f"{p}.weight"], f[f"{p}.bias"], up=1)
            res *= 2
            X = X.reshape(B, res * res, cin)
    G = _gn_nhwc(X, B, res * res, cin, f["decoder.norm_out.weight"], f["decoder.norm_out.bias"], True)
    O4 = _conv_gemm(G, B, res, cin, f["decoder.conv_out.weight"], f["decoder.conv_out.bias"])   # [B*HW, 4]
    return O4.reshape(B, res, res, 4)[..., :3].permute(0, 3, 1, 2)   # nhwc_to_nchw_kernel


def test_packed_layout_matches_oracle():
    sd = W.make_state_dict(W.decoder_spec(ch=CH, ch_mult=MULT, num_res_blocks=NRB), seed=7, init="random")
    sd = {k: v.bfloat16().float() for k, v in sd.items()}      # bf16-exact weights: packing is lossless
    dd = dict(W.DECODER_DDCONFIG, ch=CH, ch_mult=list(MULT), num_res_blocks=NRB)
    ae = FrozenAutoencoderKL(dd, 4, state_dict=sd, latent_size=8)
    pk = {name: _DecoderHandle._pack(ae, name, dt) for name, dt in _param_list(CH, MULT, NRB)}
    for name, dt in _param_list(CH, MULT, NRB):
        assert pk[name].dtype == (torch.bfloat16 if dt == _lib.PDM_BF16 else torch.float32), name
    g = torch.Generator().manual_seed(2)
    z = torch.randn(2, 4, 8, 8, generator=g)
    got = _emulate(pk, z, CH, MULT, NRB, 0.18215)
    ref = autoencoder_ref.decode(sd, z, ch_mult=MULT, num_res_blocks=NRB)
    rel = float((got - ref).norm() / ref.norm())
    assert rel < 1e-5, rel
