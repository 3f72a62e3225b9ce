"""MXFP8 (OCP e4m3 + E8M0 per 32 elements) GEMM path for BASELINE configs[4] (imagenet512_uvit_huge "fp8 MFMA"):
the block-scaled MFMA GEMM against the same product on the dequantised operands (fp64 reference: only the
fp32 accumulation order differs, rel-L2 <= 5e-5), and the MX-quantising epilogues bit-exact against the host
quantiser (_lib.mx_quantize restates csrc/pdm_common.h mx_quant8)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def rel(a, b):
    a = a.double()
    b = b.double()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


@pytest.fixture(scope="module")
def lib():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from panopticdiffusionmodels_amd import _lib
    _lib.load()
    return _lib


def _mx(lib, x):
    q, s = lib.mx_quantize(x)
    return q, s, lib.mx_dequantize(q, s)


@pytest.mark.parametrize("M,N,K", [(4133, 1152, 1152), (515, 4608, 1152), (300, 1152, 4608), (8192, 256, 128),
                                   (77, 96, 256)])
@pytest.mark.parametrize("epi", ["bf16", "gelu", "f32acc"])
def test_mxfp8_gemm_vs_dequantised(lib, M, N, K, epi):
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    a = torch.randn(M, K, device="cuda", generator=g) * 2
    w = torch.randn(N, K, device="cuda", generator=g) * K ** -0.5
    w[:, :32] *= 50.0   # blocks of very different magnitude
    bias = torch.randn(N, device="cuda", generator=g)
    qa, sa, da = _mx(lib, a)
    qw, sw, dw = _mx(lib, w)
    ref = da.double() @ dw.double().t() + bias.double()
    if epi == "bf16":
        out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        lib.gemm_ex(lib.EPI_BF16, qa, qw, bias, sa, sw, out=out)
        assert rel(out.float(), ref) < 5e-3
    elif epi == "gelu":
        out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        lib.gemm_ex(lib.EPI_GELU, qa, qw, bias, sa, sw, out=out)
        assert rel(out.float(), F.gelu(ref)) < 5e-3
    else:
        r0 = torch.randn(M, N, device="cuda", generator=g)
        out = r0.clone()
        lib.gemm_ex(lib.EPI_F32, qa, qw, bias, sa, sw, out_f32=out, accumulate=True)
        assert rel(out, ref + r0.double()) < 5e-5


@pytest.mark.parametrize("algo", [0, 7])
@pytest.mark.parametrize("epi", ["gelu", "f32acc"])
@pytest.mark.parametrize("M,N,K", [(4133, 1152, 1152), (300, 4608, 256)])
def test_mx_output_epilogue_bit_exact(lib, algo, epi, M, N, K):
    """bf16-operand GEMM whose epilogue also emits the MXFP8 copy (fc1 -> fc2 operand, residual -> qkv / fc1
    operand): e4m3 bytes and E8M0 exponents identical to the host quantiser applied to the stored values."""
    g = torch.Generator(device="cuda").manual_seed(M + N + K + algo)
    a = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    w = (torch.randn(N, K, device="cuda", generator=g) * K ** -0.5).bfloat16()
    bias = torch.randn(N, device="cuda", generator=g)
    q = torch.empty(M, N, device="cuda", dtype=torch.float8_e4m3fn)
    s = torch.zeros(N // 128 if N % 128 == 0 else N // 128 + 1, M, device="cuda", dtype=torch.int32)
    lib.check(lib.load().pdm_set_gemm_algo(algo), "pdm_set_gemm_algo")
    try:
        if epi == "gelu":
            out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            lib.gemm_ex(lib.EPI_GELU, a, w, bias, out=out, out_fp8=q, out_scale=s)
            rq, rs = lib.mx_quantize(out.float())
        else:
            out = torch.randn(M, N, device="cuda", generator=g)
            lib.gemm_ex(lib.EPI_F32, a, w, bias, out_f32=out, accumulate=True, out_fp8=q, out_scale=s)
            rq, rs = lib.mx_quantize(out)
    finally:
        lib.load().pdm_set_gemm_algo(0)
    assert torch.equal(s[: rs.shape[0]], rs)
    assert torch.equal(q.view(torch.uint8), rq.view(torch.uint8))


@pytest.mark.parametrize("algo", [0, 7, 11])
@pytest.mark.parametrize("epi,ln", [("gelu", True), ("gelu", False), ("bf16", False)])
@pytest.mark.parametrize("M,N,K", [(5160, 4608, 1152), (300, 4608, 256), (4133, 1184, 512)])
def test_mx_only_output_bit_exact(lib, algo, epi, ln, M, N, K):
    """bf16-operand GEMM whose only output is the MXFP8 copy (the H/4 bf16 fc1 emitting the fc2 operand, capi.hip
    run_block8): on the persistent kernel (algo 11, the default at these shapes) the fp8 bytes and E8M0 scales
    are computed from registers (permlane reductions over the 4 lane rows of a 32-column block); they must equal
    the host quantiser applied to the bf16 output of the same algo with the same epilogue (LayerNorm consumer +
    GELU included), bit for bit -- and rows / columns past the tile edges stay untouched."""
    g = torch.Generator(device="cuda").manual_seed(M + N + K + algo)
    a = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    w = (torch.randn(N, K, device="cuda", generator=g) * K ** -0.5).bfloat16()
    bias = torch.randn(N, device="cuda", generator=g)
    kw = {}
    if ln:
        _, st = lib.rowstats(a.float() * 1.7 + 0.3, want_bf16=False)
        kw = dict(ln_stats=st, ln_colsum=w.float().sum(1))
    e = lib.EPI_GELU if epi == "gelu" else lib.EPI_BF16
    sn = (N + 127) // 128
    q = torch.full((M, N + 32), 0x7e, device="cuda", dtype=torch.uint8)   # ldo8 = N + 32: the pad stays untouched
    s = torch.full((sn, M + 5), -1, device="cuda", dtype=torch.int32)
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    # the kernel auto-dispatch (algo 0) picks for an MXFP8 output: the persistent one from 4096 rows, else gemm8d;
    # the bf16 reference output comes from that same kernel (the 128 tile's LayerNorm arithmetic differs)
    ref_algo = algo if algo else (11 if M >= 4096 else 7)
    try:
        lib.check(lib.load().pdm_set_gemm_algo(ref_algo), "pdm_set_gemm_algo")
        lib.gemm_ex(e, a, w, bias, out=out, **kw)
        lib.check(lib.load().pdm_set_gemm_algo(algo), "pdm_set_gemm_algo")
        lib.gemm_ex(e, a, w, bias, out_fp8=q[:, :N].view(torch.float8_e4m3fn), out_scale=s, **kw)
    finally:
        lib.load().pdm_set_gemm_algo(0)
    torch.cuda.synchronize()
    rq, rs = lib.mx_quantize(out.float())
    assert torch.equal(q[:, :N], rq.view(torch.uint8))
    assert bool((q[:, N:] == 0x7e).all())
    nb = N // 32   # E8M0 bytes of the valid 32-column blocks ((kt, m) dword byte j = block kt * 4 + j)
    got = s[:, :M].contiguous().view(torch.uint8).reshape(sn, M, 4).permute(1, 0, 2).reshape(M, sn * 4)
    want = rs.contiguous().view(torch.uint8).reshape(sn, M, 4).permute(1, 0, 2).reshape(M, sn * 4)
    assert torch.equal(got[:, :nb], want[:, :nb])
    assert bool((got[:, nb:] == 0xFF).all())   # bytes of blocks past N untouched
    assert bool((s[:, M:] == -1).all())


@pytest.mark.parametrize("M,N,K", [(4133, 1152, 1152), (12900, 3456, 1152), (5000, 256, 512), (4096, 520, 1152)])
@pytest.mark.parametrize("centred", [False, True])
def test_mx_persistent_vs_tile_kernel(lib, M, N, K, centred):
    """The persistent kernel's MXFP8-operand form (gemm8s_kernel FP8 = 1, algo 11; measured slower than the tile
    kernel, so not automatic) against gemm_mx_kernel (algo 7 = auto, one tile per workgroup) on the same operands:
    the same K-ordered chain of scaled MFMAs per accumulator, so the plain bf16 + bias epilogue is bit-identical; with
    the centred LayerNorm consumer (ln_stats + ln_gcol, the correction MFMA) both compute rstd * acc + bias,
    compared at 1e-3.  Ragged M / N tiles (N = 1152: 4.5 column tiles; N = 520: a 256 + 256 + 8 split) included."""
    from panopticdiffusionmodels_amd.native import gcol_table
    g = torch.Generator(device="cuda").manual_seed(M + N + K + int(centred))
    x = torch.randn(M, K, device="cuda", generator=g) * 1.5 + 3.0
    w = torch.randn(N, K, device="cuda", generator=g) * K ** -0.5
    bias = torch.randn(N, device="cuda", generator=g)
    qw, sw, dw = _mx(lib, w)
    kw = {}
    if centred:
        _, st = lib.rowstats(x, want_bf16=False)
        qx, sx = lib.mx_quantize_centred(x, st)
        kw = dict(ln_stats=st, ln_colsum=dw.double().sum(1).float(), ln_gcol=gcol_table(dw))
    else:
        qx, sx, _ = _mx(lib, x)
    outs = {}
    try:
        for algo in (7, 11):
            lib.check(lib.load().pdm_set_gemm_algo(algo), "pdm_set_gemm_algo")
            out = torch.full((M, N + 8), 7.0, device="cuda", dtype=torch.bfloat16)   # ldo = N + 8: pad untouched
            lib.gemm_ex(lib.EPI_BF16, qx, qw, bias, sx, sw, out=out[:, :N], **kw)
            outs[algo] = out
    finally:
        lib.load().pdm_set_gemm_algo(0)
    assert bool((outs[11][:, N:] == 7.0).all())
    a, b = outs[11][:, :N].float(), outs[7][:, :N].float()
    assert torch.isfinite(a).all()
    if centred:
        assert rel(a, b) < 1e-3
    else:
        assert torch.equal(a, b)


@pytest.mark.parametrize("M,N,K", [(25800, 1152, 1152), (16400, 1152, 1152), (4133, 1152, 1152), (20000, 520, 1152)])
def test_mx_persistent_residual_vs_tile_kernel(lib, M, N, K):
    """The MXFP8 residual GEMM (the H/4 proj: bf16 residual in place + LayerNorm partials) on the persistent kernel
    (gemm8s_kernel<EPI_RES, 0, 0, 1>: algo 11, and automatic from 16,384 rows) against gemm_mx_kernel<EPI_RES> (algo 7):
    the output bit-identical ((acc + bias) + residual rounded once in both), the partials within 1e-5 (summation
    order), and against float64 torch.  Ragged M, N = 1152 (a 128-wide last column tile) and N = 520."""
    g = torch.Generator(device="cuda").manual_seed(M + N + K + 5)
    qa, sa, _ = _mx(lib, torch.randn(M, K, device="cuda", generator=g))
    qw, sw, _ = _mx(lib, torch.randn(N, K, device="cuda", generator=g) * K ** -0.5)
    bias = torch.randn(N, device="cuda", generator=g)
    res0 = (torch.randn(M, N, device="cuda", generator=g) * 3 + 2).bfloat16()
    outs = {}
    try:
        for algo in (7, 11, 0):
            lib.check(lib.load().pdm_set_gemm_algo(algo), "pdm_set_gemm_algo")
            out = res0.clone()
            st = torch.full((M, (N + 255) // 256, 2), float("nan"), device="cuda")
            lib.gemm_ex(lib.EPI_RES, qa, qw, bias, sa, sw, out=out, res_in=out, accumulate=True, stats_out=st)
            outs[algo] = (out, st)
    finally:
        lib.load().pdm_set_gemm_algo(0)
    for algo in (11, 0):
        assert torch.equal(outs[algo][0], outs[7][0])
        assert rel(outs[algo][1], outs[7][1]) < 1e-5
    x = outs[11][0].double()
    grp = [x[:, t * 256:(t + 1) * 256] for t in range((N + 255) // 256)]
    ref = torch.stack([torch.stack([c.sum(1), ((c - c.mean(1, keepdim=True)) ** 2).sum(1)], -1) for c in grp], 1)
    assert rel(outs[11][1].double(), ref) < 1e-5


@pytest.mark.parametrize("centred,offset", [(False, 0.0), (True, 0.0), (True, 2.0), (True, 8.0), (True, 32.0)])
def test_mxfp8_layernorm_consumer_chain(lib, centred, offset):
    """fc1 of a U-ViT-H block in fp8: MX(x) operand + gamma-folded MX weight + fused LayerNorm + GELU, emitting
    the MX fc2 operand; vs F.layer_norm -> linear -> GELU in fp32 (fp8 tolerance 6e-2).
    Residual rows x = randn * s + offset * s (+ a per-column pattern): the LayerNorm removes the row mean, so the
    raw-row MX operand loses the signal as |mean| / std grows (host fake-quant: 3.7e-2 / 6.5e-2 / 0.19 / 0.73 at
    offsets 0 / 2 / 8 / 32).  The forward uses the group-centred operand (include/pdm.h pdm_gemm_args.mx_center
    / ln_gcol), whose error does not depend on the offset: <= 6e-2 at every offset."""
    from panopticdiffusionmodels_amd.native import gcol_table
    g = torch.Generator(device="cuda").manual_seed(5)
    M, D, Hd = 2 * 258, 1152, 4608
    sd = 1.5
    x = torch.randn(M, D, device="cuda", generator=g) * sd + offset * sd
    x += 0.3 * sd * torch.randn(1, D, device="cuda", generator=g)   # per-channel structure, so group means differ
    gamma = 1 + 0.2 * torch.randn(D, device="cuda", generator=g)
    beta = 0.1 * torch.randn(D, device="cuda", generator=g)
    w = torch.randn(Hd, D, device="cuda", generator=g) * D ** -0.5
    b = 0.1 * torch.randn(Hd, device="cuda", generator=g)
    ref = F.gelu(F.layer_norm(x, (D,), gamma, beta, eps=1e-5) @ w.t() + b)
    qw, sw, dw = _mx(lib, w * gamma[None])
    colsum = dw.double().sum(1).float()
    bias = (w.double() @ beta.double() + b.double()).float()
    _, st = lib.rowstats(x, want_bf16=False)
    if centred:
        qx, sx = lib.mx_quantize_centred(x, st)
        gcol = gcol_table(dw)
    else:
        qx, sx, _ = _mx(lib, x)
        gcol = None
    out = torch.empty(M, Hd, device="cuda", dtype=torch.bfloat16)
    q = torch.empty(M, Hd, device="cuda", dtype=torch.float8_e4m3fn)
    s = torch.empty(Hd // 128, M, device="cuda", dtype=torch.int32)
    lib.gemm_ex(lib.EPI_GELU, qx, qw, bias, sx, sw, out=out, ln_stats=st, ln_colsum=colsum, out_fp8=q, out_scale=s,
                ln_gcol=gcol)
    err = rel(out.float(), ref)
    print(f"centred={centred} offset={offset}: rel-L2 {err:.3e}")
    assert err < 6e-2, err
    assert rel(lib.mx_dequantize(q, s), ref) < 8e-2


@pytest.mark.parametrize("algo", [0, 7])
def test_mx_centred_producer_bit_exact(lib, algo):
    """Residual epilogue with LayerNorm partials and a group-centred MXFP8 copy (mx_center, the fp8 forward's
    skip_linear / proj / fc2): the e4m3 bytes and exponents equal the host quantiser of (stored row - mu_t), mu_t
    from the partials the same epilogue wrote; rows carry a large offset."""
    g = torch.Generator(device="cuda").manual_seed(17 + algo)
    M, N, K = 1031, 1152, 1152
    a = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    w = (torch.randn(N, K, device="cuda", generator=g) * K ** -0.5).bfloat16()
    bias = torch.randn(N, device="cuda", generator=g)
    out = torch.randn(M, N, device="cuda", generator=g) + 40.0
    st = torch.empty(M, (N + 255) // 256, 2, device="cuda")
    q = torch.empty(M, N, device="cuda", dtype=torch.float8_e4m3fn)
    s = torch.zeros((N + 127) // 128, M, device="cuda", dtype=torch.int32)
    lib.check(lib.load().pdm_set_gemm_algo(algo), "pdm_set_gemm_algo")
    try:
        lib.gemm_ex(lib.EPI_F32, a, w, bias, out_f32=out, accumulate=True, stats_out=st, out_fp8=q, out_scale=s,
                    mx_center=True)
    finally:
        lib.load().pdm_set_gemm_algo(0)
    rq, rs = lib.mx_quantize_centred(out, st)
    assert torch.equal(s[: rs.shape[0]], rs)
    assert torch.equal(q.view(torch.uint8), rq.view(torch.uint8))


def test_mx_center_argument_checks(lib):
    """mx_center without the partials / MXFP8 output it is defined by is rejected with a clear message."""
    a = torch.zeros(256, 256, device="cuda", dtype=torch.bfloat16)
    w = torch.zeros(256, 256, device="cuda", dtype=torch.bfloat16)
    out = torch.zeros(256, 256, device="cuda")
    with pytest.raises(ValueError, match="mx_center"):
        lib.gemm_ex(lib.EPI_F32, a, w, out_f32=out, mx_center=True)   # no stats_out / MXFP8 output


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("R,K", [(1, 32), (17, 96), (77, 1152), (2581, 1152), (300, 4608)])
def test_mx_quantize_kernel_bit_exact(lib, dtype, R, K):
    """pdm_mx_quantize (attention output -> proj operand in the fp8 forward) == the host quantiser, bit for bit,
    including blocks of very different magnitude and all-zero blocks."""
    g = torch.Generator(device="cuda").manual_seed(R + K)
    x = torch.randn(R, K, device="cuda", generator=g) * torch.exp(3 * torch.randn(R, K // 32, 1, device="cuda",
                                                                                  generator=g)).repeat(1, 1, 32).reshape(R, K)
    x[:, :32] = 0
    x = x.to(dtype)
    q, s = lib.mx_quantize_gpu(x)
    rq, rs = lib.mx_quantize(x.float())
    assert torch.equal(s[: rs.shape[0]], rs)
    assert torch.equal(q.view(torch.uint8), rq.view(torch.uint8))


# ---- the MXFP8 U-ViT forward (BASELINE configs[4], imagenet512_uvit_huge) --------------------------------
# Tolerances ("measure first"): e4m3 keeps 3 mantissa bits, so its unit roundoff is 16x
# bf16's.  Fake-quantising the fp32 oracle exactly as the kernels do (tools/fp8_ablation.py):
# all four block Linears in MXFP8 ('fp8-all') 6.9e-2 on the H/4 forward; with mlp.fc1 kept bf16 ('fp8', the
# configs[4] default) 5.0e-2, within §8c's 6e-2.  Final 50-NFE latent vs the bf16 HIP sampler on the same
# weights / inputs (itself pinned to the reference at 1e-2): <= 3e-2.
TOL_FP8_FWD = {"fp8": 6e-2, "fp8-all": 8e-2}
TOL_FP8_FINAL = 3e-2


def _huge(name, seed, init):
    from panopticdiffusionmodels_amd import configs as C
    from panopticdiffusionmodels_amd import weights as W
    from panopticdiffusionmodels_amd.utils import get_nnet
    cfg = C.nnet_kwargs(name)
    sd = W.nnet_state_dict(cfg, seed=seed, init=init)
    net = get_nnet(**cfg)
    net.load_state_dict(sd)
    return net.to("cuda").eval(), sd, cfg


@pytest.mark.parametrize("precision,residual", [("fp8", "bf16"), ("fp8-all", "bf16"), ("fp8", "fp32")])
@pytest.mark.parametrize("name,B", [("imagenet512_uvit_huge", 2), ("imagenet256_uvit_huge", 1)])
def test_fp8_forward_vs_oracle(lib, name, B, precision, residual):
    from oracle import uvit_ref
    from panopticdiffusionmodels_amd import configs as C
    torch.set_num_threads(min(16, torch.get_num_threads()))
    net, sd, cfg = _huge(name, 3, "random")
    kw = dict(cfg)
    kw.pop("name")
    g = torch.Generator().manual_seed(1)
    x = torch.randn(B, *C.get_config(name)["z_shape"], generator=g)
    t = torch.rand(B, generator=g) * 999
    y = torch.randint(0, 1001, (B,), generator=g)
    with torch.no_grad():
        ref = uvit_ref.uvit_forward(sd, kw, x, t, y)
        e16 = net(x.cuda(), t.cuda(), y.cuda()).cpu()
        e8 = net.set_residual(residual).set_precision(precision)(x.cuda(), t.cuda(), y.cuda()).cpu()
    assert torch.isfinite(e8).all()
    err8, err16 = rel(e8, ref), rel(e16, ref)
    print(f"{name}: {precision} (residual {residual}) rel-L2 {err8:.3e}, bf16 {err16:.3e}")
    assert err8 < TOL_FP8_FWD[precision], err8
    assert err16 < 2e-2


def test_fp8_forward_offset_rows(lib):
    """A net whose residual rows carry a per-token offset (pos_embed + 5, ~8x the assembled token std): the
    LayerNorms remove it.  End to end through every centred producer (token-assembly row pass, skip_linear,
    proj, fc2) and consumer (qkv): within the fp8 tolerance of the fp32 oracle (host fake-quant of this net:
    1.35e-2 centred vs 1.68e-2 raw-row; the offset-discriminating case is test_mxfp8_layernorm_consumer_chain)."""
    from oracle import uvit_ref
    from panopticdiffusionmodels_amd import configs as C
    from panopticdiffusionmodels_amd import weights as W
    from panopticdiffusionmodels_amd.utils import get_nnet
    torch.set_num_threads(min(16, torch.get_num_threads()))
    name = "imagenet256_uvit_huge"
    cfg = C.nnet_kwargs(name)
    sd = W.nnet_state_dict(cfg, seed=3, init="random")
    sd["pos_embed"] = sd["pos_embed"] + 5.0
    net = get_nnet(**cfg)
    net.load_state_dict(sd)
    net = net.cuda().eval()
    kw = dict(cfg)
    kw.pop("name")
    g = torch.Generator().manual_seed(1)
    x = torch.randn(1, *C.get_config(name)["z_shape"], generator=g)
    t = torch.rand(1, generator=g) * 999
    y = torch.randint(0, 1001, (1,), generator=g)
    with torch.no_grad():
        ref = uvit_ref.uvit_forward(sd, kw, x, t, y)
        e8 = net.set_precision("fp8")(x.cuda(), t.cuda(), y.cuda()).cpu()
    err = rel(e8, ref)
    print(f"offset rows: fp8 rel-L2 {err:.3e}")
    assert err < TOL_FP8_FWD["fp8"], err


def test_fp8_forward_batch_invariance_and_precision_switch(lib):
    """Row b of a batched fp8 forward == the single-row forward (quantisation is per row / per weight block, so
    nothing leaks across samples); switching back to bf16 rebuilds the bf16 handle."""
    net, _, _ = _huge("imagenet512_uvit_huge", 5, "reference")
    g = torch.Generator().manual_seed(2)
    x = torch.randn(3, 4, 64, 64, generator=g).cuda()
    t = (torch.rand(3, generator=g) * 999).cuda()
    y = torch.tensor([0, 999, 1000]).cuda()
    with torch.no_grad():
        b16 = net(x, t, y)
        net.set_precision("fp8")
        full = net(x, t, y)
        one = torch.cat([net(x[i:i + 1], t[i:i + 1], y[i:i + 1]) for i in range(3)])
        again = net.set_precision("bf16")(x, t, y)
    assert rel(full, one) < 1e-6
    assert torch.equal(again, b16)


def test_fp8_sampler_vs_bf16(lib):
    """configs[4] end to end on the latents: 50-NFE dpm_solver_pp CFG 0.7 sampler with MXFP8 block Linears vs the
    bf16 sampler on the same weights / inputs; graph replay == eager."""
    from panopticdiffusionmodels_amd import configs as C
    from panopticdiffusionmodels_amd.sampler import ClassCondSampler
    net, _, _ = _huge("imagenet512_uvit_huge", 0, "reference")
    full = C.get_config("imagenet512_uvit_huge")
    g = torch.Generator().manual_seed(1234)
    z = torch.randn(2, 4, 64, 64, generator=g).cuda()
    y = torch.randint(0, 1000, (2,), generator=g).cuda()
    mk = lambda graph: ClassCondSampler(net, front_end="dpm_solver_pp", cfg_scale=full["cfg_scale"],  # noqa: E731
                                        null_label=1000, steps=50, use_graph=graph)
    z16 = mk(False).sample(z, y)
    s = mk(True)
    assert torch.equal(s.sample(z, y), z16)   # bf16 graph captured
    net.set_precision(full["precision"])       # frees the packed weights the graph points at ...
    a = s.sample(z, y)                         # ... so the sampler must recapture on the new handle
    b = mk(False).sample(z, y)
    assert torch.isfinite(a).all()
    assert torch.equal(a, b)
    err = rel(a, z16)
    print(f"fp8 vs bf16 final latent rel-L2 {err:.3e}")
    assert err < TOL_FP8_FINAL, err


def test_fp8_lanes_recapture_after_precision_switch(lib):
    """Two concurrent lanes (private workspaces sized for the bf16 handle) keep working after set_precision('fp8')
    rebuilds the handle with a larger workspace: the lanes' workspaces are re-sized and the graphs recaptured; the
    result matches the single-lane fp8 sampler."""
    from panopticdiffusionmodels_amd import configs as C
    from panopticdiffusionmodels_amd.sampler import ClassCondSampler
    net, _, _ = _huge("imagenet512_uvit_huge", 0, "reference")
    full = C.get_config("imagenet512_uvit_huge")
    g = torch.Generator().manual_seed(77)
    z = torch.randn(4, 4, 64, 64, generator=g).cuda()
    y = torch.randint(0, 1000, (4,), generator=g).cuda()
    mk = lambda lanes: ClassCondSampler(net, front_end="dpm_solver_pp", cfg_scale=full["cfg_scale"],  # noqa: E731
                                        null_label=1000, steps=10, lanes=lanes)
    net.set_precision("bf16")
    s2 = mk(2)
    b16 = s2.sample(z, y)
    assert torch.isfinite(b16).all()
    net.set_precision(full["precision"])
    a = s2.sample(z, y)
    b = mk(1).sample(z, y)
    assert torch.isfinite(a).all()
    assert rel(a, b) < 1e-5, rel(a, b)
