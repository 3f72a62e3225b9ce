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


def test_mxfp8_layernorm_consumer_chain(lib):
    """fc1 of a U-ViT-H block in fp8: MX(x) operand + gamma-folded MX weight + fused LayerNorm + GELU, emitting
    the MX fc2 operand; vs F.layer_norm -> linear -> GELU in fp32 (fp8 tolerance 6e-2)."""
    g = torch.Generator(device="cuda").manual_seed(5)
    M, D, Hd = 2 * 258, 1152, 4608
    x = torch.randn(M, D, device="cuda", generator=g) * 1.5
    gamma = 1 + 0.2 * torch.randn(D, device="cuda", generator=g)
    beta = 0.1 * torch.randn(D, device="cuda", generator=g)
    w = torch.randn(Hd, D, device="cuda", generator=g) * D ** -0.5
    b = 0.1 * torch.randn(Hd, device="cuda", generator=g)
    ref = F.gelu(F.layer_norm(x, (D,), gamma, beta, eps=1e-5) @ w.t() + b)
    qx, sx, _ = _mx(lib, x)
    qw, sw, dw = _mx(lib, w * gamma[None])
    colsum = dw.double().sum(1).float()
    bias = (w.double() @ beta.double() + b.double()).float()
    _, st = lib.rowstats(x, want_bf16=False)
    out = torch.empty(M, Hd, device="cuda", dtype=torch.bfloat16)
    q = torch.empty(M, Hd, device="cuda", dtype=torch.float8_e4m3fn)
    s = torch.empty(Hd // 128, M, device="cuda", dtype=torch.int32)
    lib.gemm_ex(lib.EPI_GELU, qx, qw, bias, sx, sw, out=out, ln_stats=st, ln_colsum=colsum, out_fp8=q, out_scale=s)
    assert rel(out.float(), ref) < 6e-2
    assert rel(lib.mx_dequantize(q, s), ref) < 8e-2
