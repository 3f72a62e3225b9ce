"""Per-kernel parity on the GPU: every libpdm kernel vs a plain fp32 PyTorch reference of the same op on
the same (bf16-rounded) inputs.  Tolerances: bf16 outputs rel-L2 <= 1e-2 (one rounding of O(1) data),
fp32 outputs from bf16 operands rel-L2 <= 2e-3."""
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


@pytest.mark.parametrize("M,N,K", [(128, 128, 64), (300, 256, 512), (25800 // 8, 1024, 1024), (77, 64, 64),
                                   (1000, 192, 256), (4096, 3456, 1152), (129, 4608, 1152)])
@pytest.mark.parametrize("epi", ["bf16", "gelu", "f32", "f32acc"])
def test_gemm(lib, M, N, K, epi):
    g = torch.Generator(device="cuda").manual_seed(M * 7 + N + K)
    a = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    w = (torch.randn(N, K, device="cuda", generator=g) * K ** -0.5).bfloat16()
    bias = torch.randn(N, device="cuda", generator=g)
    ref = a.float() @ w.float().t() + bias
    if epi == "bf16":
        out = lib.gemm(a, w, bias, lib.EPI_BF16)
        assert rel(out.float(), ref) < 1e-2
    elif epi == "gelu":
        out = lib.gemm(a, w, bias, lib.EPI_GELU)
        assert rel(out.float(), F.gelu(ref)) < 1e-2
    elif epi == "f32":
        out = lib.gemm(a, w, bias, lib.EPI_F32)
        assert rel(out, ref) < 2e-3
    else:
        r0 = torch.randn(M, N, device="cuda", generator=g)
        out = lib.gemm(a, w, bias, lib.EPI_F32, out_f32=r0.clone(), accumulate=True)
        assert rel(out, ref + r0) < 2e-3


@pytest.mark.parametrize("algo", [0, 1, 7, 11])
def test_gelu_activation_exactness(lib, algo):
    """The GELU epilogue alone: A's column 0 carries x, W = e_0, so C = x exactly in fp32 and the output is the
    bf16 rounding of the kernel's GELU(x).  Against exact-erf GELU in fp64: within one bf16 ulp everywhere
    or 2e-5 absolute where GELU ~ 0 (the polynomial's own error is <= 1.8e-5 abs / 9.5e-4 rel,
    csrc/pdm_common.h), exact 0 / x in the tails."""
    M, N, K = 4096, 256, 256   # K >= 256: the persistent kernel (algo 11) applies too
    xs = torch.linspace(-8.0, 8.0, M, device="cuda").bfloat16()
    a = torch.zeros(M, K, device="cuda", dtype=torch.bfloat16)
    a[:, 0] = xs
    w = torch.zeros(N, K, device="cuda", dtype=torch.bfloat16)
    w[:, 0] = 1
    lib.load().pdm_set_gemm_algo(algo)
    try:
        out = lib.gemm(a, w, None, lib.EPI_GELU).double()
    finally:
        lib.load().pdm_set_gemm_algo(0)
    x = xs.double()
    ref = (x * 0.5 * (1 + torch.erf(x / 2 ** 0.5)))[:, None].expand(M, N)
    ulp = torch.exp2(torch.floor(torch.log2(ref.abs().clamp_min(2.0 ** -126))) - 7)
    assert float(((out - ref).abs() / ulp.clamp_min(2e-5)).max()) <= 1.0   # 2e-5 abs where GELU ~ 0
    assert float(out[x[:, None].expand(M, N) <= -4.5].abs().max()) == 0.0
    big = x[:, None].expand(M, N) >= 4.5
    assert torch.equal(out[big], x[:, None].expand(M, N)[big])


def test_gemm_split_k(lib):
    g = torch.Generator(device="cuda").manual_seed(1)
    M, D = 517, 256
    x = torch.randn(M, D, device="cuda", generator=g).bfloat16()
    s = torch.randn(M, D, device="cuda", generator=g).bfloat16()
    w = (torch.randn(D, 2 * D, device="cuda", generator=g) * (2 * D) ** -0.5).bfloat16()
    b = torch.randn(D, device="cuda", generator=g)
    out = lib.gemm(x, w, b, lib.EPI_F32, a2=s)
    ref = torch.cat([x, s], dim=1).float() @ w.float().t() + b
    assert rel(out, ref) < 2e-3


@pytest.mark.parametrize("algo", [1, 2, 3, 4, 5, 6, 7, 8, 9, 11])
@pytest.mark.parametrize("M,N,K", [(4133, 1000, 1024), (515, 768, 2048), (8192, 512, 128), (700, 264, 64),
                                   (1100, 520, 192), (5000, 128, 1152), (700, 120, 64)])
@pytest.mark.parametrize("epi", ["gelu", "f32acc_copy", "split"])
def test_gemm_algos(lib, algo, M, N, K, epi):
    """Every tile policy (1: 128x128, 2/3: 256x256 ring, 4: 256x256 8-phase staggered, 5: 8-phase with the deep
    descriptor-addressed LDS-DMA pipeline, 6/7 its other schedules, 8 / 9: the 256x128 half-N / 512x128 tall
    tiles, which N > 128 sends to the 128 tile) on ragged M/N tails and short / odd K-tile counts."""
    g = torch.Generator(device="cuda").manual_seed(M + N + K + algo)
    a = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    w = (torch.randn(N, K, device="cuda", generator=g) * K ** -0.5).bfloat16()
    bias = torch.randn(N, device="cuda", generator=g)
    ref = a.float() @ w.float().t() + bias
    lib.check(lib.load().pdm_set_gemm_algo(algo), "pdm_set_gemm_algo")
    try:
        if epi == "gelu":
            out = lib.gemm(a, w, bias, lib.EPI_GELU)
            assert rel(out.float(), F.gelu(ref)) < 1e-2
        elif epi == "f32acc_copy":
            r0 = torch.randn(M, N, device="cuda", generator=g)
            cp = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            out = lib.gemm(a, w, bias, lib.EPI_F32, out=cp, out_f32=r0.clone(), accumulate=True)
            assert rel(out, ref + r0) < 2e-3
            assert rel(cp.float(), ref + r0) < 1e-2
        else:
            h = (K // 128) * 64 if K >= 128 else K   # split point on a 64-column boundary; K = 64 runs unsplit
            a2 = a[:, h:].contiguous() if h < K else None
            out = lib.gemm(a[:, :h].contiguous(), w, bias, lib.EPI_F32, a2=a2)
            assert rel(out, ref) < 2e-3
    finally:
        lib.load().pdm_set_gemm_algo(0)


@pytest.mark.parametrize("algo", [1, 3, 4, 5, 6, 7, 8, 9])
@pytest.mark.parametrize("B,h,Cin,N,up,epi", [(2, 16, 64, 128, 0, "f32acc"), (1, 8, 128, 256, 1, "f32"),
                                              (3, 12, 64, 64, 0, "bf16"), (1, 32, 256, 256, 0, "f32"),
                                              (2, 8, 128, 4, 0, "f32"), (2, 24, 256, 128, 1, "bf16"),
                                              (1, 40, 128, 128, 0, "f32acc")])
def test_gemm_conv3x3(lib, algo, B, h, Cin, N, up, epi):
    """Implicit-GEMM conv3x3 mode (decoder ResnetBlock / Upsample convs, libs/autoencoder.py:35-50,110-141) for
    every tile policy: ragged M (B*H*W not a tile multiple), the folded nearest-x2 upsample and the residual
    accumulate, against F.conv2d on the same bf16 operands."""
    g = torch.Generator(device="cuda").manual_seed(B * 100 + h + Cin + N + up + algo)
    x = torch.randn(B, h, h, Cin, device="cuda", generator=g).bfloat16()
    w = (torch.randn(N, Cin, 3, 3, device="cuda", generator=g) * (9 * Cin) ** -0.5).bfloat16()
    bias = torch.randn(N, device="cuda", generator=g)
    xin = x.float().permute(0, 3, 1, 2)
    if up:
        xin = F.interpolate(xin, scale_factor=2.0, mode="nearest")
    ref = F.conv2d(xin, w.float(), bias, padding=1).permute(0, 2, 3, 1).reshape(-1, N)
    lib.check(lib.load().pdm_set_gemm_algo(algo), "pdm_set_gemm_algo")
    try:
        if epi == "bf16":
            out = lib.gemm_conv3x3(x, w, bias, lib.EPI_BF16, up=up)
            assert rel(out.float(), ref) < 1e-2
        elif epi == "f32":
            out = lib.gemm_conv3x3(x, w, bias, lib.EPI_F32, up=up)
            assert rel(out, ref) < 2e-3
        else:
            r0 = torch.randn(ref.shape, device="cuda", generator=g)
            out = lib.gemm_conv3x3(x, w, bias, lib.EPI_F32, up=up, out_f32=r0.clone(), accumulate=True)
            assert rel(out, ref + r0) < 2e-3
    finally:
        lib.load().pdm_set_gemm_algo(0)


def test_gemm_rows_split_past_2gib(lib):
    """Operands past the descriptor kernels' 2 GiB offset range are split into row parts (whole images for a
    conv) by gemm_launch: the split result equals, bit for bit, the same kernel run on the parts' slices."""
    g = torch.Generator(device="cuda").manual_seed(5)
    # conv: 17 images of 256 x 256 x 256 channels nearest-x2 upsampled to 512^2 -> N = 128 (half-N tile),
    # bf16 A1 = 17 * 512^2 * 256 * 2 B > 2 GiB when read at full resolution (no upsample)
    x = torch.randn(17, 512, 512, 256, device="cuda", generator=g).bfloat16()
    w = (torch.randn(128, 256, 3, 3, device="cuda", generator=g) * (9 * 256) ** -0.5).bfloat16()
    bias = torch.randn(128, device="cuda", generator=g)
    full = lib.gemm_conv3x3(x, w, bias, lib.EPI_BF16).view(17, 512 * 512, 128)
    for b in (0, 8, 16):
        part = lib.gemm_conv3x3(x[b:b + 1].contiguous(), w, bias, lib.EPI_BF16).view(512 * 512, 128)
        assert torch.equal(full[b], part)
    del x, full
    # plain GEMM: 1.1 M rows x K = 1024 bf16 (2.25 GB)
    M, K, N = 1100 * 1024, 1024, 256
    a = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    w2 = (torch.randn(N, K, device="cuda", generator=g) * K ** -0.5).bfloat16()
    out = lib.gemm(a, w2, None, lib.EPI_F32)
    for r0 in (0, 550 * 1024, M - 4096):
        ref = lib.gemm(a[r0:r0 + 4096].contiguous(), w2, None, lib.EPI_F32)
        assert torch.equal(out[r0:r0 + 4096], ref)


@pytest.mark.parametrize("algo", [1, 3, 4, 5, 6, 7])
@pytest.mark.parametrize("Z,M,N,K", [(2, 1024, 1024, 512), (3, 300, 260, 128), (1, 4096, 512, 64)])
def test_gemm_batched(lib, algo, Z, M, N, K):
    """Batched operands (decoder AttnBlock q k^T and p v, libs/autoencoder.py:177-188) vs torch.bmm."""
    g = torch.Generator(device="cuda").manual_seed(Z + M + N + K + algo)
    a = torch.randn(Z, M, K, device="cuda", generator=g).bfloat16()
    w = (torch.randn(Z, N, K, device="cuda", generator=g) * K ** -0.5).bfloat16()
    ref = torch.bmm(a.float(), w.float().transpose(1, 2))
    lib.check(lib.load().pdm_set_gemm_algo(algo), "pdm_set_gemm_algo")
    try:
        out = lib.gemm_batched(a, w, None, lib.EPI_F32)
        assert rel(out, ref) < 2e-3
        outb = lib.gemm_batched(a, w, None, lib.EPI_BF16)
        assert rel(outb.float(), ref) < 1e-2
    finally:
        lib.load().pdm_set_gemm_algo(0)


def _ref_partials(y):
    """(sum, M2 about the group mean) per 256-column group of fp32 rows y, float64."""
    y = y.double()
    out = []
    for t in range(0, y.shape[1], 256):
        g = y[:, t:t + 256]
        out.append(torch.stack([g.sum(1), ((g - g.mean(1, keepdim=True)) ** 2).sum(1)], 1))
    return torch.stack(out, 1)


@pytest.mark.parametrize("rows,D", [(1, 64), (517, 1024), (300, 1152), (33, 512), (7, 576)])
def test_rowstats(lib, rows, D):
    g = torch.Generator(device="cuda").manual_seed(rows + D)
    x = torch.randn(rows, D, device="cuda", generator=g) * 3 + 1
    xb, st = lib.rowstats(x)
    assert torch.equal(xb, x.bfloat16())
    ref = _ref_partials(x)
    assert rel(st, ref) < 1e-5


@pytest.mark.parametrize("algo", [1, 3, 4, 5, 6, 7, 11])
@pytest.mark.parametrize("M,N,K,epi", [(4133, 1024, 1024, "bf16"), (515, 4096, 1024, "gelu"), (9000, 3456, 1152, "bf16"),
                                       (700, 520, 512, "gelu")])
def test_gemm_layernorm_consumer(lib, algo, M, N, K, epi):
    """norm -> Linear fused (libs/uvit.py:100,103): bf16(x) operand, gamma-scaled weight, per-row mean / rstd
    merged from the 256-column partials, vs F.layer_norm + linear in fp32.  The mean is large on purpose (|mean|
    ~ 2 std) so the mean-correction term is exercised."""
    g = torch.Generator(device="cuda").manual_seed(M + N + K + algo)
    x = torch.randn(M, K, device="cuda", generator=g) * 1.5 + 3.0 * torch.randn(M, 1, device="cuda", generator=g)
    gamma = 1.0 + 0.3 * torch.randn(K, device="cuda", generator=g)
    beta = 0.2 * torch.randn(K, device="cuda", generator=g)
    w = torch.randn(N, K, device="cuda", generator=g) * K ** -0.5
    b = 0.1 * torch.randn(N, device="cuda", generator=g)
    ref = F.layer_norm(x, (K,), gamma, beta, eps=1e-5) @ w.t() + b
    if epi == "gelu":
        ref = F.gelu(ref)
    wg = (w * gamma[None]).bfloat16()
    colsum = wg.double().sum(1).float()
    bias = (w.double() @ beta.double() + b.double()).float()
    xb, st = lib.rowstats(x)
    lib.check(lib.load().pdm_set_gemm_algo(algo), "pdm_set_gemm_algo")
    try:
        out = lib.gemm_ln(xb, wg, bias, lib.EPI_GELU if epi == "gelu" else lib.EPI_BF16, ln_stats=st, ln_colsum=colsum)
    finally:
        lib.load().pdm_set_gemm_algo(0)
    assert rel(out.float(), ref) < 1.5e-2


@pytest.mark.parametrize("algo", [1, 3, 4, 5, 6, 7])
@pytest.mark.parametrize("M,N,K", [(4133, 1024, 1024), (515, 1152, 2048), (8192, 512, 256)])
def test_gemm_layernorm_producer(lib, algo, M, N, K):
    """Residual epilogue emitting the LayerNorm partials of the stored fp32 rows (+ the bf16 copy)."""
    g = torch.Generator(device="cuda").manual_seed(M + N + K + algo + 1)
    a = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    w = (torch.randn(N, K, device="cuda", generator=g) * K ** -0.5).bfloat16()
    bias = torch.randn(N, device="cuda", generator=g)
    r0 = torch.randn(M, N, device="cuda", generator=g) + 2.0
    cp = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    lib.check(lib.load().pdm_set_gemm_algo(algo), "pdm_set_gemm_algo")
    try:
        out, st = lib.gemm_ln(a, w, bias, lib.EPI_F32, out=cp, out_f32=r0.clone(), accumulate=True, stats_out=True)
    finally:
        lib.load().pdm_set_gemm_algo(0)
    assert rel(out, a.float() @ w.float().t() + bias + r0) < 2e-3
    assert torch.equal(cp, out.bfloat16())
    assert rel(st, _ref_partials(out)) < 1e-5


@pytest.mark.parametrize("algo", [0, 1, 7, 11])
@pytest.mark.parametrize("M,N,K,mode", [(4133, 1024, 1024, "inplace"), (515, 1152, 2048, "outofplace"),
                                        (8192, 512, 256, "noacc"), (300, 264, 64, "inplace")])
def test_gemm_residual_bf16(lib, algo, M, N, K, mode):
    """Residual epilogue on the bf16 residual stream (EPI_RES, include/pdm.h pdm_gemm_args.res_in): out =
    bf16(A W^T + bias + res) in place or out of place, and the LayerNorm partials of the rounded rows; vs an fp32
    torch reference (one bf16 rounding of the sum)."""
    g = torch.Generator(device="cuda").manual_seed(M + N + K + algo + 7)
    a = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    w = (torch.randn(N, K, device="cuda", generator=g) * K ** -0.5).bfloat16()
    bias = torch.randn(N, device="cuda", generator=g)
    res = (torch.randn(M, N, device="cuda", generator=g) * 3 + 2.0).bfloat16()
    ref = a.float() @ w.float().t() + bias + (res.float() if mode != "noacc" else 0)
    out = res.clone() if mode == "inplace" else torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    st = torch.empty(M, (N + 255) // 256, 2, device="cuda")
    lib.check(lib.load().pdm_set_gemm_algo(algo), "pdm_set_gemm_algo")
    try:
        lib.gemm_ex(lib.EPI_RES, a, w, bias, out=out, res_in=None if mode == "noacc" else (out if mode == "inplace" else res),
                    accumulate=mode != "noacc", stats_out=st)
    finally:
        lib.load().pdm_set_gemm_algo(0)
    assert rel(out.float(), ref) < 4e-3           # one bf16 rounding (2^-9) of the fp32 sum
    assert rel(st, _ref_partials(out.float())) < 1e-5


@pytest.mark.parametrize("algo", [0, 1, 3, 7])
@pytest.mark.parametrize("M,N,K", [(4133, 1024, 1024), (515, 1152, 2048), (300, 264, 64)])
def test_gemm_residual_f32_out_of_place(lib, algo, M, N, K):
    """fp32 residual read from res_f32 (include/pdm.h pdm_gemm_args.res_f32): out_f32 = res + A W^T + bias, the
    residual untouched, the optional bf16 copy of the sum; vs fp32 torch (the training forward's x1 = x0 + proj)."""
    g = torch.Generator(device="cuda").manual_seed(M + N + K + algo + 11)
    a = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    w = (torch.randn(N, K, device="cuda", generator=g) * K ** -0.5).bfloat16()
    bias = torch.randn(N, device="cuda", generator=g)
    res = torch.randn(M, N, device="cuda", generator=g) * 3 + 2.0
    res0 = res.clone()
    out = torch.full((M, N), float("nan"), device="cuda")
    cp = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    lib.check(lib.load().pdm_set_gemm_algo(algo), "pdm_set_gemm_algo")
    try:
        lib.gemm_ex(lib.EPI_F32, a, w, bias, out=cp, out_f32=out, accumulate=True, res_f32=res)
    finally:
        lib.load().pdm_set_gemm_algo(0)
    ref = a.float() @ w.float().t() + bias + res0
    assert torch.equal(res, res0)
    assert rel(out, ref) < 2e-3
    assert torch.equal(cp, out.bfloat16())


@pytest.mark.parametrize("M,N,K,kind", [(25800, 3072, 1024, "ln"), (25800, 4096, 1024, "ln_gelu"),
                                        (12937, 1024, 1024, "res"), (25800, 1024, 4096, "res"), (12900, 1024, 2048, "skip"),
                                        (9137, 1152, 1152, "res"), (9137, 3456, 1152, "ln"), (6000, 4608, 1152, "ln_gelu"),
                                        (70000, 512, 256, "res"), (5000, 1152, 256, "bf16"), (300, 264, 512, "res")])
def test_gemm_persistent(lib, M, N, K, kind):
    """The persistent 256-tile kernel (algo 11, several tiles per workgroup, the LDS-DMA ring running across tile
    boundaries, permlane-swapped 16-byte stores, in-register residual epilogue) against the per-tile kernel (algo 7):
    the same MFMA chain, so the outputs are bit-identical (the LayerNorm-consumer epilogue to fp32 rounding: it applies
    rstd * (acc - mean * colsum) + bias as acc * rstd + (bias - mean * rstd * colsum), so a few bf16 roundings flip);
    its LayerNorm partials (per-wave partials merged with Chan's update) against float64 torch.  Ragged M, N % 256 != 0 (the 128-wide last column tile), split-K, D = 1152 (5 partials
    per row), K = 256 (4 K-tiles: the shortest the kernel takes)."""
    g = torch.Generator(device="cuda").manual_seed(M + N + K + 3)
    Ka = K // 2 if kind == "skip" else K
    a = torch.randn(M, Ka, device="cuda", generator=g).bfloat16()
    a2 = torch.randn(M, K - Ka, device="cuda", generator=g).bfloat16() if kind == "skip" else None
    w = (torch.randn(N, K, device="cuda", generator=g) * K ** -0.5).bfloat16()
    bias = torch.randn(N, device="cuda", generator=g)
    outs = {}
    for algo in (7, 11):
        lib.check(lib.load().pdm_set_gemm_algo(algo), "pdm_set_gemm_algo")
        try:
            if kind in ("ln", "ln_gelu"):
                x = torch.randn(M, K, device="cuda", generator=torch.Generator(device="cuda").manual_seed(9)) * 1.5 + 2.0
                xb, st = lib.rowstats(x)
                colsum = w.double().sum(1).float()
                outs[algo] = (lib.gemm_ln(xb, w, bias, lib.EPI_GELU if kind == "ln_gelu" else lib.EPI_BF16, ln_stats=st,
                                          ln_colsum=colsum),)
            elif kind == "bf16":
                outs[algo] = (lib.gemm(a, w, bias, lib.EPI_BF16),)
            else:
                res = (torch.randn(M, N, device="cuda", generator=torch.Generator(device="cuda").manual_seed(4)) * 3 +
                       2.0).bfloat16()
                out = res.clone()
                st = torch.full((M, (N + 255) // 256, 2), float("nan"), device="cuda")
                lib.gemm_ex(lib.EPI_RES, a, w, bias, out=out, res_in=out, accumulate=True, stats_out=st, a2=a2)
                outs[algo] = (out, st)
        finally:
            lib.load().pdm_set_gemm_algo(0)
    if kind in ("ln", "ln_gelu"):
        d = (outs[7][0].float() - outs[11][0].float()).abs()
        assert rel(outs[11][0].float(), outs[7][0].float()) < 1e-3 and float((d > 0).float().mean()) < 2e-2
    else:
        assert torch.equal(outs[7][0], outs[11][0])
    if kind in ("res", "skip"):
        assert rel(outs[11][1], _ref_partials(outs[11][0].float())) < 1e-5
        assert rel(outs[7][1], outs[11][1]) < 1e-5


def test_gemm_bad_shape(lib):
    a = torch.zeros(16, 100, device="cuda", dtype=torch.bfloat16)
    w = torch.zeros(128, 100, device="cuda", dtype=torch.bfloat16)
    with pytest.raises(ValueError):
        lib.gemm(a, w)


@pytest.mark.parametrize("rows,D", [(1, 64), (258, 1024), (1000, 1152), (33, 512), (7, 576)])
def test_layernorm(lib, rows, D):
    g = torch.Generator(device="cuda").manual_seed(rows + D)
    x = torch.randn(rows, D, device="cuda", generator=g) * 3 + 1
    gm = torch.randn(D, device="cuda", generator=g)
    bt = torch.randn(D, device="cuda", generator=g)
    y = lib.layernorm(x, gm, bt)
    ref = F.layer_norm(x, (D,), gm, bt, eps=1e-5)
    assert rel(y.float(), ref) < 1e-2


@pytest.mark.parametrize("L", [66, 257, 258, 334, 590])
@pytest.mark.parametrize("Dh", [32, 64, 72])
@pytest.mark.parametrize("q_log2", [False, True])
def test_attention(lib, L, Dh, q_log2):
    """q_log2: q pre-scaled by Dh^-0.5 log2(e) as the U-ViT forward's qkv GEMM writes it (pdm_attention_log2)."""
    H, B = 3, 2
    D = H * Dh
    g = torch.Generator(device="cuda").manual_seed(L * 10 + Dh)
    qkv = (torch.randn(B * L, 3 * D, device="cuda", generator=g) * 1.5).bfloat16()
    q, k, v = qkv.float().reshape(B, L, 3, H, Dh).permute(2, 0, 3, 1, 4)
    if q_log2:
        sq = qkv.clone()
        sq[:, :D] = (qkv[:, :D].float() * (Dh ** -0.5 * 1.4426950408889634)).bfloat16()
        out = lib.attention(sq, B, L, H, Dh, q_log2=True)
        q = sq[:, :D].float().reshape(B, L, H, Dh).permute(0, 2, 1, 3) / (Dh ** -0.5 * 1.4426950408889634)
    else:
        out = lib.attention(qkv, B, L, H, Dh)
    ref = torch.softmax(q @ k.transpose(-1, -2) * Dh ** -0.5, dim=-1) @ v
    ref = ref.permute(0, 2, 1, 3).reshape(B * L, D)
    assert rel(out.float(), ref) < 1e-2


@pytest.mark.parametrize("algo", [1, 2, 3, 4, 11])
@pytest.mark.parametrize("L", [17, 32, 64, 66, 128, 129, 257, 258, 334, 513, 590])
@pytest.mark.parametrize("ramp", [False, True])
def test_attention_algos(lib, algo, L, ramp):
    """Both attention structures (1: streamed K/V per 64-query block; 2/3: head-resident K/V, 2 or 3 query
    tiles per wave; 4: head-resident v2, a ragged last tile at nqt = k NW + 1 (L = 66, 129, 257, 258, 513) run as the
    third tile of a pass; 11: the persistent v3 streaming the next head's K/V, falling back to v2 below NW tiles) at
    Dh = 64 on ragged lengths and whole 64-key blocks (the head-resident path declines shapes
    it cannot hold).  ramp: key magnitudes
    grow along the sequence, so later key blocks raise the running max past the deferred-rescale threshold."""
    H, B, Dh = 4, 3, 64
    D = H * Dh
    g = torch.Generator(device="cuda").manual_seed(L + algo)
    qkv = torch.randn(B * L, 3 * D, device="cuda", generator=g) * 1.5
    if ramp:
        pos = torch.arange(B * L, device="cuda") % L
        qkv[:, D:2 * D] *= (1 + 5 * pos / L)[:, None]
    qkv = qkv.bfloat16()
    lib.check(lib.load().pdm_set_attention_algo(algo), "pdm_set_attention_algo")
    try:
        out = lib.attention(qkv, B, L, H, Dh)
    finally:
        lib.load().pdm_set_attention_algo(0)
    q, k, v = qkv.float().reshape(B, L, 3, H, Dh).permute(2, 0, 3, 1, 4)
    ref = torch.softmax(q @ k.transpose(-1, -2) * Dh ** -0.5, dim=-1) @ v
    ref = ref.permute(0, 2, 1, 3).reshape(B * L, D)
    assert rel(out.float(), ref) < 1e-2


@pytest.mark.parametrize("B,L,H", [(100, 258, 16), (50, 258, 16), (190, 258, 16), (7, 66, 100), (130, 66, 4),
                                   (32, 334, 8), (32, 590, 8), (41, 128, 16), (64, 256, 16)])
def test_attention_persistent_v3(lib, B, L, H):
    """The persistent v3 kernel (algo 11: workgroups loop over heads and stream the next head's K/V into LDS during
    their last pass) at the bench shapes, where every workgroup runs several heads (B*H > 2 x CUs), against fp32
    torch and BIT-identical to the one-head-per-workgroup v2 (algo 4): a query tile's MFMA / exp chain does not
    depend on the pass it runs in.  (7, 66, 100) and (130, 66, 4): one pass per head, so the first pass's per-block
    waits and the release of each block for the next head run in the same pass."""
    Dh = 64
    D = H * Dh
    g = torch.Generator(device="cuda").manual_seed(B * L + H)
    qkv = torch.randn(B * L, 3 * D, device="cuda", generator=g) * 1.5
    pos = torch.arange(B * L, device="cuda") % L
    qkv[:, D:2 * D] *= (1 + 3 * pos / L)[:, None]   # later keys raise the running max (rescale branch)
    qkv = qkv.bfloat16()
    outs = {}
    for algo in (4, 11):
        lib.check(lib.load().pdm_set_attention_algo(algo), "pdm_set_attention_algo")
        try:
            outs[algo] = lib.attention(qkv, B, L, H, Dh)
            torch.cuda.synchronize()
        finally:
            lib.load().pdm_set_attention_algo(0)
    assert torch.equal(outs[11], outs[4])
    q, k, v = qkv.float().reshape(B, L, 3, H, Dh).permute(2, 0, 3, 1, 4)
    ref = torch.nn.functional.scaled_dot_product_attention(q, k, v)
    ref = ref.permute(0, 2, 1, 3).reshape(B * L, D)
    assert rel(outs[11].float(), ref) < 1e-2


@pytest.mark.parametrize("B,L", [(100, 258), (50, 258), (7, 66), (33, 130), (40, 257)])
def test_attention_h72_persistent(lib, B, L):
    """The persistent Dh = 72 kernel (algo 14) at the U-ViT-H head count with several heads per workgroup: fp32 torch
    within 1e-2 and BIT-identical to the one-head-per-workgroup kernel (algo 7)."""
    H, Dh = 16, 72
    D = H * Dh
    g = torch.Generator(device="cuda").manual_seed(B * L + 72)
    qkv = torch.randn(B * L, 3 * D, device="cuda", generator=g) * 1.5
    pos = torch.arange(B * L, device="cuda") % L
    qkv[:, D:2 * D] *= (1 + 3 * pos / L)[:, None]
    qkv = qkv.bfloat16()
    outs = {}
    for algo in (7, 14):
        lib.check(lib.load().pdm_set_attention_algo(algo), "pdm_set_attention_algo")
        try:
            outs[algo] = lib.attention(qkv, B, L, H, Dh)
            torch.cuda.synchronize()
        finally:
            lib.load().pdm_set_attention_algo(0)
    assert torch.equal(outs[14], outs[7])
    q, k, v = qkv.float().reshape(B, L, 3, H, Dh).permute(2, 0, 3, 1, 4)
    ref = torch.nn.functional.scaled_dot_product_attention(q, k, v).permute(0, 2, 1, 3).reshape(B * L, D)
    assert rel(outs[14].float(), ref) < 1e-2


@pytest.mark.parametrize("L", [33, 66, 129, 257, 258, 280])
def test_attention_h72(lib, L):
    """Head-resident Dh = 72 kernel (64 + 8 head-dim split, unpadded 144-B K/V rows; U-ViT-H/2, H/4) at the H
    head count on ragged lengths, with a dominant key row forcing the deferred-rescale branch."""
    H, B, Dh = 16, 3, 72
    D = H * Dh
    g = torch.Generator(device="cuda").manual_seed(L + 72)
    qkv = torch.randn(B * L, 3 * D, device="cuda", generator=g) * 1.5
    qkv[L - 1, D:2 * D] *= 6.0   # the last key of sequence 0 dominates (ragged block)
    qkv = qkv.bfloat16()
    lib.check(lib.load().pdm_set_attention_algo(7), "pdm_set_attention_algo")
    try:
        out = lib.attention(qkv, B, L, H, Dh)
    finally:
        lib.load().pdm_set_attention_algo(0)
    q, k, v = qkv.float().reshape(B, L, 3, H, Dh).permute(2, 0, 3, 1, 4)
    ref = torch.softmax(q @ k.transpose(-1, -2) * Dh ** -0.5, dim=-1) @ v
    ref = ref.permute(0, 2, 1, 3).reshape(B * L, D)
    assert torch.isfinite(out.float()).all()
    assert rel(out.float(), ref) < 1e-2


def test_attention_spiky(lib):
    """A key row far above the rest forces a late running-max jump (online-softmax rescale branch)."""
    B, L, H, Dh = 1, 258, 2, 64
    D = H * Dh
    g = torch.Generator(device="cuda").manual_seed(0)
    qkv = torch.randn(B * L, 3 * D, device="cuda", generator=g)
    qkv[200, D:2 * D] *= 8.0   # key 200 (third chunk) dominates
    qkv = qkv.bfloat16()
    out = lib.attention(qkv, B, L, H, Dh)
    q, k, v = qkv.float().reshape(B, L, 3, H, Dh).permute(2, 0, 3, 1, 4)
    ref = (torch.softmax(q @ k.transpose(-1, -2) * Dh ** -0.5, dim=-1) @ v).permute(0, 2, 1, 3).reshape(B * L, D)
    assert rel(out.float(), ref) < 1e-2


def test_stage_epilogue(lib):
    g = torch.Generator(device="cuda").manual_seed(3)
    B, C, H, W = 3, 4, 8, 8
    pre = torch.randn(2 * B, C, H, W, device="cuda", generator=g)
    w = torch.randn(C, C, 3, 3, device="cuda", generator=g) * 0.2
    b = torch.randn(C, device="cuda", generator=g)
    xin = torch.randn(B, C, H, W, device="cuda", generator=g)
    T0 = torch.randn(B, C, H, W, device="cuda", generator=g)
    T1 = torch.randn(B, C, H, W, device="cuda", generator=g)
    m = torch.empty_like(xin)
    xo = torch.empty_like(xin)
    lib.stage_epilogue(pre, B, conv_w=w, conv_b=b, cfg_scale=0.4, xin=xin, ax=1.7, ae=-0.3, m_out=m,
                       terms=[T0, T1], coeffs=[0.5, -2.0], cm=0.25, x_out=xo)
    c = F.conv2d(pre[:B], w, b, padding=1)
    u = F.conv2d(pre[B:], w, b, padding=1)
    e = c + 0.4 * (c - u)
    mr = 1.7 * xin - 0.3 * e
    assert rel(m, mr) < 1e-5
    assert rel(xo, 0.5 * T0 - 2.0 * T1 + 0.25 * mr) < 1e-5
    # tanh per call before the combine (mask head)
    lib.stage_epilogue(pre, B, conv_w=w, conv_b=b, cfg_scale=1.0, act_tanh=True, m_out=m)
    mt = torch.tanh(c) + 1.0 * (torch.tanh(c) - torch.tanh(u))
    assert rel(m, mt) < 1e-5


def test_lincomb(lib):
    g = torch.Generator(device="cuda").manual_seed(4)
    ts = [torch.randn(5, 4, 7, 9, device="cuda", generator=g) for _ in range(4)]
    out = lib.lincomb(ts, [1.0, -0.5, 0.25, 3.0])
    assert rel(out, ts[0] - 0.5 * ts[1] + 0.25 * ts[2] + 3 * ts[3]) < 1e-6


@pytest.mark.parametrize("case", ["qkv_ln", "fc1_ln_gelu", "proj_res", "fc2_res", "fc2_res_inplace", "skip_split",
                                  "mixed_n"])
def test_gemm_pair_grouped_vs_separate(lib, case):
    """pdm_gemm_pair (one grouped persistent launch over the t2i image- and mask-stream Linears of a layer, csrc
    capi.hip run_block16_pair) against the same two GEMMs launched alone: bit-identical outputs and partials (each
    tile runs the same arithmetic in either launch).  Rows of the two problems as at the t2i bench (32 rows x 334 /
    590 tokens), D = 512; 'mixed_n' cannot be grouped (different N) and takes the two-launch path.  The residual
    cases accumulate res_in (as the forward's res_args); 'fc2_res_inplace' reads the residual from the output
    itself (res_in == out, the image block's fc2 adding into XT2)."""
    D, Hd = 512, 2048
    Ma, Mb = 32 * 334, 32 * 590
    g = torch.Generator(device="cuda").manual_seed(hash(case) % 1000)
    N, K, epi = {"qkv_ln": (3 * D, D, lib.EPI_BF16), "fc1_ln_gelu": (Hd, D, lib.EPI_GELU), "proj_res": (D, D, lib.EPI_RES),
                 "fc2_res": (D, Hd, lib.EPI_RES), "fc2_res_inplace": (D, Hd, lib.EPI_RES),
                 "skip_split": (D, 2 * D, lib.EPI_RES), "mixed_n": (3 * D, D, lib.EPI_BF16)}[case]

    def problem(M, n):
        kk = K // 2 if case == "skip_split" else K
        a = torch.randn(M, kk, device="cuda", generator=g).bfloat16()
        w = (torch.randn(n, K, device="cuda", generator=g) * K ** -0.5).bfloat16()
        kw = dict(a=a, w=w, bias=torch.randn(n, device="cuda", generator=g),
                  out=torch.empty(M, n, device="cuda", dtype=torch.bfloat16))
        if case == "skip_split":
            kw["a2"] = torch.randn(M, kk, device="cuda", generator=g).bfloat16()
        if epi == lib.EPI_RES:
            if case == "fc2_res_inplace":
                kw["out"] = torch.randn(M, n, device="cuda", generator=g).bfloat16()
                kw["res_in"] = kw["out"]
            else:
                kw["res_in"] = torch.randn(M, n, device="cuda", generator=g).bfloat16()
            kw["accumulate"] = True
            kw["stats_out"] = torch.empty(M, (n + 255) // 256, 2, device="cuda")
        else:
            _, st = lib.rowstats(torch.randn(M, K, device="cuda", generator=g) * 1.3 + 0.2, want_bf16=False)
            kw["ln_stats"], kw["ln_colsum"] = st, w.float().sum(1)
        return kw

    pa = problem(Mb, N)
    pb = problem(Ma, D if case == "mixed_n" else N)
    init = [kw["out"].clone() for kw in (pa, pb)]
    ref = []
    for kw in (pa, pb):
        lib.gemm_ex(epi, **kw)
        ref.append({k: kw[k].clone() for k in ("out", "stats_out") if k in kw})
    for kw, o in zip((pa, pb), init):
        if case == "fc2_res_inplace":
            kw["out"].copy_(o)     # the residual it reads
        else:
            kw["out"].fill_(7.0)
        if "stats_out" in kw:
            kw["stats_out"].fill_(7.0)
    lib.gemm_pair(epi, pa, pb)
    torch.cuda.synchronize()
    for kw, r in zip((pa, pb), ref):
        for k, v in r.items():
            assert torch.equal(kw[k], v), (case, k)
    if epi == lib.EPI_RES:   # the residual really entered the sum (fp32 torch on the same bf16 operands)
        for kw, o in zip((pa, pb), init):
            a = torch.cat([kw["a"], kw["a2"]], 1) if "a2" in kw else kw["a"]
            res = o if case == "fc2_res_inplace" else kw["res_in"]
            want = a.float() @ kw["w"].float().t() + kw["bias"] + res.float()
            assert rel(kw["out"].float(), want) < 1e-2, case


@pytest.mark.parametrize("G,Lx,Lm,algo", [(32, 334, 590, 0), (16, 334, 590, 0), (5, 70, 100, 0), (32, 334, 590, 1),
                                          (3, 257, 300, 0)])
def test_gemm_gather_second_output(lib, G, Lx, Lm, algo):
    """The t2i injection GEMM (capi.hip t2i_two_stream16 inject): A rows gathered from the image rows of the mask
    stream (row m -> (m // Lx) * Lm + m % Lx), EPI_RES with partials, and the second output writing the rounded rows
    and their partials into the image rows of the next mask-stream input.  The product and partials are
    BIT-identical to the same GEMM on a contiguous copy of the gathered rows; out2 / stats_out2 hold exactly out /
    stats_out at the scattered rows and leave the mask rows untouched.  algo 1: the 128 tile (its out2 is a row
    copy after the launch)."""
    D = 512
    g = torch.Generator(device="cuda").manual_seed(G * Lx + Lm)
    src = torch.randn(G * Lm, D, device="cuda", generator=g).bfloat16()
    w = (torch.randn(D, D, device="cuda", generator=g) * D ** -0.5).bfloat16()
    bias = torch.randn(D, device="cuda", generator=g)
    res = torch.randn(G * Lx, D, device="cuda", generator=g).bfloat16()
    M = G * Lx
    idx = (torch.arange(M, device="cuda") // Lx) * Lm + torch.arange(M, device="cuda") % Lx
    a_c = src[idx].contiguous()
    out_ref = torch.empty(M, D, device="cuda", dtype=torch.bfloat16)
    st_ref = torch.empty(M, 2, 2, device="cuda")
    out = torch.empty_like(out_ref)
    st = torch.empty_like(st_ref)
    mb = torch.full((G * Lm, D), 7.0, device="cuda", dtype=torch.bfloat16)
    stm = torch.full((G * Lm, 2, 2), -3.0, device="cuda")
    # the reference on the kernel the gathered launch takes (the persistent kernel has no row gather: the 256 tile
    # of algo 7, or the 128 tile below 4096 rows), whose partials come from the same reduction order
    try:
        lib.check(lib.load().pdm_set_gemm_algo(algo or (7 if M >= 4096 else 1)), "pdm_set_gemm_algo")
        lib.gemm_ex(lib.EPI_RES, a_c, w, bias, out=out_ref, res_in=res, accumulate=True, stats_out=st_ref)
        lib.check(lib.load().pdm_set_gemm_algo(algo), "pdm_set_gemm_algo")
        lib.gemm_ex(lib.EPI_RES, src, w, bias, out=out, res_in=res, accumulate=True, stats_out=st,
                    a_gather=(M, Lx, Lm), out2=mb, out2_gather=(Lx, Lm), stats_out2=stm)
        torch.cuda.synchronize()
    finally:
        lib.load().pdm_set_gemm_algo(0)
    ref = a_c.float() @ w.float().t() + bias + res.float()
    assert rel(out_ref.float(), ref) < 1e-2
    assert torch.equal(out, out_ref)
    assert torch.equal(st, st_ref)
    assert torch.equal(mb[idx], out)
    assert torch.equal(stm[idx], st)
    rest = torch.ones(G * Lm, dtype=torch.bool, device="cuda")
    rest[idx] = False
    assert bool((mb[rest] == 7.0).all()) and bool((stm[rest] == -3.0).all())
