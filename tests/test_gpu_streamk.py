"""Stream-K persistent GEMM (csrc/gemm.hip gemm8s_body, SK = 1) at the U-ViT block shapes.

A workgroup's tail piece continues its predecessor's accumulators (handed over through an fp32 slab) instead of
starting a second partial sum, so every output element is the same chain of MFMA accumulations as in a whole-tile
launch: stream-K vs whole tiles must be BIT-identical (bf16 outputs, LayerNorm partials, MXFP8 copies), for the
hand-off and for its fallback (the tail recomputing the tile when the hand-off is not taken, pdm_set_gemm_tuning
bit 7), and across repeated launches.  The reference op is the block Linear of libs/uvit.py:66-120 /
libs/timm.py:96-112 (nn.Linear + residual / LayerNorm consumer / GELU); an fp32 torch check keeps the comparison
anchored (bf16 rel-L2 <= 1e-2)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


@pytest.fixture(scope="module")
def lib():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from panopticdiffusionmodels_amd import _lib
    _lib.load()
    yield _lib
    _lib.load().pdm_set_gemm_sk(0)
    _lib.load().pdm_set_gemm_tuning(0, 0)


# (name, M, N, K, kind): L/2 at the bench's 100 rows (258 tokens), U-ViT-H (D 1152), odd row counts, odd K-step count
CASES = [
    ("proj_res", 25800, 1024, 1024, "res"),
    ("fc2_res", 25800, 1024, 4096, "res"),
    ("skip_split", 25800, 1024, 2048, "skip"),
    ("qkv_ln", 25800, 3072, 1024, "ln"),
    ("fc1_ln_gelu", 25800, 4096, 1024, "ln_gelu"),
    ("h_proj_res", 25800, 1152, 1152, "res"),
    ("h_fc1_mxo", 25800, 4608, 1152, "mxo"),
    ("ragged_rows", 25800 + 1337, 1024, 1024, "res"),
    ("odd_ksteps", 25800, 1024, 1088, "ln"),
]


def _problem(lib, M, N, K, kind, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    kk = K // 2 if kind == "skip" else K
    a = torch.randn(M, kk, device="cuda", generator=g).bfloat16()
    w = (torch.randn(N, K, device="cuda", generator=g) * K ** -0.5).bfloat16()
    kw = dict(a=a, w=w, bias=torch.randn(N, device="cuda", generator=g))
    epi = lib.EPI_BF16
    if kind in ("res", "skip"):
        epi = lib.EPI_RES
        kw["out"] = torch.randn(M, N, device="cuda", generator=g).bfloat16()
        kw["res_in"] = kw["out"]            # in place, as the forward's residual stream
        kw["accumulate"] = True
        kw["stats_out"] = torch.empty(M, (N + 255) // 256, 2, device="cuda")
        if kind == "skip":
            kw["a2"] = torch.randn(M, kk, device="cuda", generator=g).bfloat16()
    else:
        _, st = lib.rowstats(torch.randn(M, K, device="cuda", generator=g) * 1.3 + 0.2, want_bf16=False)
        kw["ln_stats"], kw["ln_colsum"] = st, w.float().sum(1)
        if kind in ("ln_gelu", "mxo"):
            epi = lib.EPI_GELU
        if kind == "mxo":
            kw["out_fp8"] = torch.empty(M, N, device="cuda", dtype=torch.float8_e4m3fn)
            kw["out_scale"] = torch.zeros(N // 128, M, device="cuda", dtype=torch.int32)
        else:
            kw["out"] = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    return epi, kw


def _outputs(kw):
    return {k: kw[k] for k in ("out", "stats_out", "out_fp8", "out_scale") if k in kw}


def _run(lib, epi, kw, init, mode, dbg=0):
    """One launch from the same initial output state; returns copies of every output."""
    for k, v in init.items():
        kw[k].copy_(v)
    L = lib.load()
    lib.check(L.pdm_set_gemm_sk(mode), "pdm_set_gemm_sk")
    L.pdm_set_gemm_tuning(0, dbg)
    try:
        lib.gemm_ex(epi, **kw)
        torch.cuda.synchronize()
    finally:
        L.pdm_set_gemm_tuning(0, 0)
        L.pdm_set_gemm_sk(0)
    return {k: v.clone() for k, v in _outputs(kw).items()}


@pytest.mark.parametrize("name,M,N,K,kind", CASES, ids=[c[0] for c in CASES])
def test_streamk_bit_identical(lib, name, M, N, K, kind):
    epi, kw = _problem(lib, M, N, K, kind, seed=hash(name) % 10007)
    init = {k: v.clone() for k, v in _outputs(kw).items()}
    L = lib.load()
    whole = _run(lib, epi, kw, init, 0)
    n0 = L.pdm_gemm_sk_launches()
    sk = _run(lib, epi, kw, init, 2 | 4)
    assert L.pdm_gemm_sk_launches() == n0 + 1, "stream-K was not taken for this shape"
    sk2 = _run(lib, epi, kw, init, 2 | 4)
    fb = _run(lib, epi, kw, init, 2 | 4, dbg=128)   # every tail recomputes its tile
    for k in whole:
        assert torch.equal(sk[k].view(torch.uint8), whole[k].view(torch.uint8)), (name, k, "stream-K vs whole tiles")
        assert torch.equal(sk2[k].view(torch.uint8), sk[k].view(torch.uint8)), (name, k, "repeat")
        assert torch.equal(fb[k].view(torch.uint8), whole[k].view(torch.uint8)), (name, k, "fallback")
    # anchor: the fp32 torch op on the same bf16 operands
    a = kw["a"].float() if kind != "skip" else torch.cat([kw["a"], kw["a2"]], 1).float()
    ref = a @ kw["w"].float().t()
    if kind in ("res", "skip"):
        ref = ref + kw["bias"] + init["out"].float()
        assert rel(sk["out"].float(), ref) < 1e-2
    elif kind == "mxo":
        assert torch.isfinite(sk["out_fp8"].float()).all()
    else:
        assert torch.isfinite(sk["out"].float()).all()


def test_streamk_auto_policy(lib):
    """The automatic policy takes stream-K for the partly filled last wave (404 tiles on 256 CUs) and leaves exact
    waves (512 tiles) and single partial waves (< 256 tiles) to whole tiles."""
    L = lib.load()
    for M, N, expect in ((25800, 1024, 1), (256 * 128, 1024, 0), (12900, 1024, 0)):
        epi, kw = _problem(lib, M, N, 1024, "res", seed=M)
        init = {k: v.clone() for k, v in _outputs(kw).items()}
        n0 = L.pdm_gemm_sk_launches()
        _run(lib, epi, kw, init, 1 | 4)
        assert L.pdm_gemm_sk_launches() - n0 == expect, (M, N)


def test_streamk_forward_bit_identical(lib):
    """The U-ViT-L/2 forward at the bench's 100 rows with the automatic stream-K policy (every N = 1024 / 3072 / 4096
    block Linear on stream-K, flag blocks from the forward's workspace) equals the whole-tile forward (the default)
    bit for bit, twice."""
    from panopticdiffusionmodels_amd import configs as C
    from panopticdiffusionmodels_amd import weights as W
    from panopticdiffusionmodels_amd.utils import get_nnet
    cfg = C.nnet_kwargs("imagenet256_uvit_large")
    net = get_nnet(**cfg)
    net.load_state_dict(W.nnet_state_dict(cfg, seed=0, init="reference"))
    net = net.cuda().eval()
    g = torch.Generator().manual_seed(5)
    x = torch.randn(100, 4, 32, 32, generator=g).cuda()
    t = (torch.rand(100, generator=g) * 999).cuda()
    y = torch.randint(0, 1001, (100,), generator=g).cuda()
    L = lib.load()
    with torch.no_grad():
        L.pdm_set_gemm_sk(0)
        whole = net(x, t, y).clone()
        L.pdm_set_gemm_sk(1)
        try:
            n0 = L.pdm_gemm_sk_launches()
            a = net(x, t, y).clone()
            b = net(x, t, y).clone()
        finally:
            L.pdm_set_gemm_sk(0)
    assert L.pdm_gemm_sk_launches() - n0 >= 2 * 21 * 3   # proj, fc1, fc2 of 21 blocks per forward at least
    assert torch.isfinite(a).all()
    assert torch.equal(a, whole)
    assert torch.equal(b, whole)
