"""Output-stage HIP kernels vs the oracle, bit-exact (uint8 pixels, int32 ids)."""
import numpy as np
import pytest
import torch

from oracle import utils_ref
from panopticdiffusionmodels_amd import output
from test_output import _edge_images

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def test_images_to_u8(dev):
    x = _edge_images()
    got = output.images_to_u8(x.to(dev)).cpu().numpy()
    np.testing.assert_array_equal(got, utils_ref.save_image_u8(x.numpy()))
    g = torch.Generator().manual_seed(9)
    big = torch.randn(5, 3, 256, 256, generator=g) * 0.8
    np.testing.assert_array_equal(output.images_to_u8(big.to(dev)).cpu().numpy(), utils_ref.save_image_u8(big.numpy()))


def test_masks_to_ids_rgb(dev):
    g = torch.Generator().manual_seed(10)
    bits = torch.randn(3, 8, 32, 32, generator=g)
    bits[0, :, 0, 0] = torch.tensor([1.0, -1, 0.0, 2, -0.0, 1e-30, -1e-30, 3])   # ties at 0 count as 0
    cmap = output.default_colormap(5)
    ids, rgb = output.masks_to_ids_rgb(bits.to(dev), cmap)
    ref_ids = utils_ref.bits2int(bits.numpy() > 0)[:, 0]
    np.testing.assert_array_equal(ids.cpu().numpy(), ref_ids)
    np.testing.assert_array_equal(rgb.cpu().numpy(), utils_ref.color_map(ref_ids, cmap.numpy()))


@pytest.mark.parametrize("n,off_x,off_y", [(0, 0, 0), (7, 0, 0), (8, 0, 0), (1 << 20, 0, 0), (1_000_003, 0, 0),
                                           (4099, 1, 0), (4099, 0, 3), (4104, 4, 8)])
def test_f32_to_bf16_cast(dev, n, off_x, off_y):
    """pdm_f32_to_bf16 (the decoder / t2i context cast): vector body + scalar tail + unaligned views, bit-exact vs
    torch's round-to-nearest-even, inf / nan / denormals included."""
    from panopticdiffusionmodels_amd import _lib
    lib = _lib.load()
    g = torch.Generator(device=dev).manual_seed(n)
    xs = torch.randn(n + off_x, device=dev, generator=g) * 100
    if n > 16:
        xs[off_x:off_x + 4] = torch.tensor([float("inf"), -float("inf"), 1e-40, -0.0], device=dev)
    x = xs[off_x:]
    ys = torch.full((n + off_y,), 7.0, device=dev, dtype=torch.bfloat16)
    y = ys[off_y:]
    rc = lib.pdm_f32_to_bf16(x.data_ptr(), y.data_ptr(), n, _lib.stream_ptr(dev))
    assert rc == 0, lib.pdm_last_error()
    torch.cuda.synchronize(dev)
    assert torch.equal(y.view(torch.int16), x.bfloat16().view(torch.int16))
    assert torch.equal(ys[:off_y], torch.full((off_y,), 7.0, device=dev, dtype=torch.bfloat16))
