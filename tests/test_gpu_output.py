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
