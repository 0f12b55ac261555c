"""8-channel image stems on the GPU (kernels.u8_normalize_chan cout=8 + nn.Conv2d weight padding):
the normalised channels equal the 3-channel kernel's, channels 3..7 are zero, and a ResNet step with
the padded stem matches the unpadded one (HOPSX_DISABLE=stem_pad)."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from hops_examples_amd.ops import kernels as K  # noqa: E402

dev = "cuda"


def test_u8_normalize_chan8():
    x = torch.randint(0, 256, (4, 17, 19, 3), device=dev, dtype=torch.uint8)
    sc, sh = [0.5, 1.0, 2.0], [-103.9, -116.8, -123.7]
    y3 = K.u8_normalize_chan(x, sc, sh, reverse=True)
    y8 = K.u8_normalize_chan(x, sc, sh, reverse=True, cout=8)
    assert y8.shape == (4, 17, 19, 8)
    assert torch.equal(y8[..., :3], y3)
    assert int(torch.count_nonzero(y8[..., 3:])) == 0


def _stem(disable: str, depth=None):
    """The image normalisation + stem ConvBN alone (the tight comparison: a whole random-init ResNet
    amplifies any last-bit difference layer by layer, see test_bnstats_gpu.py)."""
    from hops_examples_amd.models.resnet import _as_nhwc_image, cifar_resnet, resnet50

    old = os.environ.get("HOPSX_DISABLE", "")
    os.environ["HOPSX_DISABLE"] = disable
    try:
        torch.manual_seed(0)
        m = (cifar_resnet(depth) if depth else resnet50()).to(dev).train()
        hw = 32 if depth else 96
        x = torch.randint(0, 256, (8, hw, hw, 3), device=dev, dtype=torch.uint8)
        xn = _as_nhwc_image(x, m)
        assert xn.shape[-1] == (3 if disable else 8)
        y = m.stem(xn)
        g = torch.randn(y.shape, device=dev, generator=torch.Generator(device=dev).manual_seed(1))
        (y.float() * g).sum().backward()
        return y.float().detach(), m.stem.conv.weight.grad.float().clone()
    finally:
        os.environ["HOPSX_DISABLE"] = old


@pytest.mark.parametrize("depth", [None, 20])
def test_padded_stem_matches_unpadded(depth):
    y1, g1 = _stem("", depth)
    y0, g0 = _stem("stem_pad", depth)
    assert g1.shape == g0.shape and g1.shape[-1] == 3
    torch.testing.assert_close(y1, y0, rtol=2e-2, atol=2e-2)
    rel = float((g1 - g0).norm() / g0.norm())
    assert rel < 1e-2, rel
