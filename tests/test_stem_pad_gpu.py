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


def test_pad_cin_kernels_and_zero_at_rest_grad_buffer():
    """_PadCinFn on the GPU: one kernel writes the padded fp32 weight and its bf16 shadow; the conv's
    weight gradient lands in a zero-at-rest buffer on the parameter that the backward folds into the
    arena gradient (channels < C) and re-zeroes — three steps in a row accumulate exactly."""
    from hops_examples_amd.ops import functional as HF

    torch.manual_seed(2)
    w = torch.nn.Parameter(torch.randn(16, 3, 3, 3, device=dev))
    w._hx_grad = torch.zeros_like(w)
    w.grad = w._hx_grad
    total = torch.zeros(16, 3, 3, 8, device=dev)
    for _ in range(3):
        w8 = HF.pad_input_channels(w, 8)
        assert torch.equal(w8[..., :3], w.detach()) and int(torch.count_nonzero(w8[..., 3:])) == 0
        assert torch.equal(w8._hx_shadow, w8.to(torch.bfloat16))
        buf = w8._hx_wbuf
        assert buf is w._hx_padgrad and int(torch.count_nonzero(buf)) == 0
        g = torch.randn(16, 3, 3, 8, device=dev)
        buf.copy_(g)  # what the conv's weight-gradient kernel accumulates
        total += g
        w8.backward(buf)
        torch.cuda.synchronize()
        assert int(torch.count_nonzero(buf)) == 0  # re-zeroed
    torch.testing.assert_close(w._hx_grad, total[..., :3])
