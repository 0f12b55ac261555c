"""Zero-padded input channels (ResNet image stems laid out as 8 channels, nn.Conv2d + _PadCinFn): the
conv and every gradient equal the unpadded conv's (CPU reference path; the GPU run of the same model
is covered by tests/test_models_gpu.py and tests/test_stem_pad_gpu.py)."""
import torch

from hops_examples_amd import nn as hnn


def test_padded_input_channels_match_unpadded():
    torch.manual_seed(0)
    conv = hnn.Conv2d(3, 16, 7, stride=2, padding=3, bias=False, init="he")
    x = torch.randn(2, 20, 20, 3)
    y0 = conv(x)
    g = torch.randn_like(y0)
    (y0 * g).sum().backward()
    gw0 = conv.weight.grad.clone()
    conv.weight.grad = None
    x8 = torch.nn.functional.pad(x, (0, 5))  # channels 3..7 zero
    y1 = conv(x8)
    (y1 * g).sum().backward()
    torch.testing.assert_close(y1, y0, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(conv.weight.grad, gw0, rtol=1e-5, atol=1e-5)
    assert conv.weight.shape == (16, 7, 7, 3)  # the parameter itself is unchanged


def test_padded_weight_gradient_goes_to_the_arena_buffer():
    from hops_examples_amd.ops import functional as HF

    w = torch.nn.Parameter(torch.randn(4, 3, 3, 3))
    w._hx_grad = torch.zeros_like(w)
    w.grad = w._hx_grad
    w8 = HF.pad_input_channels(w, 8)
    assert w8.shape == (4, 3, 3, 8) and float(w8[..., 3:].abs().sum()) == 0.0
    g = torch.randn(4, 3, 3, 8)
    w8.backward(g)
    torch.testing.assert_close(w._hx_grad, g[..., :3])
    assert w.grad is w._hx_grad  # accumulated in place, not replaced
