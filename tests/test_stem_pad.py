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
    x8._hx_chpad = 3  # (as models/resnet.py tags the normalisation kernel's 8-channel output)
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


def test_untagged_channel_mismatch_raises():
    """Extra input channels are only dropped when the producer says they are zero padding."""
    import pytest

    conv = hnn.Conv2d(3, 4, 3)
    with pytest.raises(ValueError, match="expects 3 input channels"):
        conv(torch.randn(1, 8, 8, 4))  # e.g. an RGBA image
    with pytest.raises(ValueError):
        conv(torch.randn(1, 8, 8, 2))


def test_stem_pad_grad_is_accumulated_before_grad_ready():
    """_PadCinFn.backward adds the stem gradient into the arena BEFORE announcing it to the DP overlap
    hook (a bucket all-reduce launched on the announcement must see the gradient)."""
    from hops_examples_amd.ops import functional as HF
    from hops_examples_amd.runtime import hooks

    w = torch.nn.Parameter(torch.randn(4, 3, 3, 3))
    w._hx_grad = torch.zeros_like(w)
    w.grad = w._hx_grad
    seen = []
    fn = lambda p: seen.append(float(p._hx_grad.abs().sum()))  # noqa: E731
    hooks.subscribe(fn)
    try:
        HF.pad_input_channels(w, 8).backward(torch.ones(4, 3, 3, 8))
    finally:
        hooks.unsubscribe(fn)
    assert seen == [4 * 3 * 3 * 3]
