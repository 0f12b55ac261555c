"""TF 'same' padding with an even kernel (the HPO kernels 2..8 of evolutionary_search_mnist.ipynb:264 /
grid_search_fashion_mnist.ipynb:224-236): an asymmetric geometry (one more row / column of zero padding at
the end, K.conv_geom 4-tuple padding) instead of a padded copy of the input — forward, input and weight
gradients against the CPU reference (F.pad + conv)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from hops_examples_amd.ops import functional as HF  # noqa: E402
from hops_examples_amd.ops import kernels as K  # noqa: E402


def test_conv_geom_asymmetric_same():
    g = K.conv_geom((2, 28, 28, 1), (32, 4, 4, 1), (1, 1), (1, 1, 2, 2), (1, 1))
    assert g[4:6] == [28, 28] and g[11:13] == [1, 1]
    assert K.conv_geom((2, 9, 7, 8), (8, 2, 2, 8), (1, 1), (0, 0, 1, 1), (1, 1))[4:6] == [9, 7]


@pytest.mark.parametrize("k,C,CO,H", [(2, 1, 32, 28), (4, 1, 32, 28), (2, 32, 64, 14), (4, 32, 64, 14), (6, 16, 16, 11)])
def test_same_even_kernel_matches_padded_reference(k, C, CO, H):
    torch.manual_seed(k * 100 + C)
    x = torch.randn(4, H, H, C)
    w = torch.randn(CO, k, k, C) / (k * k * C) ** 0.5
    b = torch.randn(CO) * 0.1
    dy = torch.randn(4, H, H, CO)
    outs = []
    for dev in ("cpu", "cuda"):
        xb = x.to(torch.bfloat16).to(dev)
        xd = (xb.float() if dev == "cpu" else xb).detach().clone().requires_grad_(True)
        wd = w.to(torch.bfloat16).float().to(dev).detach().clone().requires_grad_(True)
        bd = b.to(dev).detach().clone().requires_grad_(True)
        y = HF.conv2d(xd, wd, bd, padding="same", act="relu")
        assert tuple(y.shape) == (4, H, H, CO)
        y.backward(dy.to(dev).to(y.dtype))
        outs.append([t.detach().float().cpu() for t in (y, xd.grad, wd.grad, bd.grad)])
    for name, a, r in zip(("y", "dx", "dw", "db"), outs[1], outs[0]):
        scale = r.abs().max().item() + 1e-6
        torch.testing.assert_close(a, r, rtol=3e-2, atol=3e-2 * scale, msg=name)


def test_same_even_uint8_input_layer():
    """A uint8 image into a k=2 'same' conv with the input normalisation (the HPO models' first layer)."""
    torch.manual_seed(1)
    x8 = torch.randint(0, 256, (4, 28, 28, 1), dtype=torch.uint8)
    w = torch.randn(32, 2, 2, 1) * 0.5
    ref = HF.conv2d(x8.float() / 255.0, w, None, padding="same", act="relu")
    got = HF.conv2d(x8.cuda(), w.cuda(), None, padding="same", act="relu", in_affine=(1 / 255.0, 0.0))
    torch.testing.assert_close(got.float().cpu(), ref, rtol=2e-2, atol=2e-2)
