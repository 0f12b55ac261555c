"""Projection-shortcut blocks: conv a's input gradient handed to the short conv's dgrad epilogue
(ops.functional.GiveGrad, models/resnet.py) instead of an autograd add — same gradients as the unfused
block (HOPSX_DISABLE=proj_addend) up to the rounding of one bf16 add, and order-safe when the taker
runs first."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

dev = "cuda"


def _block_grads(make, shape, disable):
    old = os.environ.get("HOPSX_DISABLE", "")
    os.environ["HOPSX_DISABLE"] = disable + ",bnstats"  # (statistics order fixed: same forward both runs)
    try:
        torch.manual_seed(0)
        m = make().to(dev).train()
        x = torch.randn(shape, device=dev).to(torch.bfloat16).requires_grad_(True)
        y = m(x)
        g = torch.randn(y.shape, device=dev, generator=torch.Generator(device=dev).manual_seed(3))
        (y.float() * g).sum().backward()
        return y.float().detach(), x.grad.float().clone(), [p.grad.float().clone() for p in m.parameters()]
    finally:
        os.environ["HOPSX_DISABLE"] = old


def _rel(a, b):
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


@pytest.mark.parametrize("which", ["bottleneck_s2", "bottleneck_s1", "basic_s2"])
def test_projection_block_grads_match_unfused(which):
    from hops_examples_amd.models.resnet import BasicBlock, Bottleneck

    make, shape = {
        "bottleneck_s2": (lambda: Bottleneck(256, 128, 2), (8, 28, 28, 256)),
        "bottleneck_s1": (lambda: Bottleneck(64, 64, 1), (8, 28, 28, 64)),
        "basic_s2": (lambda: BasicBlock(16, 32, 2), (16, 32, 32, 16)),
    }[which]
    y1, dx1, g1 = _block_grads(make, shape, "")
    y0, dx0, g0 = _block_grads(make, shape, "proj_addend")
    assert _rel(y1, y0) < 1e-3
    assert _rel(dx1, dx0) < 1e-2, _rel(dx1, dx0)
    for a, b in zip(g1, g0):
        assert _rel(a, b) < 2e-2, _rel(a, b)


def test_give_grad_taker_first_is_safe():
    """If the taker runs first it marks the slot late and the giver returns its gradient itself."""
    from hops_examples_amd.ops import functional as HF

    torch.manual_seed(1)
    x = torch.randn(4, 8, 8, 16, device=dev).to(torch.bfloat16).requires_grad_(True)
    w1 = torch.randn(16, 1, 1, 16, device=dev) * 0.2
    w2 = torch.randn(16, 1, 1, 16, device=dev) * 0.2
    slot = {}
    # taker created LAST -> backpropagated FIRST (the reverse of the ResNet blocks' order)
    ya = HF.conv2d(x, w1, gslot=HF.GiveGrad(slot))
    yb = HF.conv2d(x, w2, gslot=slot)
    (ya.float().sum() + 2 * yb.float().sum()).backward()
    got = x.grad.float().clone()
    x.grad = None
    ya = HF.conv2d(x, w1)
    yb = HF.conv2d(x, w2)
    (ya.float().sum() + 2 * yb.float().sum()).backward()
    assert _rel(got, x.grad.float()) < 1e-2
    assert "g" not in slot
