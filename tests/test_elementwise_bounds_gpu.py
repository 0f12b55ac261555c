"""Per-element error bounds for the flagship's fused kernels at the real shapes (realistic K).

The other kernel tests bound the error relative to the tensor's max magnitude; here every element
is checked against an fp64 reference computed from the SAME bf16 operands, so the only admissible
differences are fp32 accumulation order and the final rounding of the stored dtype:
  * fp32 outputs (weight gradients): |err| <= 1e-4 |ref| + 1e-5 rms(ref)
  * bf16 outputs: |err| <= 2^-8 |ref| (one rounding) + 1e-3 rms(ref) (a rounding-boundary flip of an
    element whose fp32 value sits next to a bf16 tie, plus accumulation order on near-zero sums)
"""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from hops_examples_amd.ops import kernels as K  # noqa: E402

dev = "cuda"
bf = torch.bfloat16


def _check(out, ref, rel, rms_frac):
    out, ref = out.double(), ref.double()
    rms = ref.pow(2).mean().sqrt().item()
    bound = rel * ref.abs() + rms_frac * rms
    bad = (out - ref).abs() > bound
    n = int(bad.sum())
    assert n == 0, (f"{n} of {ref.numel()} elements out of bounds; worst excess "
                    f"{((out - ref).abs() - bound).max().item():.3e} (rms {rms:.3e})")


def test_conv2_backward_pair_per_element():
    """conv_bwd_pair_k at the flagship conv2 (B 32, 27x27x32 -> 26x26x64, 2x2): dX (bf16) and dW
    (fp32, K = 21,632-long reductions)."""
    torch.manual_seed(0)
    x = torch.randn(32, 27, 27, 32, device=dev).relu().to(bf)
    w = (torch.randn(64, 2, 2, 32, device=dev) / math.sqrt(128)).to(bf)
    dy = (torch.randn(32, 26, 26, 64, device=dev) * 0.05).to(bf)
    g = K.conv_geom(x.shape, w.shape, (1, 1), (0, 0), (1, 1))
    dw = torch.zeros(64, 2, 2, 32, device=dev)
    dx = K.conv2d_bwd_pair(dy, w, g, x, dw)
    assert dx is not False
    xr = x.double().permute(0, 3, 1, 2).requires_grad_(True)
    wr = w.double().permute(0, 3, 1, 2).requires_grad_(True)
    yr = torch.nn.functional.conv2d(xr, wr)
    gx, gw = torch.autograd.grad(yr, (xr, wr), dy.double().permute(0, 3, 1, 2))
    _check(dx, gx.permute(0, 2, 3, 1), 2.0 ** -8, 1e-3)
    _check(dw, gw.permute(0, 2, 3, 1), 1e-4, 1e-5)


def test_fc1_backward_pair_per_element():
    """linear_bwd_pair_k at the flagship fc1 (32 x 10816 -> 128): dX (bf16) and dW stored (fp32)."""
    torch.manual_seed(1)
    x = torch.randn(32, 10816, device=dev).relu().to(bf)
    w = (torch.randn(128, 10816, device=dev) / math.sqrt(10816)).to(bf)
    dy = (torch.randn(32, 128, device=dev) * 0.1).to(bf)
    dw = torch.zeros(128, 10816, device=dev)
    dx = K.linear_bwd_pair(dy, w, x, dw, dw_store=True)
    assert dx is not False
    _check(dx, dy.double() @ w.double(), 2.0 ** -8, 1e-3)
    _check(dw, dy.double().t() @ x.double(), 1e-4, 1e-5)


def test_mlp_head_per_element():
    """mlp_head_k at the flagship shape (fc1 split-K over 10,816 + relu, fc2 10-way head, softmax CE,
    head gradients): y / logits (bf16), dW2 (fp32), dh (bf16)."""
    torch.manual_seed(2)
    B, Kd, N1, C = 32, 10816, 128, 10
    x = torch.randn(B, Kd, device=dev).relu().to(bf)
    w1 = (torch.randn(N1, Kd, device=dev) / math.sqrt(Kd)).to(bf)
    b1 = torch.randn(N1, device=dev) * 0.1
    w2 = (torch.randn(C, N1, device=dev) / math.sqrt(N1)).to(bf)
    b2 = torch.randn(C, device=dev) * 0.1
    t = torch.randint(0, C, (B,), device=dev)
    y = torch.empty(B, N1, device=dev, dtype=bf)
    lg = torch.empty(B, C, device=dev, dtype=bf)
    dw2 = torch.zeros(C, N1, device=dev)
    db2 = torch.zeros(C, device=dev)
    loss = torch.empty(1, device=dev)
    corr = torch.empty(1, device=dev, dtype=torch.int32)
    dh = K.mlp_head(x, w1, b1, "relu", y, 0, lg, t, w2, b2, dw2, db2, 1.0 / B, loss, corr)
    assert dh is not False
    torch.cuda.synchronize()
    yref = (x.double() @ w1.double().t() + b1.double()).relu()
    _check(y, yref, 2.0 ** -8, 1e-3)
    # the head consumes the STORED bf16 y (as the unfused chain would): reference from y itself
    lref = y.double() @ w2.double().t() + b2.double()
    _check(lg, lref, 2.0 ** -8, 1e-3)
    p = torch.softmax(lg.double(), 1)
    dl = (p - torch.nn.functional.one_hot(t, C).double()) / B
    _check(dw2, dl.t() @ y.double(), 1e-3, 1e-4)  # dl is fp32 in-kernel (from bf16 logits): 1e-3
    _check(dh, dl @ w2.double(), 2.0 ** -8, 2e-3)
    ref_loss = torch.nn.functional.cross_entropy(lg.double(), t).item()
    assert abs(loss.item() - ref_loss) <= 1e-5 * abs(ref_loss) + 1e-6
