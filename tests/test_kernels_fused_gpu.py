"""Prologue-fused backward GEMMs: act' mask applied while staging the A operand,
and bias gradients produced as row sums of the staged dY^T (no elementwise pass)."""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from hops_examples_amd.ops import kernels as K  # noqa: E402

dev = "cuda"


def bf(t):
    return t.to(torch.bfloat16)


def close(a, b, tol=2e-2):
    a, b = a.float(), b.float()
    err = (a - b).abs().max().item()
    scale = b.abs().max().item() + 1e-6
    assert err <= tol * scale + 1e-4, f"max err {err} vs scale {scale}"


@pytest.mark.parametrize("M,Kd,N", [(32, 10816, 128), (64, 800, 500), (2048, 256, 384), (33, 20, 10), (300, 77, 64)])
@pytest.mark.parametrize("act", ["relu", "sigmoid"])
def test_linear_backward_prologue_fused(M, Kd, N, act):
    torch.manual_seed(0)
    x = bf(torch.randn(M, Kd, device=dev)).relu()
    w = bf(torch.randn(N, Kd, device=dev) / math.sqrt(Kd))
    pre = x.float() @ w.float().t()
    y = bf(pre.relu() if act == "relu" else pre.sigmoid())
    dy = bf(torch.randn(M, N, device=dev))
    der = (y.float() > 0).float() if act == "relu" else y.float() * (1 - y.float())
    dpre = dy.float() * der
    dx = K.linear_dgrad(dy, w, y=y, act=act)
    close(dx, dpre @ w.float())
    dw = torch.zeros(N, Kd, device=dev)
    db = torch.zeros(N, device=dev)
    K.linear_wgrad(dy, x, dw, y=y, act=act, dbias=db)
    close(dw, dpre.t() @ x.float())
    close(db, dpre.sum(0), tol=3e-2)


@pytest.mark.parametrize("B,H,W,C,CO,k,s,p", [
    (32, 27, 27, 32, 64, 2, 1, 0),   # mirrored conv2 (implicit GEMM)
    (32, 28, 28, 1, 32, 2, 1, 0),    # mirrored conv1 (direct kernel)
    (64, 28, 28, 1, 20, 5, 1, 0),    # torch Net conv1 (direct)
    (8, 16, 16, 64, 128, 3, 2, 1),   # resnet stride 2
])
def test_conv_backward_prologue_fused(B, H, W, C, CO, k, s, p):
    torch.manual_seed(1)
    x = bf(torch.randn(B, H, W, C, device=dev)).relu()
    w = bf(torch.randn(CO, k, k, C, device=dev) / math.sqrt(k * k * C))
    g = K.conv_geom(x.shape, w.shape, (s, s), (p, p), (1, 1))
    y = K.conv2d_fwd(x, w, g, act="relu")
    dy = bf(torch.randn_like(y.float()))
    xr = x.float().permute(0, 3, 1, 2).requires_grad_(True)
    wr = w.float().permute(0, 3, 1, 2).requires_grad_(True)
    pre = F.conv2d(xr, wr, None, stride=s, padding=p)
    dpre = (dy.float() * (y.float() > 0)).permute(0, 3, 1, 2)
    gx, gw = torch.autograd.grad(pre, (xr, wr), dpre)
    if C > 1:
        dx = K.conv2d_dgrad(dy, w, g, y=y, act="relu")
        close(dx, gx.permute(0, 2, 3, 1))
    dw = torch.zeros(CO, k, k, C, device=dev)
    db = torch.zeros(CO, device=dev)
    K.conv2d_wgrad(dy, x, g, dw, dbias=db, y=y, act="relu")
    close(dw, gw.permute(0, 2, 3, 1))
    close(db, dpre.sum((0, 2, 3)), tol=3e-2)
