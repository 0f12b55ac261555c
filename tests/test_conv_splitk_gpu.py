"""Small-M split-K path of the conv forward / dgrad GEMMs (conv.hip conv_split: gemm_core.h
EpiAtomicTicket into a zero-at-rest workspace, the tile's last K-slice applies the real epilogue)
against plain PyTorch fp32 convolutions, and against the unsplit kernel (HOPSX_DISABLE=conv_splitk).
Shapes: the ResNet-50 stage-4 3x3 at small batch (392 / 98 output pixels, K = 4,608) and a stage-3
3x3 stride-2 conv."""
import os

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from hops_examples_amd.ops import kernels as K  # noqa: E402

dev = "cuda"
SHAPES = [(8, 7, 512, 512, 3, 1), (2, 7, 512, 512, 3, 1), (8, 14, 256, 256, 3, 2)]


def _bf(t):
    return t.to(torch.bfloat16)


def _close(a, b, tol=2e-2):
    a, b = a.float(), b.float()
    err = float((a - b).abs().max())
    scale = float(b.abs().max())
    assert err <= tol * scale + 1e-3, (err, scale)


def _with(disable, fn):
    old = os.environ.get("HOPSX_DISABLE", "")
    os.environ["HOPSX_DISABLE"] = disable
    try:
        return fn()
    finally:
        os.environ["HOPSX_DISABLE"] = old


@pytest.mark.parametrize("shape", SHAPES)
def test_conv_fwd_dgrad_splitk(shape):
    B, H, C, CO, k, s = shape
    torch.manual_seed(11)
    x = _bf(torch.randn(B, H, H, C, device=dev))
    w = _bf(torch.randn(CO, k, k, C, device=dev) / (k * k * C) ** 0.5)
    g = K.conv_geom(x.shape, w.shape, (s, s), (k // 2, k // 2), (1, 1))
    dy = _bf(torch.randn(B, g[4], g[5], CO, device=dev))
    xt, wt = x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2)
    yref = F.conv2d(xt, wt, None, s, k // 2).permute(0, 2, 3, 1)
    xr = xt.clone().requires_grad_(True)
    F.conv2d(xr, wt, None, s, k // 2).backward(dy.float().permute(0, 3, 1, 2))
    dxref = xr.grad.permute(0, 2, 3, 1)
    for rep in range(2):  # twice: the workspace and the tickets must be back at zero
        y = K.conv2d_fwd(x, w, g)
        dx = K.conv2d_dgrad(dy, w, g)
        torch.cuda.synchronize()
        _close(y, yref)
        _close(dx, dxref)
    y0 = _with("conv_splitk", lambda: K.conv2d_fwd(x, w, g))
    dx0 = _with("conv_splitk", lambda: K.conv2d_dgrad(dy, w, g))
    _close(y, y0, 1e-2)
    _close(dx, dx0, 1e-2)


@pytest.mark.parametrize("shape", SHAPES[:2])
def test_conv_fwd_bnstats_splitk(shape):
    """The split path's finish also writes the BN statistics of the stored bf16 output."""
    B, H, C, CO, k, s = shape
    torch.manual_seed(12)
    x = _bf(torch.randn(B, H, H, C, device=dev))
    w = _bf(torch.randn(CO, k, k, C, device=dev) / (k * k * C) ** 0.5)
    g = K.conv_geom(x.shape, w.shape, (s, s), (k // 2, k // 2), (1, 1))
    gamma, beta = torch.rand(CO, device=dev) + 0.5, torch.randn(CO, device=dev)
    for rep in range(2):
        y = K.conv2d_fwd_bnstats(x, w, g)
        assert y is not None
        mean, rstd = torch.empty(CO, device=dev), torch.empty(CO, device=dev)
        rm, rv = torch.zeros(CO, device=dev), torch.ones(CO, device=dev)
        out = K.bn_fwd_apply_fin(y.view(-1, CO), gamma, beta, mean, rstd, rm, rv, 0.1, 1e-5, act="relu")
        torch.cuda.synchronize()
    assert int(torch.count_nonzero(K.bn_acc(torch.device(dev), CO))) == 0
    yb = y.float().view(-1, CO)
    _close(mean, yb.mean(0), 1e-3)
    _close(rstd, (yb.var(0, unbiased=False) + 1e-5).rsqrt(), 1e-3)
    ref = F.batch_norm(yb, None, None, gamma, beta, True, 0.1, 1e-5).relu()
    _close(out, ref)
