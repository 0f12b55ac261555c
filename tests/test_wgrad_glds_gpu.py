"""Numerics of the LDS-DMA conv weight gradient (csrc/ops/wgrad_glds.hip) vs an fp32 PyTorch
reference: 1x1 / 3x3, stride 1 / 2, padding, ragged tile edges (CO, KH*KW*C and the pixel count not
multiples of 128 / 64), split-K accumulation into a non-zero dW, and the dispatch through
``conv2d_wgrad`` (the ResNet-50 path)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from hops_examples_amd.ops import _C  # noqa: E402
from hops_examples_amd.ops import kernels as K  # noqa: E402

dev = torch.device("cuda", 0)
bf = torch.bfloat16


def _ref(dy, x, CO, C, k, stride, pad):
    wr = torch.zeros(CO, C, k, k, device=dev, requires_grad=True)
    F.conv2d(x.float().permute(0, 3, 1, 2), wr, stride=stride, padding=pad).backward(dy.float().permute(0, 3, 1, 2))
    return wr.grad.permute(0, 2, 3, 1).reshape(CO, -1)


CASES = [  # B, H, C, CO, k, stride, pad
    (8, 14, 64, 256, 1, 1, 0),     # ResNet-50 bottleneck expand
    (4, 28, 128, 128, 3, 2, 1),    # strided 3x3
    (4, 28, 256, 512, 1, 2, 0),    # downsample projection
    (3, 17, 72, 136, 3, 1, 1),     # ragged: N = 648, CO = 136, 867 pixels
    (2, 9, 512, 64, 1, 1, 0),      # 162 pixels -> fails the >= 8 k-steps rule: not eligible
    (16, 7, 512, 2048, 1, 1, 0),   # stage-4 expand, many tiles
    (8, 56, 64, 64, 3, 1, 1),      # stage-1 3x3: 576 x 64 output, the 256x64 tile (RC B, 64 live columns)
    (8, 56, 64, 64, 1, 1, 0),      # 64 x 64 output
]


@pytest.mark.parametrize("B,H,C,CO,k,stride,pad", CASES)
def test_wgrad_glds_direct(B, H, C, CO, k, stride, pad):
    torch.manual_seed(11)
    x = torch.randn(B, H, H, C, device=dev).to(bf)
    g = K.conv_geom(x.shape, (CO, k, k, C), (stride, stride), (pad, pad), (1, 1))
    dy = torch.randn(B, g[4], g[5], CO, device=dev).to(bf)
    ok = bool(_C.ext().conv_wgrad_glds_ok(g))
    assert ok == (B * g[4] * g[5] >= 512)
    if not ok:
        return
    base = torch.randn(CO, k * k * C, device=dev)
    dw = base.clone()
    rc = _C.ext().conv2d_wgrad_glds(K.ptr(dy), K.ptr(x), g, K.ptr(dw), 1, K.stream())
    assert rc == 0
    torch.cuda.synchronize()
    ref = _ref(dy, x, CO, C, k, stride, pad)
    got = dw - base
    torch.testing.assert_close(got, ref, atol=1e-2 * ref.abs().max().item(), rtol=1e-2)


def test_wgrad_glds_via_dispatch():
    """conv2d_wgrad (no mask, no bias grad) routes eligible shapes through the glds kernel."""
    torch.manual_seed(3)
    B, H, C, CO = 8, 14, 256, 256
    x = torch.randn(B, H, H, C, device=dev).to(bf)
    g = K.conv_geom(x.shape, (CO, 3, 3, C), (1, 1), (1, 1), (1, 1))
    dy = torch.randn(B, H, H, CO, device=dev).to(bf)
    dw = torch.zeros(CO, 3, 3, C, device=dev)
    K.conv2d_wgrad(dy, x, g, dw)
    ref = _ref(dy, x, CO, C, 3, 1, 1)
    torch.testing.assert_close(dw.reshape(CO, -1), ref, atol=1e-2 * ref.abs().max().item(), rtol=1e-2)


FWD_CASES = [  # B, H, C, CO, k, stride  (big enough that the gg engine takes them)
    (8, 56, 64, 256, 1, 1),
    (32, 28, 128, 128, 3, 1),
    (32, 56, 64, 128, 3, 2),
    (16, 28, 256, 512, 1, 2),
    # 64 output (or, for dgrad, input) channels: the 256x64 tile (gg_plan cfg 3)
    (16, 56, 64, 64, 3, 1),
    (8, 56, 256, 64, 1, 1),
    (8, 56, 64, 128, 3, 2),   # dgrad N = 64 over the stride-2 parity classes
    (48, 224, 8, 64, 7, 2),   # the ResNet-50 stem (channels padded to 8): gg instead of the direct kernel
    (64, 56, 64, 256, 1, 1),  # stage-1 expand at batch 64: its dgrad (N = 64, K = 256) on gg, not the direct kernel
]


@pytest.mark.parametrize("B,H,C,CO,k,stride", FWD_CASES)
def test_gg_conv_fwd_and_dgrad(B, H, C, CO, k, stride):
    """Forward (KC x KC: dense or im2col rows) and dgrad (KC dY gather x RC transposed weight) on the gg
    engine vs fp32 PyTorch."""
    torch.manual_seed(7)
    pad = k // 2
    x = torch.randn(B, H, H, C, device=dev).to(bf)
    w = (torch.randn(CO, k, k, C, device=dev) * 0.05).to(bf)
    g = K.conv_geom(x.shape, w.shape, (stride, stride), (pad, pad), (1, 1))
    y = K.conv2d_fwd(x, w, g)
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), stride=stride, padding=pad)
    ref = ref.permute(0, 2, 3, 1)
    torch.testing.assert_close(y.float(), ref, atol=2e-2 * ref.abs().max().item(), rtol=2e-2)
    dy = torch.randn(B, g[4], g[5], CO, device=dev).to(bf)
    dx = K.conv2d_dgrad(dy, w, g)
    xr = torch.zeros(B, C, H, H, device=dev, requires_grad=True)
    F.conv2d(xr, w.float().permute(0, 3, 1, 2), stride=stride, padding=pad).backward(dy.float().permute(0, 3, 1, 2))
    rdx = xr.grad.permute(0, 2, 3, 1)
    torch.testing.assert_close(dx.float(), rdx, atol=2e-2 * rdx.abs().max().item(), rtol=2e-2)


@pytest.mark.parametrize("B,H,C,CO,k,stride", [(8, 56, 64, 256, 1, 1), (16, 28, 256, 512, 1, 2),
                                               (32, 28, 128, 128, 3, 1)])
def test_conv_dgrad_addend_epilogue(B, H, C, CO, k, stride):
    """A shortcut's gradient passed as `addend` is added in the dgrad epilogue (no separate add)."""
    torch.manual_seed(9)
    pad = k // 2
    x = torch.randn(B, H, H, C, device=dev).to(bf)
    w = (torch.randn(CO, k, k, C, device=dev) * 0.05).to(bf)
    g = K.conv_geom(x.shape, w.shape, (stride, stride), (pad, pad), (1, 1))
    dy = torch.randn(B, g[4], g[5], CO, device=dev).to(bf)
    add = torch.randn(B, H, H, C, device=dev).to(bf)
    plain = K.conv2d_dgrad(dy, w, g).float()
    fused = K.conv2d_dgrad(dy, w, g, addend=add).float()
    ref = plain + add.float()
    torch.testing.assert_close(fused, ref, atol=2e-2 * ref.abs().max().item(), rtol=2e-2)


def test_gg_n64_fwd_bnstats_and_path(monkeypatch):
    """The 256x64 gg tile with the BN-statistics epilogue (the stage-1 3x3 conv feeding a BatchNorm), and
    that the planner takes it (HOPSX_DISABLE=gg_n64 gives the same result on the other engine)."""
    torch.manual_seed(3)
    B, H, C, CO = 16, 56, 64, 64
    x = torch.randn(B, H, H, C, device=dev).to(bf)
    w = (torch.randn(CO, 3, 3, C, device=dev) * 0.05).to(bf)
    g = K.conv_geom(x.shape, w.shape, (1, 1), (1, 1), (1, 1))
    y = K.conv2d_fwd_bnstats(x, w, g)
    torch.cuda.synchronize()
    K.bn_acc(dev, CO).zero_()  # (the statistics are not consumed here: re-zero the shared accumulator)
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), padding=1).permute(0, 2, 3, 1)
    if y is not None:
        torch.testing.assert_close(y.float(), ref, atol=2e-2 * ref.abs().max().item(), rtol=2e-2)
    y1 = K.conv2d_fwd(x, w, g)
    monkeypatch.setenv("HOPSX_DISABLE", "gg_n64")
    y2 = K.conv2d_fwd(x, w, g)
    torch.testing.assert_close(y1.float(), y2.float(), atol=1e-2 * ref.abs().max().item(), rtol=1e-2)
