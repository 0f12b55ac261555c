"""Strided conv dgrad as dense parity-class GEMMs (csrc/ops/gemm_glds.h GgDgradParA, conv.hip
gg_dgrad_par) against the fp32 PyTorch reference of the same op (torch.nn.grad.conv2d_input on the
bf16-rounded operands), and against the zero-inserting path it replaces (HOPSX_DISABLE=dgrad_par).
Shapes: the ResNet-50 stride-2 3x3 convs (stage entries) at gg-engine sizes, an odd input size (the
classes have unequal row counts), a 5x5 / stride-2 kernel, the fused act' and added gradient.
"""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from hops_examples_amd.ops import kernels as K  # noqa: E402

dev = torch.device("cuda", 0)
BF = torch.bfloat16


def _case(B, H, C, CO, k, s, p, seed, yprev=False, addend=False, disable=""):
    g = torch.Generator(device="cpu").manual_seed(seed)
    geom = K.conv_geom((B, H, H, C), (CO, k, k, C), (s, s), (p, p), (1, 1))
    OH = geom[4]
    dy = torch.randn(B, OH, OH, CO, generator=g).to(dev, BF)
    w = (torch.randn(CO, k, k, C, generator=g) * (2.0 / (k * k * C)) ** 0.5).to(dev, BF)
    yp = torch.relu(torch.randn(B, H, H, C, generator=g)).to(dev, BF) if yprev else None
    ad = torch.randn(B, H, H, C, generator=g).to(dev, BF) if addend else None
    old = os.environ.get("HOPSX_DISABLE", "")
    os.environ["HOPSX_DISABLE"] = disable
    try:
        dx = K.conv2d_dgrad(dy, w, geom, yprev=yp, act_prev="relu" if yprev else 0, addend=ad)
        torch.cuda.synchronize()
    finally:
        os.environ["HOPSX_DISABLE"] = old
    ref = torch.nn.grad.conv2d_input((B, C, H, H), w.float().permute(0, 3, 1, 2), dy.float().permute(0, 3, 1, 2),
                                     stride=s, padding=p).permute(0, 2, 3, 1)
    if yp is not None:
        ref = ref * (yp.float() > 0)
    if ad is not None:
        ref = ref + ad.float()
    return dx.float(), ref


@pytest.mark.parametrize("B,H,C,CO,k,s,p,yprev,addend", [
    (32, 28, 128, 128, 3, 2, 1, False, False),  # ResNet-50 stage-3 entry (B=32)
    (16, 56, 64, 64, 3, 2, 1, True, False),     # stage-2 entry at half batch, fused relu'
    (32, 27, 128, 64, 3, 2, 1, False, True),    # odd size: 14 even / 13 odd rows per class, addend
    (16, 32, 128, 128, 5, 2, 2, True, True),    # 5x5 / stride 2: 9 / 6 / 6 / 4 taps per class
    (32, 56, 256, 512, 1, 2, 0, False, True),   # 1x1 / stride 2 projection: one class, three filled
    (32, 28, 128, 256, 1, 2, 0, True, False),
])
def test_strided_dgrad_parity_classes_match_reference(B, H, C, CO, k, s, p, yprev, addend):
    dx, ref = _case(B, H, C, CO, k, s, p, seed=H + k, yprev=yprev, addend=addend)
    err = (dx - ref).abs().max().item()
    scale = ref.abs().max().item()
    # bf16 output rounding (2^-8 relative) + fp32 accumulation over k*k*CO / 4 products
    assert err <= 1e-2 * scale, (err, scale)
    old, _ = _case(B, H, C, CO, k, s, p, seed=H + k, yprev=yprev, addend=addend, disable="dgrad_par")
    # the zero-inserting path computes the same sums (plus exact zeros): equal up to fp32 order
    assert (dx - old).abs().max().item() <= 1e-2 * scale
