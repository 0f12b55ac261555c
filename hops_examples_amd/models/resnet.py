"""ResNets on the gfx950 kernels (NHWC, bf16 activations, fp32 master weights).

* ``cifar_resnet(depth)`` — CIFAR-10 ResNet-20/32/44/56/110 (He et al. 2016, 6n+2 layers,
  widths 16/32/64, 1x1-conv projection shortcuts).  The reference names a CIFAR-10 ResNet
  trained with ``experiment.collective_allreduce`` only in prose (SURVEY §0.5,
  README.md / BASELINE.json config 5), so the architecture is the standard one.
* ``resnet50()`` — ImageNet ResNet-50 v1.5 (stride on the 3x3 conv; 25,557,032 params),
  the model of the reference benchmark notebook (notebooks/ml/Benchmarks/benchmark.ipynb).

MI355X mapping: every conv is the implicit-GEMM MFMA kernel with no bias (BN follows) whose
epilogue also accumulates the BN batch statistics (sum / sum of squares per channel);
BatchNorm then runs ONE fused NHWC kernel that finalizes them and applies
``act(bn(x) + residual)`` in one pass, so the residual add and the ReLU of every block
cost no extra kernel or HBM round trip; the classifier head is global-average-pool + the MFMA linear kernel.
"""
from __future__ import annotations

import os

import torch
from torch import nn

from .. import nn as hnn
from ..ops import functional as HF


class ConvBN(nn.Module):
    def __init__(self, cin, cout, k, stride=1, act="relu"):
        super().__init__()
        self.conv = hnn.Conv2d(cin, cout, k, stride=stride, padding=k // 2, bias=False, init="he")
        self.bn = hnn.BatchNorm2d(cout, activation=act)

    def forward(self, x, residual=None, gslot=None, res_gslot=None, sole=False, fold_next=False):
        # training: the conv epilogue accumulates the BN statistics (functional.conv2d bnstats), so
        # the BN is one apply launch instead of a statistics pass + an apply.  gslot / res_gslot:
        # see BasicBlock.forward.  sole: this conv is the only autograd consumer of x (when x is a BN
        # output, the conv's dgrad epilogue then reduces that BN's backward column sums).  fold_next: the
        # output goes only to the next ConvBN, whose conv applies this BN in its operand gather
        if sole:
            HF.bn_sole_consumer(x)
        return self.bn(self.conv(x, bnstats=self.bn.training, gslot=gslot), residual, gslot=res_gslot,
                       fold_next=fold_next)


def _fuse_proj(block, x) -> bool:
    return (block.training and x.is_cuda and torch.is_grad_enabled() and x.requires_grad
            and "proj_addend" not in os.environ.get("HOPSX_DISABLE", ""))


class BasicBlock(nn.Module):
    expansion = 1
    # a's BN apply is folded into b's conv (functional.batch_norm fold_next) from this width up: measured on
    # ResNet-20 B=128 (profiles/r6_bn_fold_resnet20.txt), conv + apply 14.8 -> 12.6 us at 32 channels but
    # 14.9 -> 16.8 us at 16 (4x the pixels: the gather applies the BN once per tap, 9x per element)
    fold_min_width = 32

    def __init__(self, cin, cout, stride=1):
        super().__init__()
        self.a = ConvBN(cin, cout, 3, stride)
        self.b = ConvBN(cout, cout, 3, 1)  # relu applied after the residual add
        self.short = ConvBN(cin, cout, 1, stride, act=None) if (stride != 1 or cin != cout) else None

    def forward(self, x):
        # a's BN output feeds only b's conv: where that conv has the direct MFMA forward (K = 9 * cout <= 512:
        # the 16 / 32-channel CIFAR stages) and cout >= fold_min_width, a's BN apply runs inside it
        # (functional.batch_norm fold_next)
        cout = self.b.conv.weight.shape[0]
        fn = self.training and x.is_cuda and 9 * cout <= 512 and cout >= self.fold_min_width
        if self.short is None and self.training and x.is_cuda and torch.is_grad_enabled() and \
                "res_addend" not in os.environ.get("HOPSX_DISABLE", ""):
            # identity shortcut: the residual's gradient (from b's BN backward, which always runs
            # first) is handed to a's conv backward, whose dgrad epilogue adds it — no autograd add
            # (a's conv is then x's only autograd consumer, and b's conv always is a's output's)
            slot = {}
            return self.b(self.a(x, gslot=slot, sole=True, fold_next=fn), residual=x, res_gslot=slot, sole=True)
        if self.short is not None and _fuse_proj(self, x):
            # projection shortcut: conv a's dX goes to the short conv's dgrad epilogue (backpropagated
            # after a's: created first), not to an autograd add (ops.functional.GiveGrad)
            slot = {}
            s = self.short(x, gslot=slot)
            return self.b(self.a(x, gslot=HF.GiveGrad(slot), fold_next=fn), residual=s, sole=True)
        s = x if self.short is None else self.short(x)
        return self.b(self.a(x, fold_next=fn), residual=s, sole=True)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, cin, width, stride=1):
        super().__init__()
        cout = width * 4
        self.a = ConvBN(cin, width, 1)
        self.b = ConvBN(width, width, 3, stride)
        self.c = ConvBN(width, cout, 1)
        self.short = ConvBN(cin, cout, 1, stride, act=None) if (stride != 1 or cin != cout) else None

    def forward(self, x):
        if self.short is None and self.training and x.is_cuda and torch.is_grad_enabled() and \
                "res_addend" not in os.environ.get("HOPSX_DISABLE", ""):
            # identity shortcut: c's BN backward hands the residual's gradient to a's (1x1) dgrad,
            # whose vectorized epilogue adds it (gemm_glds.h store8) — no autograd add launch
            slot = {}
            return self.c(self.b(self.a(x, gslot=slot, sole=True), sole=True), residual=x, res_gslot=slot,
                          sole=True)
        if self.short is not None and _fuse_proj(self, x):  # (see BasicBlock.forward)
            slot = {}
            s = self.short(x, gslot=slot)
            return self.c(self.b(self.a(x, gslot=HF.GiveGrad(slot)), sole=True), residual=s, sole=True)
        s = x if self.short is None else self.short(x)
        return self.c(self.b(self.a(x), sole=True), residual=s, sole=True)


class CifarResNet(nn.Module):
    def __init__(self, depth: int = 20, num_classes: int = 10, widths=(16, 32, 64)):
        super().__init__()
        if (depth - 2) % 6:
            raise ValueError("CIFAR ResNet depth must be 6n+2")
        n = (depth - 2) // 6
        self.stem = ConvBN(3, widths[0], 3)
        blocks, cin = [], widths[0]
        for i, w in enumerate(widths):
            for j in range(n):
                blocks.append(BasicBlock(cin, w, 2 if (j == 0 and i > 0) else 1))
                cin = w
        self.blocks = nn.Sequential(*blocks)
        self.pool = hnn.GlobalAvgPool2d()
        self.fc = hnn.Linear(cin, num_classes, init="torch", out_f32=True)
        self.depth = depth
        _norm_buffers(self, "cifar")

    def forward(self, x):
        x = _as_nhwc_image(x, self)
        return self.fc(self.pool(self.blocks(self.stem(x))))


class ResNet50(nn.Module):
    def __init__(self, num_classes: int = 1000, layers=(3, 4, 6, 3)):
        super().__init__()
        self.stem = ConvBN(3, 64, 7, 2)
        self.maxpool = hnn.MaxPool2d(3, 2, 1)
        blocks, cin = [], 64
        for i, (nb, w) in enumerate(zip(layers, (64, 128, 256, 512))):
            for j in range(nb):
                blocks.append(Bottleneck(cin, w, 2 if (j == 0 and i > 0) else 1))
                cin = w * 4
        self.blocks = nn.Sequential(*blocks)
        self.pool = hnn.GlobalAvgPool2d()
        self.fc = hnn.Linear(cin, num_classes, init="torch", out_f32=True)
        _norm_buffers(self, "caffe")

    def forward(self, x):
        x = _as_nhwc_image(x, self)
        return self.fc(self.pool(self.blocks(self.maxpool(self.stem(x)))))


# per-channel input normalisation of the two model families (uint8 NHWC pixels in):
#   cifar : (x / 255 - mean) / std with the CIFAR-10 statistics
#   caffe : Keras ResNet50 preprocess_input — RGB -> BGR, minus the ImageNet BGR means, no scaling
#           (notebooks/ml/Inference/Inference_Hello_World.ipynb:263-266); inference.preprocess_input
#           produces exactly this float tensor on the host, which the model then takes unchanged
_NORM = {
    "cifar": dict(mean=(0.4914, 0.4822, 0.4465), std=(0.2470, 0.2435, 0.2616), scale255=True, reverse=False),
    "caffe": dict(mean=(103.939, 116.779, 123.68), std=(1.0, 1.0, 1.0), scale255=False, reverse=True),
}


def _norm_buffers(m, kind: str = "cifar"):
    """Per-channel scale/shift of the input normalisation, kept on the module (host floats: the
    normalisation kernel takes them by value, so it is capture-safe)."""
    spec = _NORM[kind]
    m.img_norm = kind
    m.img_reverse = spec["reverse"]
    m.img_scale_c = [1.0 / ((255.0 if spec["scale255"] else 1.0) * s) for s in spec["std"]]
    m.img_shift_c = [-mu / s for mu, s in zip(spec["mean"], spec["std"])]


def _as_nhwc_image(x, m):
    """uint8 NHWC images are normalised per channel on the device (one hopsx kernel: bf16 out);
    float inputs are taken as already preprocessed."""
    import torch

    if x.dtype != torch.uint8:
        return x
    if x.is_cuda:
        from ..ops import kernels as K

        # 8 output channels (3..7 zero): the stem conv then runs on the C % 8 == 0 MFMA paths with its
        # weight zero-padded to match (nn.Conv2d), instead of the generic narrow-channel gather
        cout = 8 if "stem_pad" not in os.environ.get("HOPSX_DISABLE", "") else None
        y = K.u8_normalize_chan(x.contiguous(), m.img_scale_c, m.img_shift_c, reverse=m.img_reverse, cout=cout)
        if cout:
            y._hx_chpad = x.shape[-1]  # channels beyond this are zero (nn.Conv2d pads its weight only then)
        return y
    y = x.float()
    if m.img_reverse:
        y = y.flip(-1)
    return y * torch.tensor(m.img_scale_c) + torch.tensor(m.img_shift_c)


def cifar_resnet(depth: int = 20, num_classes: int = 10) -> CifarResNet:
    return CifarResNet(depth, num_classes)


def resnet50(num_classes: int = 1000) -> ResNet50:
    return ResNet50(num_classes)
