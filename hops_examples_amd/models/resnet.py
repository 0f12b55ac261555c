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


class ConvBN(nn.Module):
    def __init__(self, cin, cout, k, stride=1, act="relu"):
        super().__init__()
        self.conv = hnn.Conv2d(cin, cout, k, stride=stride, padding=k // 2, bias=False, init="he")
        self.bn = hnn.BatchNorm2d(cout, activation=act)

    def forward(self, x, residual=None, gslot=None, res_gslot=None):
        # training: the conv epilogue accumulates the BN statistics (functional.conv2d bnstats), so
        # the BN is one apply launch instead of a statistics pass + an apply.  gslot / res_gslot:
        # see BasicBlock.forward
        return self.bn(self.conv(x, bnstats=self.bn.training, gslot=gslot), residual, gslot=res_gslot)


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, cin, cout, stride=1):
        super().__init__()
        self.a = ConvBN(cin, cout, 3, stride)
        self.b = ConvBN(cout, cout, 3, 1)  # relu applied after the residual add
        self.short = ConvBN(cin, cout, 1, stride, act=None) if (stride != 1 or cin != cout) else None

    def forward(self, x):
        if self.short is None and self.training and x.is_cuda and torch.is_grad_enabled() and \
                "res_addend" not in os.environ.get("HOPSX_DISABLE", ""):
            # identity shortcut: the residual's gradient (from b's BN backward, which always runs
            # first) is handed to a's conv backward, whose dgrad epilogue adds it — no autograd add
            slot = {}
            return self.b(self.a(x, gslot=slot), residual=x, res_gslot=slot)
        s = x if self.short is None else self.short(x)
        return self.b(self.a(x), residual=s)


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
        s = x if self.short is None else self.short(x)
        return self.c(self.b(self.a(x)), residual=s)


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
        _norm_buffers(self)

    def forward(self, x):
        x = _as_nhwc_image(x, self.img_shift, self.img_scale)
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
        _norm_buffers(self)

    def forward(self, x):
        x = _as_nhwc_image(x, self.img_shift, self.img_scale)
        return self.fc(self.pool(self.blocks(self.maxpool(self.stem(x)))))


_MEAN = (0.4914, 0.4822, 0.4465)
_STD = (0.2470, 0.2435, 0.2616)


def _norm_buffers(m):
    """Per-channel (x/255 - mean)/std folded into one scale/shift pair, kept as buffers so the
    normalisation is capture-safe (no host->device constants inside a hipGraph)."""
    import torch

    std = torch.tensor(_STD)
    m.register_buffer("img_scale", 1.0 / (255.0 * std), persistent=False)
    m.register_buffer("img_shift", -torch.tensor(_MEAN) / std, persistent=False)


def _as_nhwc_image(x, shift, scale):
    """uint8 NHWC images are normalised per channel on the device; float inputs pass through."""
    import torch

    if x.dtype == torch.uint8:
        y = torch.addcmul(shift, x, scale)  # one fused elementwise pass: shift + x * scale
        return y.to(torch.bfloat16) if x.is_cuda else y
    return x


def cifar_resnet(depth: int = 20, num_classes: int = 10) -> CifarResNet:
    return CifarResNet(depth, num_classes)


def resnet50(num_classes: int = 1000) -> ResNet50:
    return ResNet50(num_classes)
