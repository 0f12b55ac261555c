"""MNIST / Fashion-MNIST CNNs from the reference notebooks, NHWC, on hopsx layers.

* :class:`KerasMnistCNN`   — E1, notebooks/ml/Experiment/Tensorflow/mnist.ipynb:154-164
  (Conv32 k4 → Conv64 k4 → MaxPool4 → Drop .5 → Dense128 → Drop .5 → Dense10; 239,594 params).
  ``kernel``/``pool``/``dropout`` are the hyper-parameters the maggy/DE searches tune
  (notebooks/ml/Parallel_Experiments/Maggy/maggy-fashion-mnist-example.ipynb:188-240).
* :class:`MirroredMnistCNN` — E3/E5, the MirroredStrategy / MultiWorkerMirrored model
  (notebooks/ml/Distributed_Training/mirrored_strategy/mirroredstrategy_mnist_example.ipynb:189-207;
  Conv32 k2 → Conv64 k2 → MaxPool2 → Drop .01 → Dense128 → Dense10; 1,394,282 params).
  This is the flagship benchmark model.
* :class:`FashionMnistCNN`  — E8/E9 grid search / evolutionary search model with 'same' convs
  (…/grid_search_fashion_mnist.ipynb:224-236; 1,625,866 params at k3/pool2).
* :class:`TorchMnistNet`    — E2/E10 PyTorch ``Net`` (notebooks/ml/Experiment/PyTorch/mnist.ipynb:118-134;
  431,080 params), log-softmax head.

Inputs: uint8 or float images, [B, 28, 28] / [B, 28, 28, 1] / [B, 784]; uint8 is
normalised on the GPU by the landing kernel (x * scale + shift).
"""
from __future__ import annotations

import torch
from torch import nn

from .. import nn as hnn
from ..ops import functional as HF
from ..ops import kernels as K


def _as_nhwc(x: torch.Tensor) -> torch.Tensor:
    if x.dim() == 2:
        x = x.view(x.shape[0], 28, 28, 1)
    elif x.dim() == 3:
        x = x.unsqueeze(-1)
    return x


class _ImageModel(nn.Module):
    """uint8 images go straight into conv1, which applies ``x * input_scale + input_shift``
    itself (fused into its kernels on the GPU when the layer qualifies)."""

    input_scale = 1.0 / 255.0
    input_shift = 0.0

    def __init__(self):
        super().__init__()

    def _set_input_affine(self):
        self.conv1.in_affine = (self.input_scale, self.input_shift)

    def prep(self, x):
        return _as_nhwc(x)


class KerasMnistCNN(_ImageModel):
    def __init__(self, kernel=4, pool=4, dropout=0.5, num_classes=10, in_hw=28):
        super().__init__()
        self.conv1 = hnn.Conv2d(1, 32, kernel, activation="relu")
        self.conv2 = hnn.Conv2d(32, 64, kernel, activation="relu")
        self.pool = hnn.MaxPool2d(pool, dropout=dropout)  # MaxPool + Dropout fused
        s = (in_hw - 2 * (kernel - 1)) // pool
        self.fc1 = hnn.Dense(s * s * 64, 128, activation="relu")
        self.drop2 = hnn.Dropout(dropout)
        self.fc2 = hnn.Dense(128, num_classes)
        self._set_input_affine()

    def forward(self, x):
        x = hnn.input_conv_pool(self.conv1, self.conv2, self.pool, self.prep(x))
        return self.fc2(self.drop2(self.fc1(x.reshape(x.shape[0], -1))))


class MirroredMnistCNN(_ImageModel):
    input_shift = -0.5  # image / 255 - 0.5 (mirroredstrategy_mnist_example.ipynb:163-173)

    def __init__(self, num_classes=10):
        super().__init__()
        self.conv1 = hnn.Conv2d(1, 32, 2, activation="relu")
        self.conv2 = hnn.Conv2d(32, 64, 2, activation="relu")
        self.pool = hnn.MaxPool2d(2, dropout=0.01)  # MaxPool2D + Dropout(0.01) fused
        self.fc1 = hnn.Dense(13 * 13 * 64, 128, activation="relu")
        self.fc2 = hnn.Dense(128, num_classes)
        self._set_input_affine()

    def forward(self, x):
        x = hnn.input_conv_pool(self.conv1, self.conv2, self.pool, self.prep(x))  # conv1 + conv2 + pool + dropout: 1 launch
        return self.fc2(self.fc1(x.reshape(x.shape[0], -1)))


class FashionMnistCNN(_ImageModel):
    def __init__(self, kernel=3, pool=2, dropout=0.45, num_classes=10, in_hw=28):
        super().__init__()
        self.conv1 = hnn.Conv2d(1, 32, kernel, padding="same", activation="relu")
        self.conv2 = hnn.Conv2d(32, 64, kernel, padding="same", activation="relu")
        self.pool = hnn.MaxPool2d(pool, dropout=dropout)
        s = in_hw // pool
        self.fc1 = hnn.Dense(s * s * 64, 128, activation="relu")
        self.drop2 = hnn.Dropout(dropout)
        self.fc2 = hnn.Dense(128, num_classes)
        self._set_input_affine()

    def forward(self, x):
        x = hnn.input_conv_pool(self.conv1, self.conv2, self.pool, self.prep(x))
        return self.fc2(self.drop2(self.fc1(x.reshape(x.shape[0], -1))))


class TorchMnistNet(_ImageModel):
    """torchvision Normalize((0.1307,), (0.3081,)) is folded into the landing kernel."""

    input_scale = 1.0 / 255.0 / 0.3081
    input_shift = -0.1307 / 0.3081

    def __init__(self, num_classes=10):
        super().__init__()
        self.conv1 = hnn.Conv2d(1, 20, 5, activation="relu", init="torch")
        self.conv2 = hnn.Conv2d(20, 50, 5, activation="relu", init="torch")
        self.fc1 = hnn.Linear(4 * 4 * 50, 500, activation="relu", init="torch")
        self.fc2 = hnn.Linear(500, num_classes, init="torch")
        self._set_input_affine()

    def forward(self, x):
        x = HF.max_pool2d(self.conv1(self.prep(x)), 2)
        x = HF.max_pool2d(self.conv2(x), 2)
        return self.fc2(self.fc1(x.reshape(x.shape[0], -1)))


def param_count(m: nn.Module) -> int:
    return sum(p.numel() for p in m.parameters())
