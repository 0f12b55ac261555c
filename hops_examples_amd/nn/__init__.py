"""Keras-flavoured layer set on top of the gfx950 kernels (NHWC images).

Layers mirror what the reference notebooks build with ``tf.keras.layers``
(Conv2D / MaxPooling2D / Dropout / Flatten / Dense with fused activations,
e.g. notebooks/ml/Experiment/Tensorflow/mnist.ipynb:154-164) and with
``torch.nn`` (notebooks/ml/Experiment/PyTorch/mnist.ipynb:118-134), but run on
hand-written MFMA kernels: the activation is fused into the producing GEMM's
epilogue and the weights are read from the ParamArena's bf16 shadow.
"""
from __future__ import annotations

import math

import torch
from torch import nn

from ..ops import functional as HF

__all__ = [
    "Linear", "Dense", "Conv2d", "Conv2D", "MaxPool2d", "MaxPooling2D", "Dropout", "Flatten", "BatchNorm2d",
    "GlobalAvgPool2d", "EmbeddingBag", "Activation", "Sequential", "functional",
]

functional = HF
Sequential = nn.Sequential


def _glorot(shape, fan_in, fan_out):
    lim = math.sqrt(6.0 / (fan_in + fan_out))
    return torch.empty(shape).uniform_(-lim, lim)


class Linear(nn.Module):
    """y = act(x W^T + b); W: [out, in]. ``activation`` in {None, 'relu', 'sigmoid', 'tanh'}."""

    def __init__(self, in_features, out_features, bias=True, activation=None, init="glorot", out_f32=False):
        super().__init__()
        self.in_features, self.out_features = in_features, out_features
        self.activation = activation
        self.out_f32 = out_f32
        if init == "glorot":
            w = _glorot((out_features, in_features), in_features, out_features)
        else:  # torch default (kaiming-uniform a=sqrt(5))
            w = torch.empty(out_features, in_features)
            nn.init.kaiming_uniform_(w, a=math.sqrt(5))
        self.weight = nn.Parameter(w)
        self.weight._hx_wire_bf16 = True  # the kernels read it only through the bf16 shadow
        if bias:
            if init == "glorot":
                b = torch.zeros(out_features)
            else:
                bound = 1 / math.sqrt(in_features)
                b = torch.empty(out_features).uniform_(-bound, bound)
            self.bias = nn.Parameter(b)
        else:
            self.register_parameter("bias", None)

    # (p, salt) of a Dropout right before this layer that this layer applies (keras.Sequential sets it with
    # the Dropout module passing through): the logits layer's fused loss kernel then applies it
    _drop_in = None

    def forward(self, x):
        drop = self._drop_in if self.training else None
        return HF.linear(x, self.weight, self.bias, self.activation, self.out_f32, drop_in=drop)

    def extra_repr(self):
        return f"{self.in_features}, {self.out_features}, act={self.activation}"


Dense = Linear


class Conv2d(nn.Module):
    """NHWC conv; weight [out, kh, kw, in]. padding: int | 'valid' | 'same'."""

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, dilation=1, bias=True,
                 activation=None, init="glorot"):
        super().__init__()
        kh, kw = (kernel_size, kernel_size) if isinstance(kernel_size, int) else kernel_size
        self.cfg = dict(stride=stride, padding=padding, dilation=dilation)
        self.activation = activation
        self.in_affine = None  # (scale, shift) when this layer receives raw uint8 pixels
        # (pool,): the max-pool right after this conv runs in this conv's epilogue (keras.Sequential sets
        # it; a tuple, so the pool is not registered as a child module)
        self._pool_next = ()
        self.in_channels, self.out_channels, self.kernel_size = in_channels, out_channels, (kh, kw)
        fan_in, fan_out = in_channels * kh * kw, out_channels * kh * kw
        if init == "glorot":
            w = _glorot((out_channels, kh, kw, in_channels), fan_in, fan_out)
        elif init == "he":
            w = torch.randn(out_channels, kh, kw, in_channels) * math.sqrt(2.0 / fan_in)
        else:
            bound = 1 / math.sqrt(fan_in)
            w = torch.empty(out_channels, kh, kw, in_channels).uniform_(-bound, bound)
        self.weight = nn.Parameter(w)
        self.weight._hx_wire_bf16 = True  # the kernels read it only through the bf16 shadow
        if bias:
            self.bias = nn.Parameter(torch.zeros(out_channels) if init != "torch" else
                                     torch.empty(out_channels).uniform_(-1 / math.sqrt(fan_in), 1 / math.sqrt(fan_in)))
        else:
            self.register_parameter("bias", None)

    def forward(self, x, bnstats: bool = False, gslot=None):
        if self._pool_next and not bnstats and gslot is None:
            return conv_pool(self, self._pool_next[0], x)
        return self.conv_only(x, bnstats, gslot)

    def conv_only(self, x, bnstats: bool = False, gslot=None):
        w = self.weight
        if x.shape[-1] != self.in_channels:
            # an input laid out with zero channels beyond in_channels (models/resnet.py image stems: the
            # normalisation kernel writes 8 channels and tags the tensor): the weight is zero-padded to
            # match.  Any other channel mismatch (an RGBA image, a wrong layout) is an error, not data to drop.
            if getattr(x, "_hx_chpad", None) != self.in_channels or x.shape[-1] < self.in_channels:
                raise ValueError(f"Conv2d expects {self.in_channels} input channels (NHWC), got input of shape "
                                 f"{tuple(x.shape)}")
            w = HF.pad_input_channels(w, x.shape[-1])
        return HF.conv2d(x, w, self.bias, act=self.activation, in_affine=self.in_affine, bnstats=bnstats,
                         gslot=gslot, **self.cfg)

    def extra_repr(self):
        return f"{self.in_channels}, {self.out_channels}, k={self.kernel_size}, {self.cfg}, act={self.activation}"


Conv2D = Conv2d


class MaxPool2d(nn.Module):
    """NHWC max-pool; ``dropout`` > 0 fuses the Dropout that follows it in the
    reference models into the same kernel (mask regenerated in backward)."""

    def __init__(self, kernel_size, stride=None, padding=0, dropout=0.0):
        super().__init__()
        self.k, self.s, self.p = kernel_size, stride, padding
        self.dropout = float(dropout)
        self._absorbed = False  # run by the preceding conv (Conv2d._pool_next): a pass-through here
        _salt_counter[0] += 1
        self.salt = _salt_counter[0] * 7919

    def forward(self, x):
        return x if self._absorbed else self.pool_only(x)

    def pool_only(self, x):
        return HF.max_pool2d(x, self.k, self.s, self.p, self.dropout, self.training, self.salt)


MaxPooling2D = MaxPool2d


def conv_pool(conv: Conv2d, pool: MaxPool2d, x):
    """``pool(conv(x))`` as ONE fused launch when the pair qualifies (functional.conv2d_maxpool);
    parameters and results are those of the two modules applied in sequence."""
    if conv.in_affine is not None or x.dtype == torch.uint8 or x.shape[-1] != conv.in_channels:
        return pool.pool_only(conv.conv_only(x))
    return HF.conv2d_maxpool(x, conv.weight, conv.bias, act=conv.activation, pool_kernel=pool.k,
                             pool_stride=pool.s, pool_padding=pool.p, dropout_p=pool.dropout,
                             training=pool.training, salt=pool.salt, **conv.cfg)


def input_conv_pool(conv0: Conv2d, conv: Conv2d, pool: MaxPool2d, x):
    """``pool(conv(conv0(x)))`` where ``conv0`` is the network's input layer (raw uint8 images):
    ONE launch when the chain qualifies (functional.conv_input_maxpool: the input layer runs inside
    the second conv's operand gather), else ``conv_pool(conv, pool, conv0(x))``."""
    y = HF.conv_input_maxpool(x, conv0.weight, conv0.bias, conv0.activation, conv0.in_affine, conv0.cfg,
                              conv.weight, conv.bias, conv.activation, conv.cfg, pool_kernel=pool.k,
                              pool_stride=pool.s, pool_padding=pool.p, dropout_p=pool.dropout,
                              training=pool.training, salt=pool.salt)
    return y if y is not None else conv_pool(conv, pool, conv0.conv_only(x))


class GlobalAvgPool2d(nn.Module):
    def forward(self, x):
        return HF.global_avg_pool(x)


_salt_counter = [0]


class Dropout(nn.Module):
    """Counter-RNG dropout; the mask is regenerated (not stored) in backward."""

    def __init__(self, p=0.5):
        super().__init__()
        self.p = float(p)
        self._absorbed = False  # applied by the next Linear (its _drop_in): a pass-through here
        _salt_counter[0] += 1
        self.salt = _salt_counter[0] * 7919

    def forward(self, x):
        return x if self._absorbed else HF.dropout(x, self.p, self.training, self.salt)


class Flatten(nn.Module):
    def forward(self, x):
        return x.reshape(x.shape[0], -1)


class Activation(nn.Module):
    def __init__(self, act):
        super().__init__()
        self.act = act

    def forward(self, x):
        if self.act in (None, "linear"):
            return x
        if x.is_cuda:
            x = HF.to_compute(x)
            return {"relu": torch.relu, "sigmoid": torch.sigmoid, "tanh": torch.tanh}[self.act](x)
        return HF._cpu_act(x, self.act)


class BatchNorm2d(nn.Module):
    """NHWC batch norm; ``forward(x, residual=None)`` computes act(bn(x) + residual)."""

    def __init__(self, num_features, momentum=0.1, eps=1e-5, activation=None, zero_init=False):
        super().__init__()
        self.weight = nn.Parameter(torch.zeros(num_features) if zero_init else torch.ones(num_features))
        self.bias = nn.Parameter(torch.zeros(num_features))
        self.register_buffer("running_mean", torch.zeros(num_features))
        self.register_buffer("running_var", torch.ones(num_features))
        self.momentum, self.eps, self.activation = momentum, eps, activation

    def forward(self, x, residual=None, gslot=None, fold_next=False):
        return HF.batch_norm(x, self.weight, self.bias, self.running_mean, self.running_var, self.training,
                             self.momentum, self.eps, residual, self.activation, gslot=gslot, fold_next=fold_next)


class EmbeddingBag(nn.Module):
    def __init__(self, num_embeddings, embedding_dim, mode="sum", init_std=None):
        super().__init__()
        std = init_std if init_std is not None else 1.0 / math.sqrt(embedding_dim)
        self.weight = nn.Parameter(torch.randn(num_embeddings, embedding_dim) * std)
        self.mode = mode

    def forward(self, idx, offsets=None):
        return HF.embedding_bag(idx, self.weight, offsets, self.mode)
