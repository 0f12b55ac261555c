"""A Keras-style front end (``Sequential`` + ``compile``/``fit``/``evaluate``/``predict``)
over the hopsx engine: layers resolve to the MFMA kernel layers in :mod:`hops_examples_amd.nn`,
``fit`` drives a hipGraph-captured :class:`~hops_examples_amd.runtime.step.TrainStep` with a
fused optimizer, and metrics stay on the device until the epoch ends.

The reference notebooks build almost every model this way
(notebooks/ml/Experiment/Tensorflow/mnist.ipynb:154-190, …/Maggy/maggy-fashion-mnist-example.ipynb:214-265,
…/Maggy/maggy-ablation-titanic-example.ipynb:196-430, notebooks/ml/Benchmarks/benchmark.ipynb:140-170),
so a user can port a notebook by swapping ``tf.keras`` for ``hops_examples_amd.keras``.

MI355X-specific choices:
  * layer specs are lazy (Keras infers ``in_features``), so ablations can drop layers by name
    and the model is materialised once with concrete shapes;
  * a final ``softmax``/``sigmoid`` activation feeding a cross-entropy loss is folded into the
    fused loss kernel (logits in, probabilities never materialised during training); ``predict``
    applies it explicitly;
  * ``MaxPooling2D`` followed by ``Dropout`` becomes one fused pool+dropout kernel.
"""
from __future__ import annotations

import os
import time
from pathlib import Path

import numpy as np
import torch
from torch import nn as tnn

from . import nn as hnn
from . import optim as hoptim
from .ops import functional as HF

# --------------------------------------------------------------------------- layers


class Layer:
    _counts: dict = {}

    def __init__(self, name=None, input_shape=None, **_):
        kind = type(self).__name__.lower()
        if name is None:
            n = Layer._counts.get(kind, 0)
            Layer._counts[kind] = n + 1
            name = kind if n == 0 else f"{kind}_{n}"
        self.name = name
        self.input_shape = tuple(input_shape) if input_shape is not None else None
        self.module = None
        self.output_shape = None

    def build(self, in_shape: tuple) -> tuple:  # returns output shape (without batch)
        raise NotImplementedError

    def count_params(self) -> int:
        return sum(p.numel() for p in self.module.parameters()) if self.module is not None else 0


def _act(a):
    if a is None or a == "linear":
        return None
    return a


class Dense(Layer):
    def __init__(self, units, activation=None, use_bias=True, name=None, input_shape=None, input_dim=None,
                 kernel_initializer="glorot_uniform", **kw):
        super().__init__(name, input_shape if input_dim is None else (input_dim,), **kw)
        self.units, self.activation, self.use_bias = int(units), activation, use_bias
        self.init = "glorot" if "glorot" in str(kernel_initializer) else "torch"

    def build(self, in_shape):
        act = _act(self.activation)
        fused = act if act in ("relu", "sigmoid", "tanh") else None
        lin = hnn.Linear(int(np.prod(in_shape)), self.units, bias=self.use_bias, activation=fused, init=self.init)
        self.module = lin if (act == fused) else tnn.Sequential(lin, _Softmax() if act == "softmax" else hnn.Activation(act))
        return (self.units,)


class Conv2D(Layer):
    def __init__(self, filters, kernel_size, strides=1, padding="valid", activation=None, use_bias=True,
                 name=None, input_shape=None, dilation_rate=1, **kw):
        super().__init__(name, input_shape, **kw)
        self.filters = int(filters)
        self.k = (kernel_size, kernel_size) if isinstance(kernel_size, int) else tuple(kernel_size)
        self.s = strides if isinstance(strides, int) else strides[0]
        self.padding, self.activation, self.use_bias, self.d = padding, activation, use_bias, dilation_rate

    def build(self, in_shape):
        H, W, C = in_shape
        self.module = hnn.Conv2d(C, self.filters, self.k, stride=self.s, padding=self.padding,
                                 dilation=self.d, bias=self.use_bias, activation=_act(self.activation))
        if self.padding == "same":
            Ho, Wo = -(-H // self.s), -(-W // self.s)
        else:
            Ho = (H - self.d * (self.k[0] - 1) - 1) // self.s + 1
            Wo = (W - self.d * (self.k[1] - 1) - 1) // self.s + 1
        return (Ho, Wo, self.filters)


class MaxPooling2D(Layer):
    def __init__(self, pool_size=(2, 2), strides=None, padding="valid", name=None, **kw):
        super().__init__(name, **kw)
        self.k = pool_size if isinstance(pool_size, int) else pool_size[0]
        self.s = self.k if strides is None else (strides if isinstance(strides, int) else strides[0])
        self.padding = padding
        self.dropout = 0.0

    def build(self, in_shape):
        H, W, C = in_shape
        p = (self.k - 1) // 2 if self.padding == "same" else 0
        self.module = hnn.MaxPool2d(self.k, self.s, p, dropout=self.dropout)
        return ((H + 2 * p - self.k) // self.s + 1, (W + 2 * p - self.k) // self.s + 1, C)


class Dropout(Layer):
    def __init__(self, rate, name=None, **kw):
        super().__init__(name, **kw)
        self.rate = float(rate)

    def build(self, in_shape):
        self.module = hnn.Dropout(self.rate)
        return in_shape


class Flatten(Layer):
    def build(self, in_shape):
        self.module = hnn.Flatten()
        return (int(np.prod(in_shape)),)


class Activation(Layer):
    def __init__(self, activation, name=None, **kw):
        super().__init__(name, **kw)
        self.activation = activation

    def build(self, in_shape):
        self.module = _Softmax() if self.activation == "softmax" else hnn.Activation(self.activation)
        return in_shape


class BatchNormalization(Layer):
    def __init__(self, momentum=0.99, epsilon=1e-3, name=None, **kw):
        super().__init__(name, **kw)
        self.momentum, self.eps = momentum, epsilon

    def build(self, in_shape):
        self.module = hnn.BatchNorm2d(in_shape[-1], momentum=1 - self.momentum, eps=self.eps)
        return in_shape


class GlobalAveragePooling2D(Layer):
    def build(self, in_shape):
        self.module = hnn.GlobalAvgPool2d()
        return (in_shape[-1],)


class Reshape(Layer):
    def __init__(self, target_shape, name=None, **kw):
        super().__init__(name, **kw)
        self.target = tuple(target_shape)

    def build(self, in_shape):
        t = self.target
        self.module = _Reshape(t)
        return t


class InputLayer(Layer):
    def __init__(self, input_shape=None, shape=None, name=None, **kw):
        super().__init__(name, input_shape if input_shape is not None else shape, **kw)

    def build(self, in_shape):
        self.module = tnn.Identity()
        return in_shape


def Input(shape, name=None):
    return InputLayer(shape=shape, name=name)


class _Softmax(tnn.Module):
    def forward(self, x):
        return torch.softmax(x.float(), dim=-1)


class _Reshape(tnn.Module):
    def __init__(self, t):
        super().__init__()
        self.t = t

    def forward(self, x):
        return x.reshape(x.shape[0], *self.t)


class _InputNorm(tnn.Module):
    """uint8 inputs are normalised to [0,1] on the device (one vectorised kernel) — or, when the first
    layer is a conv that applies the normalisation itself (``raw_u8``: its ``in_affine``), passed on raw."""

    raw_u8 = False

    def forward(self, x):
        if x.dtype == torch.uint8 and self.raw_u8:
            return x
        if x.dtype == torch.uint8:
            if x.is_cuda:
                from .ops import kernels as K

                return K.u8_normalize(x.contiguous(), 1.0 / 255.0, 0.0)
            return x.float() / 255.0
        return HF.to_compute(x) if x.is_cuda else x.float()


class layers:  # noqa: N801  (namespace, like tf.keras.layers)
    Layer, Dense, Conv2D, MaxPooling2D, MaxPool2D, Dropout, Flatten = Layer, Dense, Conv2D, MaxPooling2D, \
        MaxPooling2D, Dropout, Flatten
    Activation, BatchNormalization, GlobalAveragePooling2D, Reshape, InputLayer, Input = \
        Activation, BatchNormalization, GlobalAveragePooling2D, Reshape, InputLayer, Input


# --------------------------------------------------------------------------- optimizers


class _OptSpec:
    cls = hoptim.SGD
    defaults: dict = {}
    rename = {"learning_rate": "lr", "rho": "rho", "epsilon": "eps"}

    def __init__(self, learning_rate=None, lr=None, **kw):
        self.kw = dict(self.defaults)
        if learning_rate is not None or lr is not None:
            self.kw["lr"] = float(learning_rate if learning_rate is not None else lr)
        for k, v in kw.items():
            self.kw[self.rename.get(k, k)] = v

    def make(self, module):
        return self.cls(module, **self.kw)


class _optimizers:  # noqa: N801
    class SGD(_OptSpec):
        cls, defaults = hoptim.SGD, {"lr": 0.01}

    class Adam(_OptSpec):
        cls, defaults = hoptim.Adam, {"lr": 0.001, "eps": 1e-7}
        rename = {"beta_1": "_b1", "beta_2": "_b2", "epsilon": "eps"}

        def make(self, module):
            kw = dict(self.kw)
            b1, b2 = kw.pop("_b1", 0.9), kw.pop("_b2", 0.999)
            kw.pop("amsgrad", None)
            return hoptim.Adam(module, betas=(b1, b2), **kw)

    class Adadelta(_OptSpec):
        cls, defaults = hoptim.Adadelta, {"lr": 1.0, "rho": 0.95, "eps": 1e-7}

    class RMSprop(_OptSpec):
        cls, defaults = hoptim.RMSprop, {"lr": 0.001, "alpha": 0.9, "eps": 1e-7}
        rename = {"rho": "alpha", "epsilon": "eps"}

    class Adagrad(_OptSpec):
        cls, defaults = hoptim.Adagrad, {"lr": 0.001, "eps": 1e-7, "initial_accumulator_value": 0.1}
        rename = {"epsilon": "eps"}

    class Ftrl(_OptSpec):
        cls, defaults = hoptim.Ftrl, {"lr": 0.001}
        rename = {"l1_regularization_strength": "l1", "l2_regularization_strength": "l2",
                  "initial_accumulator_value": "initial_accumulator_value"}


optimizers = _optimizers
_OPT_BY_NAME = {"sgd": _optimizers.SGD, "adam": _optimizers.Adam, "adadelta": _optimizers.Adadelta,
                "rmsprop": _optimizers.RMSprop, "adagrad": _optimizers.Adagrad, "ftrl": _optimizers.Ftrl}

_LOSS_ALIASES = {
    "sparse_categorical_crossentropy": "sparse_ce", "categorical_crossentropy": "ce",
    "binary_crossentropy": "bce", "mse": "mse", "mean_squared_error": "mse",
}


# --------------------------------------------------------------------------- callbacks


class Callback:
    model = None

    def set_model(self, model):
        self.model = model

    def on_train_begin(self, logs=None): ...
    def on_train_end(self, logs=None): ...
    def on_epoch_begin(self, epoch, logs=None): ...
    def on_epoch_end(self, epoch, logs=None): ...
    def on_batch_end(self, batch, logs=None): ...


class _TensorBoardCB(Callback):
    def __init__(self, log_dir=None, **_):
        from . import tensorboard as tb

        self.w = tb.SummaryWriter(log_dir or tb.logdir())

    def on_epoch_end(self, epoch, logs=None):
        for k, v in (logs or {}).items():
            self.w.add_scalar(f"epoch_{k}", v, epoch)
        self.w.flush()

    def on_train_end(self, logs=None):
        self.w.close()


class _ModelCheckpointCB(Callback):
    def __init__(self, filepath, monitor="val_loss", save_best_only=False, mode="auto", **_):
        self.filepath, self.monitor, self.best_only = str(filepath), monitor, save_best_only
        self.mode = mode if mode != "auto" else ("max" if "acc" in monitor else "min")
        self.best = None

    def on_epoch_end(self, epoch, logs=None):
        v = (logs or {}).get(self.monitor)
        if self.best_only and v is not None and self.best is not None:
            if (self.mode == "max" and v <= self.best) or (self.mode == "min" and v >= self.best):
                return
        self.best = v if v is not None else self.best
        self.model.save(self.filepath.format(epoch=epoch + 1, **(logs or {})))


class _EarlyStoppingCB(Callback):
    def __init__(self, monitor="val_loss", patience=0, min_delta=0.0, mode="auto", **_):
        self.monitor, self.patience, self.min_delta = monitor, patience, min_delta
        self.mode = mode if mode != "auto" else ("max" if "acc" in monitor else "min")
        self.best, self.wait = None, 0

    def on_epoch_end(self, epoch, logs=None):
        v = (logs or {}).get(self.monitor)
        if v is None:
            return
        better = self.best is None or (v > self.best + self.min_delta if self.mode == "max"
                                       else v < self.best - self.min_delta)
        if better:
            self.best, self.wait = v, 0
        else:
            self.wait += 1
            if self.wait > self.patience:
                self.model.stop_training = True


class callbacks:  # noqa: N801
    Callback, TensorBoard, ModelCheckpoint, EarlyStopping = Callback, _TensorBoardCB, _ModelCheckpointCB, \
        _EarlyStoppingCB


class History(Callback):
    def __init__(self):
        self.history: dict[str, list] = {}
        self.epoch: list[int] = []

    def on_epoch_end(self, epoch, logs=None):
        self.epoch.append(epoch)
        for k, v in (logs or {}).items():
            self.history.setdefault(k, []).append(v)


# --------------------------------------------------------------------------- model


def _default_device() -> torch.device:
    return torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")


def _fits_hbm(x, y, limit=8 << 30) -> bool:
    """Whole training arrays small enough to keep resident on the device during fit."""
    def nbytes(a):
        return a.numel() * a.element_size() if isinstance(a, torch.Tensor) else np.asarray(a).nbytes

    return os.environ.get("HOPSX_KERAS_DEVICE_BATCHES", "1") == "1" and nbytes(x) + nbytes(y) <= limit


def _batches(x, y, batch_size, shuffle, rng):
    n = len(x)
    idx = rng.permutation(n) if shuffle else np.arange(n)
    for s in range(0, n, batch_size):
        j = idx[s:s + batch_size]
        yield x[j], y[j]


def _to_tensor(a, dev, label=False):
    if isinstance(a, torch.Tensor):
        t = a
    else:
        a = np.asarray(a)
        t = torch.from_numpy(np.ascontiguousarray(a))
    if label:
        t = t.long() if t.dtype in (torch.int32, torch.int64, torch.int16, torch.uint8) and t.dim() == 1 else t.float()
    return t.to(dev, non_blocking=True)


class Sequential(tnn.Module):
    def __init__(self, layers_=None, name=None):
        super().__init__()
        self.name = name or "sequential"
        self._specs: list[Layer] = []
        self.net = None
        self.stop_training = False
        self.device = None
        self._opt_spec = None
        self._step = None
        self._final_act = None
        for l in layers_ or []:
            self.add(l)

    # ------------------------------------------------------------------ structure
    def add(self, layer: Layer):
        if self.net is not None:
            raise RuntimeError("cannot add layers after the model was built")
        self._specs.append(layer)

    @property
    def layers(self):
        return list(self._specs)

    def get_layer(self, name):
        for l in self._specs:
            if l.name == name:
                return l
        raise ValueError(f"no layer named {name!r}")

    def build(self, input_shape=None):
        if self.net is not None:
            return
        shape = input_shape or next((l.input_shape for l in self._specs if l.input_shape is not None), None)
        if shape is None:
            raise ValueError("input shape unknown: pass input_shape= to the first layer or call fit() first")
        shape = tuple(int(s) for s in shape if s is not None) if len(shape) and shape[0] is None else tuple(shape)
        specs = list(self._specs)
        for a, b in zip(specs, specs[1:]):  # fuse MaxPooling2D + Dropout
            if isinstance(a, MaxPooling2D) and isinstance(b, Dropout):
                a.dropout, b.rate = b.rate, 0.0
        mods = [_InputNorm()]
        if len(shape) == 2 and any(isinstance(l, Conv2D) for l in specs):
            shape = shape + (1,)
            mods.append(_Reshape(shape))
        for l in specs:
            if isinstance(l, Dense) and len(shape) > 1:
                mods.append(hnn.Flatten())
            shape = l.build(shape)
            l.output_shape = (None,) + tuple(shape)
            if not (isinstance(l, Dropout) and l.rate == 0.0):
                mods.append(l.module)
        # uint8 pixels go straight into a first conv, which applies x / 255 itself (fused into its kernel
        # where the layer qualifies): the same arithmetic as _InputNorm, one launch less, and the layout the
        # persistent MNIST engine expects (see _flagship_view)
        first = next((m for m in mods[1:] if not isinstance(m, _Reshape)), None)
        if isinstance(first, hnn.Conv2d) and first.in_affine is None:
            first.in_affine = (1.0 / 255.0, 0.0)
            mods[0].raw_u8 = True
        # Conv2D -> MaxPooling2D: the pool (+ its fused dropout) runs in the conv's epilogue where the pair
        # qualifies (functional.conv2d_maxpool; the unfused chain otherwise), the pool module passes through
        # Dropout -> Dense: the Dense applies the dropout to its input (HF.linear drop_in), which the logits
        # layer's fused loss kernel does in-kernel (no dropout launch forward or backward)
        dis = os.environ.get("HOPSX_DISABLE", "")
        for a, b in zip(mods, mods[1:]):
            if isinstance(a, hnn.Conv2d) and isinstance(b, hnn.MaxPool2d) and "keras_conv_pool" not in dis:
                a._pool_next, b._absorbed = (b,), True
            lin = b[0] if isinstance(b, tnn.Sequential) and len(b) and isinstance(b[0], hnn.Linear) else b
            if isinstance(a, hnn.Dropout) and isinstance(lin, hnn.Linear) and a.p > 0 and "keras_drop_in" not in dis:
                lin._drop_in, a._absorbed = (a.p, a.salt), True  # (Dense(softmax) is Sequential(Linear, softmax))
        self.net = tnn.Sequential(*mods)
        self._input_shape = shape

    def forward(self, x):
        return self.net(x)

    def count_params(self) -> int:
        return sum(p.numel() for p in self.net.parameters()) if self.net is not None else 0

    def summary(self, print_fn=print):
        print_fn(f'Model: "{self.name}"')
        print_fn("_" * 65)
        print_fn(f"{'Layer (type)':<30}{'Output Shape':<22}{'Param #':>10}")
        print_fn("=" * 65)
        for l in self._specs:
            print_fn(f"{l.name + ' (' + type(l).__name__ + ')':<30}{str(l.output_shape):<22}{l.count_params():>10}")
        print_fn("=" * 65)
        print_fn(f"Total params: {self.count_params():,}")

    # ------------------------------------------------------------------ compile / fit
    def compile(self, optimizer="rmsprop", loss="sparse_categorical_crossentropy", metrics=None, **_):
        self._opt_spec = _OPT_BY_NAME[optimizer.lower()]() if isinstance(optimizer, str) else optimizer
        self._loss_name = loss
        self._metrics = list(metrics or [])
        self._step = None
        self._fast = None

    def _flagship_view(self):
        """A MirroredMnistCNN-shaped view sharing this model's layers when the stack is the reference's
        MirroredStrategy MNIST CNN (mirroredstrategy_mnist_example.ipynb:189-207: Conv2D(32, 2, relu),
        Conv2D(64, 2, relu), MaxPooling2D + Dropout, Flatten, Dense(128, relu), Dense(10[, softmax])) —
        matched on the layers by runtime.persist.flagship_layers — else None."""
        from .models.mnist import MirroredMnistCNN
        from .runtime.persist import flagship_layers

        mods = [m for m in self.net if not isinstance(m, (_InputNorm, _Reshape, hnn.Flatten))]
        if len(mods) != 5:
            return None
        c1, c2, pool, f1, f2 = mods
        if isinstance(f2, tnn.Sequential) and len(f2) == 2 and isinstance(f2[1], _Softmax):
            f2 = f2[0]
        v = MirroredMnistCNN.__new__(MirroredMnistCNN)
        tnn.Module.__init__(v)
        v.conv1, v.conv2, v.pool, v.fc1, v.fc2 = c1, c2, pool, f1, f2
        return v if flagship_layers(v) is not None else None

    def _prepare_fast(self, batch_size):
        """The persistent whole-step engine (runtime.persist, via runtime.step.make_step) for fit's
        resident-epoch path when this model is the flagship MNIST CNN with sparse CE, Adadelta and
        batch 32 on a GPU that can hold its grid; else None (fit keeps the TrainStep)."""
        if self.device.type != "cuda" or self._kind != "sparse_ce":  # (HOPSX_PERSIST=0: supported() says no)
            return None
        view = self._flagship_view()
        if view is None:
            return None
        from .parallel import dist as hdist
        from .runtime.persist import PersistentMnistStep
        from .runtime.step import make_step

        view.train(self.training)
        if not PersistentMnistStep.supported(view, self.optimizer, int(batch_size), hdist.world_size()):
            return None
        eng = make_step(view, self.optimizer, self._kind, dp="auto", graph=True, batch=int(batch_size))
        return eng if getattr(eng, "kind", None) == "persistent" else None

    def _prepare(self, xb):
        if self.net is None:
            self.build(tuple(xb.shape[1:]))
        if self.device is None:
            self.device = _default_device()
            self.to(self.device)
            from .runtime.arena import ParamArena

            if self.device.type == "cuda":
                ParamArena.from_module(self, self.device)
        if self._step is None:
            if self._opt_spec is None:
                raise RuntimeError("call compile() before fit()")
            kind = _LOSS_ALIASES.get(self._loss_name, self._loss_name)
            last = self._specs[-1] if self._specs else None
            act = getattr(last, "activation", None)
            self._final_act = act
            self._train_fwd = None
            if act == "softmax" and kind in ("sparse_ce", "ce"):
                self._train_fwd = self._strip_last(_Softmax)
            elif act == "sigmoid" and kind == "bce":
                kind = "bce_logits"
                self._train_fwd = self._strip_sigmoid()
            self._kind = kind
            from .runtime.step import TrainStep

            self.optimizer = self._opt_spec.make(self)
            fwd = self._train_fwd
            self._step = TrainStep(self, self.optimizer, kind, graph=True,
                                   forward_fn=(lambda m, x: fwd(x)) if fwd is not None else None)
            self._fast = self._prepare_fast(self._batch_hint) if getattr(self, "_batch_hint", None) else None
            self.geom_batch = getattr(self, "_batch_hint", None)

    def _resident(self, x, y):
        """Device copies of a whole uint8 image array [N, 28, 28(, 1)] and its int labels, uploaded once
        and kept while fit is called with the same arrays."""
        key = (id(x), id(y), len(x))
        c = getattr(self, "_res_cache", None)
        if c is not None and c[0] == key:
            return c[1], c[2]
        xs = _to_tensor(x, self.device).reshape(len(x), 28, 28, 1).contiguous()
        ys = _to_tensor(y, self.device, label=True).reshape(-1).contiguous()
        self._res_cache = (key, xs, ys)
        return xs, ys

    def _device_batches(self, x, y, batch_size, shuffle, rng):
        key = (id(x), id(y), len(x), "any")
        c = getattr(self, "_res_any", None)
        if c is None or c[0] != key:
            xs = _to_tensor(x, self.device)
            ys = _to_tensor(y, self.device, label=True)
            self._res_any = c = (key, xs, ys)
        xs, ys = c[1], c[2]
        n = xs.shape[0]
        if shuffle:
            g = torch.Generator(device=self.device)
            g.manual_seed(int(rng.integers(1 << 62)))
            idx = torch.randperm(n, device=self.device, generator=g)
        else:
            idx = torch.arange(n, device=self.device)
        for s in range(0, n, batch_size):
            j = idx[s:s + batch_size]
            yield xs.index_select(0, j), ys.index_select(0, j)

    def _fit_epoch_resident(self, x, y, batch_size, shuffle, rng):
        """One epoch of the multi-kernel TrainStep on device-resident data: the epoch's shuffled batches are
        written into ONE persistent [nbatch, B, ...] buffer (so the captured multi-step graphs and the
        optimizer's next-batch prefetch stay bound to it), then ``run_resident`` replays
        steps_per_execution steps per graph launch with no per-batch host work; every step's loss /
        correct count is added on the device (``on_out``).  A partial last batch runs as one step."""
        st = self._step
        key = (id(x), id(y), len(x), "any")
        c = getattr(self, "_res_any", None)
        if c is None or c[0] != key:
            self._res_any = c = (key, _to_tensor(x, self.device), _to_tensor(y, self.device, label=True))
        xs_all, ys_all = c[1], self._labels(c[2])
        N, B = xs_all.shape[0], int(batch_size)
        nb = N // B
        buf = getattr(self, "_ep_buf", None)
        if buf is None or buf[0].shape != (nb, B) + tuple(xs_all.shape[1:]) or buf[1].shape != (nb, B) + tuple(ys_all.shape[1:]):
            buf = (torch.empty((nb, B) + tuple(xs_all.shape[1:]), device=self.device, dtype=xs_all.dtype),
                   torch.empty((nb, B) + tuple(ys_all.shape[1:]), device=self.device, dtype=ys_all.dtype))
            self._ep_buf = buf
        xs, ys = buf
        if shuffle:
            g = torch.Generator(device=self.device)
            g.manual_seed(int(rng.integers(1 << 62)))
            idx = torch.randperm(N, device=self.device, generator=g)
        else:
            idx = torch.arange(N, device=self.device)
        torch.index_select(xs_all, 0, idx[: nb * B], out=xs.view((nb * B,) + tuple(xs_all.shape[1:])))
        torch.index_select(ys_all, 0, idx[: nb * B], out=ys.view((nb * B,) + tuple(ys_all.shape[1:])))
        # the epoch starts at its first batch: the graph's static input buffers hold the batch the next
        # replay trains on (the previous epoch's prefetch), so they are refilled and the cursor reset
        st._rn = 0
        if st._cursor is not None and st._sx is not None and not isinstance(st._sx, (tuple, list)):
            st._sx.copy_(xs[0])
            st._sy.copy_(ys[0])
            st._cursor.zero_()
        tot_l = torch.zeros((), device=self.device)
        tot_c = torch.zeros((), device=self.device, dtype=torch.int64)

        def on_out(outs):  # one launch's steps: a stack + a sum per statistic, not ops per step
            tot_l.add_(torch.stack([o["loss"].reshape(()) for o in outs]).sum(), alpha=B)
            if outs[0].get("correct") is not None:
                tot_c.add_(torch.stack([o["correct"].reshape(()) for o in outs]).sum())

        st.prepare_resident(xs, ys, n=nb)
        st.run_resident(xs, ys, nb, on_out=on_out)
        if N > nb * B:
            j = idx[nb * B:]
            r = st(xs_all.index_select(0, j), ys_all.index_select(0, j))
            tot_l.add_(r["loss"].reshape(()), alpha=N - nb * B)
            if r.get("correct") is not None:
                tot_c.add_(r["correct"].reshape(()))
        return tot_l, tot_c, N, ys_all

    def _fit_epoch_fast(self, x, y, shuffle, rng):
        """One epoch on the persistent engine: the epoch's batches (shuffled on the device) resident in
        HBM, 32 steps per launch, per-step loss / correct read back once per launch on the device; a
        last partial batch goes through the TrainStep.  Returns device (sum of losses * n, correct, n)."""
        eng = self._fast
        xs_all, ys_all = self._resident(x, y)
        N = xs_all.shape[0]
        B = int(self.geom_batch)
        nb = N // B
        if shuffle:
            g = torch.Generator(device=self.device)
            g.manual_seed(int(rng.integers(1 << 62)))
            idx = torch.randperm(N, device=self.device, generator=g)
        else:
            idx = torch.arange(N, device=self.device)
        xs = xs_all.index_select(0, idx[: nb * B]).view(nb, B, 28, 28, 1)
        ys = ys_all.index_select(0, idx[: nb * B]).view(nb, B)
        eng.cursor.zero_()  # the epoch starts at its first batch
        tot = torch.zeros(2, device=self.device)
        left = nb
        while left > 0:
            k = min(left, eng.spl)
            eng.run_resident(xs, ys, k)
            L = eng.losses(k)
            tot += torch.stack((L[:, 0].sum() * B, L[:, 1].sum()))
            left -= k
        n = nb * B
        if N > n:  # the remainder (Keras trains on the partial last batch too)
            r = self._step(xs_all.index_select(0, idx[n:]), ys_all.index_select(0, idx[n:]))
            tot += torch.stack((r["loss"].reshape(-1)[0] * (N - n), r["correct"].reshape(-1)[0].float()))
        return tot[0], tot[1], N

    def _strip_last(self, cls):
        last = self.net[-1]
        if isinstance(last, tnn.Sequential) and isinstance(last[-1], cls):
            head = tnn.Sequential(*self.net[:-1], *last[:-1])
            return head.forward
        if isinstance(last, cls):
            return tnn.Sequential(*self.net[:-1]).forward
        return None

    def _strip_sigmoid(self):
        last = self.net[-1]
        if isinstance(last, hnn.Linear) and last.activation == "sigmoid":
            def fwd(x, net=self.net, lin=last):
                h = x
                for m in net[:-1]:
                    h = m(h)
                return HF.linear(h, lin.weight, lin.bias, None, lin.out_f32)

            return fwd
        return None

    def _labels(self, yb):
        if self._kind == "sparse_ce":
            return yb.long().reshape(-1)
        return yb.float().reshape(yb.shape[0], -1)

    def fit(self, x=None, y=None, batch_size=32, epochs=1, verbose=1, callbacks=None, validation_data=None,
            shuffle=True, steps_per_epoch=None, initial_epoch=0, seed=0, **_):
        hist = History()
        cbs = [hist] + list(callbacks or [])
        for c in cbs:
            if hasattr(c, "set_model"):
                c.set_model(self)
            elif hasattr(c, "model"):
                c.model = self
        per_batch = any(type(c).on_batch_end is not Callback.on_batch_end if isinstance(c, Callback)
                        else hasattr(c, "on_batch_end") or hasattr(c, "on_train_batch_end") for c in cbs)
        rng = np.random.default_rng(seed)
        self.stop_training = False
        self.train()
        # resident-epoch path on the persistent engine (runtime.persist): whole arrays of uint8 images, no
        # per-batch callbacks — the model then trains 32 steps per launch (see _fit_epoch_fast)
        arrays = isinstance(x, (np.ndarray, torch.Tensor)) and y is not None
        fast_ok = (arrays and not per_batch and steps_per_epoch is None and len(x) >= batch_size
                   and str(x.dtype) in ("uint8", "torch.uint8") and tuple(x.shape[1:]) in ((28, 28), (28, 28, 1)))
        if arrays and self._step is None:  # build / place the model now (the device decides the batch source)
            if fast_ok:
                self._batch_hint = int(batch_size)
            self._prepare(_to_tensor(x[:1], "cpu"))
        fast = fast_ok and self._fast is not None and int(batch_size) == self.geom_batch
        # any other model on whole arrays: the TrainStep's resident multi-step path (same epoch semantics)
        resident = (not fast and arrays and not per_batch and steps_per_epoch is None and len(x) >= batch_size
                    and self.device is not None and self.device.type == "cuda" and self._step is not None
                    and getattr(self._step, "dp", None) is None and _fits_hbm(x, y)
                    and os.environ.get("HOPSX_KERAS_RESIDENT", "1") == "1")
        for c in cbs:
            getattr(c, "on_train_begin", lambda *a: None)({})
        dataset_iter = None
        for epoch in range(initial_epoch, epochs):
            t0 = time.time()
            for c in cbs:
                getattr(c, "on_epoch_begin", lambda *a: None)(epoch, {})
            if fast or resident:
                if fast:
                    tl, tcor, tn = self._fit_epoch_fast(x, y, shuffle, rng)
                    width = 1
                else:
                    tl, tcor, tn, ys_all = self._fit_epoch_resident(x, y, batch_size, shuffle, rng)
                    width = self._label_width(ys_all)
                logs = {"loss": float(tl) / tn}
                if "accuracy" in self._metrics or "acc" in self._metrics:
                    logs["accuracy"] = float(tcor) / (tn * width)
                if validation_data is not None:
                    vl = self.evaluate(*validation_data, batch_size=batch_size, verbose=0, return_dict=True)
                    logs.update({"val_" + k: v for k, v in vl.items()})
                    self.train()
                if verbose:
                    s = " - ".join(f"{k}: {v:.4f}" for k, v in logs.items())
                    print(f"Epoch {epoch + 1}/{epochs} - {time.time() - t0:.1f}s - {s}", flush=True)
                for cb in cbs:
                    getattr(cb, "on_epoch_end", lambda *a: None)(epoch, logs)
                if self.stop_training:
                    break
                continue
            if arrays and self.device is not None and self.device.type == "cuda" and _fits_hbm(x, y):
                # whole arrays: uploaded once, the epoch's batches gathered on the device (no host-to-device
                # copy per batch; the numpy permutation's seed drives the device permutation)
                src = self._device_batches(x, y, batch_size, shuffle, rng)
            elif y is None and x is not None and not isinstance(x, (np.ndarray, torch.Tensor)):
                if dataset_iter is None or steps_per_epoch is None:
                    dataset_iter = iter(x)
                src = dataset_iter
            else:
                src = _batches(x, y, batch_size, shuffle, rng)
            tot_loss = tot_correct = None
            tot_n = 0
            nb = 0
            while steps_per_epoch is None or nb < steps_per_epoch:
                try:
                    xb, yb = next(src)
                except StopIteration:
                    if steps_per_epoch is not None and y is None and nb > 0:
                        dataset_iter = iter(x)
                        src = dataset_iter
                        continue
                    break
                if self._step is None:
                    self._prepare(_to_tensor(xb, "cpu"))
                xb = _to_tensor(xb, self.device)
                yb = self._labels(_to_tensor(yb, self.device, label=True))
                r = self._step(xb, yb)
                n = xb.shape[0]
                l = r["loss"].reshape(-1)[0] * n
                c = r["correct"].reshape(-1)[0].float() if r.get("correct") is not None else None
                tot_loss = l.clone() if tot_loss is None else tot_loss + l
                if c is not None:
                    tot_correct = c.clone() if tot_correct is None else tot_correct + c
                tot_n += n
                nb += 1
                if per_batch:
                    logs = {"loss": float(l) / n}
                    if c is not None:
                        logs["accuracy"] = float(c) / (n * self._label_width(yb))
                    for cb in cbs:
                        f = getattr(cb, "on_batch_end", None) or getattr(cb, "on_train_batch_end", None)
                        if f is not None:
                            f(nb - 1, logs)
                if self.stop_training:
                    break
            logs = {"loss": float(tot_loss) / max(tot_n, 1)}
            if tot_correct is not None and ("accuracy" in self._metrics or "acc" in self._metrics):
                logs["accuracy"] = float(tot_correct) / max(tot_n * self._label_width(yb), 1)
            if validation_data is not None:
                vl = self.evaluate(*validation_data, batch_size=batch_size, verbose=0, return_dict=True)
                logs.update({"val_" + k: v for k, v in vl.items()})
                self.train()
            if verbose:
                s = " - ".join(f"{k}: {v:.4f}" for k, v in logs.items())
                print(f"Epoch {epoch + 1}/{epochs} - {time.time() - t0:.1f}s - {s}", flush=True)
            for cb in cbs:
                getattr(cb, "on_epoch_end", lambda *a: None)(epoch, logs)
            if self.stop_training:
                break
        for c in cbs:
            getattr(c, "on_train_end", lambda *a: None)({})
        return hist

    def _label_width(self, yb):
        return 1 if self._kind == "sparse_ce" or yb.dim() == 1 else (1 if self._kind in ("ce",) else yb.shape[1])

    @torch.no_grad()
    def evaluate(self, x=None, y=None, batch_size=32, verbose=1, return_dict=False, steps=None, **_):
        self.eval()
        if self._step is None:
            first = next(iter(x)) if y is None else (x[:1], y[:1])
            self._prepare(_to_tensor(first[0], "cpu"))
        src = iter(x) if y is None else _batches(x, y, batch_size, False, None)
        fwd = self._train_fwd or self.forward
        tl = tc = 0.0
        tn = 0
        w = 1
        for i, (xb, yb) in enumerate(src):
            if steps is not None and i >= steps:
                break
            xb = _to_tensor(xb, self.device)
            yb = self._labels(_to_tensor(yb, self.device, label=True))
            st: dict = {}
            l = HF.loss(fwd(xb), yb, self._kind, stats=st)
            n = xb.shape[0]
            tl += float(l.reshape(-1)[0]) * n
            tc += float(st["correct"].reshape(-1)[0]) if "correct" in st else 0.0
            tn += n
            w = self._label_width(yb)
        out = {"loss": tl / max(tn, 1)}
        if "accuracy" in self._metrics or "acc" in self._metrics:
            out["accuracy"] = tc / max(tn * w, 1)
        if verbose:
            print(" - ".join(f"{k}: {v:.4f}" for k, v in out.items()))
        if return_dict:
            return out
        return list(out.values()) if len(out) > 1 else out["loss"]

    @torch.no_grad()
    def predict(self, x, batch_size=256, **_):
        self.eval()
        if self.net is None or self.device is None:
            xs = x if isinstance(x, (np.ndarray, torch.Tensor)) else np.asarray(x)
            if self.net is None:
                self.build(tuple(xs.shape[1:]))
            self.device = _default_device()
            self.to(self.device)
            if self.device.type == "cuda":
                from .runtime.arena import ParamArena

                ParamArena.from_module(self, self.device)
        outs = []
        for s in range(0, len(x), batch_size):
            xb = _to_tensor(x[s:s + batch_size], self.device)
            outs.append(self.forward(xb).float().cpu())
        return torch.cat(outs).numpy()

    def predict_classes(self, x, batch_size=256):
        return self.predict(x, batch_size).argmax(-1)

    # ------------------------------------------------------------------ persistence
    def save(self, path):
        path = Path(path)
        path.parent.mkdir(parents=True, exist_ok=True)
        sd = {k: v.detach().cpu() for k, v in self.state_dict().items()}
        torch.save(sd, str(path))

    def load_weights(self, path):
        sd = torch.load(str(path), map_location="cpu", weights_only=True)
        dev = self.device
        self.load_state_dict(sd)
        if dev is not None and dev.type == "cuda" and getattr(self, "_hx_arena", None) is not None:
            self._hx_arena.refresh_shadow()

    save_weights = save


class Model(Sequential):
    pass


__all__ = ["layers", "optimizers", "callbacks", "Sequential", "Model", "Input", "Dense", "Conv2D", "MaxPooling2D",
           "Dropout", "Flatten", "Activation", "BatchNormalization", "GlobalAveragePooling2D"]
