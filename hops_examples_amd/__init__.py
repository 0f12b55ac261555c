"""hopsx — an MI355X-native framework with the capabilities of the hops-examples
collection: experiment API (launch / search / distributed), maggy, feature store,
model registry + serving, Keras-style and torch-style training on hand-written
gfx950 (CDNA4) kernels, RCCL data parallelism.

Submodules are imported lazily so ``import hops_examples_amd`` is cheap and never
touches the GPU.
"""
from __future__ import annotations

import importlib

__version__ = "0.1.0"

_SUBMODULES = {
    "config", "devices", "experiment", "featurestore", "hdfs", "io", "kafka", "keras", "maggy", "model", "models",
    "nn", "numpy_helper", "ops", "optim", "pandas_helper", "parallel", "runtime", "serving", "tensorboard", "util",
}


def __getattr__(name):
    if name in _SUBMODULES:
        mod = importlib.import_module(f".{name}", __name__)
        globals()[name] = mod
        return mod
    raise AttributeError(f"module {__name__!r} has no attribute {name!r}")


def __dir__():
    return sorted(set(globals()) | _SUBMODULES)
