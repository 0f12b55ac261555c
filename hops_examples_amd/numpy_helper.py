"""``hops.numpy_helper``: numpy load/save with project-relative paths
(notebooks/ml/numpy/numpy-hdfs.ipynb:29-36)."""
from __future__ import annotations

import numpy as np

from . import hdfs


def load(path: str, mmap_mode=None, allow_pickle: bool = False, **kw):
    return np.load(hdfs.abs_path(path), mmap_mode=mmap_mode, allow_pickle=allow_pickle, **kw)


def save(path: str, arr) -> None:
    p = hdfs.abs_path(path)
    import os

    os.makedirs(os.path.dirname(p) or ".", exist_ok=True)
    np.save(p, arr)


def loadtxt(path: str, **kw):
    return np.loadtxt(hdfs.abs_path(path), **kw)


def savetxt(path: str, arr, **kw):
    np.savetxt(hdfs.abs_path(path), arr, **kw)
