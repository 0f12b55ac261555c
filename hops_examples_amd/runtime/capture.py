"""hipGraph capture with the Python garbage collector held off.

A collection that runs while a stream is being captured can finalise an unrelated object (an old
graph, a tensor of a private pool) whose release calls into HIP, which is illegal during capture
and aborts the process.  torch collects once before capture; allocations inside the captured
region can still trigger a collection, so capture regions here run with ``gc`` disabled.
"""
from __future__ import annotations

import contextlib
import gc

import torch


@contextlib.contextmanager
def graph(g: "torch.cuda.CUDAGraph", pool=None, stream=None):
    was = gc.isenabled()
    gc.collect()
    gc.disable()
    try:
        kw = {"pool": pool} if pool is not None else {}
        if stream is not None:
            kw["stream"] = stream
        with torch.cuda.graph(g, **kw):
            yield g
    finally:
        if was:
            gc.enable()
