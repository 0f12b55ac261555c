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
        upload(g)
    finally:
        if was:
            gc.enable()


def upload(g: "torch.cuda.CUDAGraph") -> None:
    """hipGraphUpload the instantiated executable now: the first replay otherwise pays the upload
    (measured ~70 us of fixed cost in a 20-step timed window of the flagship at 8 steps per graph)."""
    try:
        from ..ops import _C

        ex = g.raw_cuda_graph_exec()
        if ex:
            _C.ext().graph_upload(int(ex), torch.cuda.current_stream().cuda_stream)
    except Exception:  # noqa: BLE001 - an optimisation only (older torch: no raw exec handle)
        pass
