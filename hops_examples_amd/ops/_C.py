"""Loader for the in-tree HIP kernel library ``_hopsx_ops`` (gfx950).

On a machine with a GPU the extension is REQUIRED: every op fails loudly if it
cannot be imported, so a GPU run can never silently fall back to eager PyTorch.
On a CPU-only machine the ops use their PyTorch reference implementations
(``hops_examples_amd.ops.reference``), which is what the CPU test-suite and the
``experiment.launch`` CPU config exercise.
"""
from __future__ import annotations

import importlib
import os

import torch

_ext = None
_err: Exception | None = None


def _load():
    global _ext, _err
    if _ext is not None or _err is not None:
        return _ext
    if debug():
        # the debug build (python -m hops_examples_amd._build --debug): no autobuild, no fallback
        try:
            _ext = importlib.import_module("hops_examples_amd._hopsx_ops_dbg")
        except Exception as e:
            _err = e
        return _ext
    try:
        _ext = importlib.import_module("hops_examples_amd._hopsx_ops")
    except Exception as e:  # pragma: no cover - depends on build state
        if os.environ.get("HOPSX_AUTOBUILD", "1") == "1":
            try:
                from .. import _build

                _build.build(verbose=False)
                _ext = importlib.import_module("hops_examples_amd._hopsx_ops")
                return _ext
            except Exception as e2:
                _err = e2
        else:
            _err = e
    return _ext


_det_done = False


def debug() -> bool:
    """``HOPSX_DEBUG=1``: load ``_hopsx_ops_dbg`` (device-side bound checks, common.h hx_check); every
    checked launch outside graph capture is followed by a synchronize and a read of the records."""
    return os.environ.get("HOPSX_DEBUG", "0") == "1"


def debug_errors(clear: bool = True) -> list:
    """Device-side check records since the last read: [(translation unit, failures, source line,
    workgroup, thread)].  Release builds record the always-on guards (hx_guard: embedding ids, class
    labels) too.  Reading clears them."""
    m = _load()
    if m is None or not torch.cuda.is_available() or not hasattr(m, "dbg_read"):
        return []
    torch.cuda.synchronize()
    return [tuple(r) for r in m.dbg_read()]


def deterministic() -> bool:
    """``HOPSX_DETERMINISTIC=1``: order-fixed cross-workgroup float reductions (common.h
    "deterministic mode"): replays from the same state are bit-identical, at some speed cost."""
    return os.environ.get("HOPSX_DETERMINISTIC", "0") == "1"


def ext():
    """The kernel module; raises if it is unavailable."""
    global _det_done
    m = _load()
    if m is None:
        raise RuntimeError(
            "hopsx HIP kernel library _hopsx_ops is not built/importable "
            f"({_err!r}); run `python -m hops_examples_amd._build`"
        )
    if not _det_done:
        _det_done = True
        if deterministic() and torch.cuda.is_available():
            # the device-side flag of every kernel translation unit (host-side planning reads the
            # environment itself); set before the first launch, outside any graph capture
            e = m.set_deterministic(1)
            if e:
                raise RuntimeError(f"hopsx: enabling deterministic mode failed (hip error {e})")
    return m


def available() -> bool:
    return _load() is not None


def gpu_enabled() -> bool:
    return torch.cuda.is_available()


def ptr(t: torch.Tensor | None) -> int:
    return 0 if t is None else t.data_ptr()


_stream_cache: dict = {}


def stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"hopsx kernel {what} failed with hipError {rc}")
    if _DEBUG and not torch.cuda.is_current_stream_capturing():
        errs = debug_errors()
        if errs:
            raise RuntimeError(f"hopsx kernel {what}: device-side check failed: " + "; ".join(
                f"{tu}.hip line {ln} (workgroup {wg}, thread {th}; {n} failure(s))" for tu, n, ln, wg, th in errs))


_DEBUG = debug()


# mirror of csrc/ops/ops_api.h
EPI_STORE_BF16, EPI_STORE_F32, EPI_ATOMIC_F32, EPI_DACT_BF16 = 0, 1, 2, 3
ACT = {None: 0, "linear": 0, "none": 0, "relu": 1, "sigmoid": 2, "tanh": 3}
LOSS = {"sparse_ce": 0, "ce": 1, "bce_logits": 2, "mse": 3, "bce": 4}
OPTIM = {"sgd": 0, "adam": 1, "adamw": 2, "adadelta": 3, "rmsprop": 4, "adagrad": 5, "ftrl": 6}
