"""Gradient-readiness notifications from hopsx kernels to the DP engine.

hopsx autograd Functions accumulate weight gradients straight into the
ParamArena and return ``None`` to autograd, so the usual per-parameter autograd
hooks never fire for them.  Instead they call :func:`grad_ready`, which the
data-parallel engine subscribes to in order to launch a bucket's all-reduce as
soon as its last gradient has been produced (overlapping the rest of backward).
"""
from __future__ import annotations

_subscribers: list = []


def subscribe(fn) -> None:
    if fn not in _subscribers:
        _subscribers.append(fn)


def unsubscribe(fn) -> None:
    if fn in _subscribers:
        _subscribers.remove(fn)


def grad_ready(p) -> None:
    for fn in list(_subscribers):
        fn(p)
