"""Metrics registry: counters, gauges and timers with three sinks.

The reference's observability is the experiment result dict, stdout captured into
``output.log`` / ``chief_0_output.log`` and TensorBoard scalars (Keras callback,
``SummaryWriter.add_scalar('Loss/train', …)`` at notebooks/ml/Experiment/PyTorch/mnist.ipynb:153).
Here every process owns a :class:`Registry` (``metrics.registry()``) whose values go to

* a per-rank JSON-lines file ``<logdir>/metrics_rank<r>.jsonl`` (``flush()``; one record per
  flush with wall time, step and every metric) — merged across ranks by :func:`merge_jsonl`;
* TensorBoard scalars through hopsx's own event writer (``to_tensorboard``);
* Prometheus text exposition (``prometheus_text()``; served by ``serving`` endpoints).

Timers measure host wall time; for device time wrap the region with ``timer(..., cuda=True)``
which brackets it with HIP events (no device synchronisation until ``flush``).
"""
from __future__ import annotations

import json
import os
import threading
import time
from contextlib import contextmanager
from pathlib import Path


class _Timer:
    __slots__ = ("count", "total", "min", "max", "last", "_pending")

    def __init__(self):
        self.count, self.total, self.min, self.max, self.last = 0, 0.0, float("inf"), 0.0, 0.0
        self._pending = []  # (start_event, end_event) pairs resolved at flush

    def add(self, seconds: float):
        self.count += 1
        self.total += seconds
        self.last = seconds
        self.min = min(self.min, seconds)
        self.max = max(self.max, seconds)

    def resolve(self):
        for s, e in self._pending:
            e.synchronize()
            self.add(s.elapsed_time(e) / 1e3)
        self._pending.clear()

    def value(self) -> dict:
        self.resolve()
        if not self.count:
            return {"count": 0}
        return {"count": self.count, "mean_ms": 1e3 * self.total / self.count, "min_ms": 1e3 * self.min,
                "max_ms": 1e3 * self.max, "last_ms": 1e3 * self.last}


class Registry:
    def __init__(self, logdir: str | None = None, rank: int | None = None):
        self.rank = int(os.environ.get("RANK", "0")) if rank is None else rank
        self.logdir = logdir
        self.counters: dict[str, float] = {}
        self.gauges: dict[str, float] = {}
        self.timers: dict[str, _Timer] = {}
        self.step = 0
        self._lock = threading.Lock()
        self._tb = None

    # ----------------------------------------------------------- instruments
    def inc(self, name: str, value: float = 1.0) -> None:
        with self._lock:
            self.counters[name] = self.counters.get(name, 0.0) + value

    def set(self, name: str, value: float) -> None:
        with self._lock:
            self.gauges[name] = float(value)

    def observe(self, name: str, seconds: float) -> None:
        with self._lock:
            self.timers.setdefault(name, _Timer()).add(seconds)

    @contextmanager
    def timer(self, name: str, cuda: bool = False):
        if cuda:
            import torch

            if torch.cuda.is_available():
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                try:
                    yield
                finally:
                    e.record()
                    with self._lock:
                        self.timers.setdefault(name, _Timer())._pending.append((s, e))
                return
        t0 = time.perf_counter()
        try:
            yield
        finally:
            self.observe(name, time.perf_counter() - t0)

    def throughput(self, name: str, items: float, seconds: float) -> None:
        """Gauge ``name`` = items / seconds (e.g. images/sec for the last window)."""
        self.set(name, items / seconds if seconds > 0 else 0.0)

    # ---------------------------------------------------------------- sinks
    def snapshot(self) -> dict:
        with self._lock:
            return {"time": time.time(), "rank": self.rank, "step": self.step, "counters": dict(self.counters),
                    "gauges": dict(self.gauges), "timers": {k: t.value() for k, t in self.timers.items()}}

    def _dir(self) -> Path:
        d = self.logdir
        if d is None:
            from .tensorboard import logdir

            d = logdir()
        p = Path(d)
        p.mkdir(parents=True, exist_ok=True)
        return p

    def flush(self, step: int | None = None, to_tensorboard: bool = False) -> dict:
        if step is not None:
            self.step = int(step)
        snap = self.snapshot()
        with open(self._dir() / f"metrics_rank{self.rank}.jsonl", "a") as f:
            f.write(json.dumps(snap) + "\n")
        if to_tensorboard:
            self.to_tensorboard(snap)
        return snap

    def to_tensorboard(self, snap: dict | None = None) -> None:
        from .tensorboard import SummaryWriter

        snap = snap or self.snapshot()
        if self._tb is None:
            self._tb = SummaryWriter(str(self._dir() / f"metrics_rank{self.rank}"))
        for k, v in {**snap["counters"], **snap["gauges"]}.items():
            self._tb.add_scalar(k, v, snap["step"])
        for k, v in snap["timers"].items():
            if v.get("count"):
                self._tb.add_scalar(f"{k}/mean_ms", v["mean_ms"], snap["step"])
        self._tb.flush()

    def prometheus_text(self, prefix: str = "hopsx_") -> str:
        snap = self.snapshot()
        lines = []

        def name(k):
            return prefix + "".join(c if c.isalnum() else "_" for c in k)

        for k, v in snap["counters"].items():
            lines += [f"# TYPE {name(k)} counter", f'{name(k)}{{rank="{self.rank}"}} {v}']
        for k, v in snap["gauges"].items():
            lines += [f"# TYPE {name(k)} gauge", f'{name(k)}{{rank="{self.rank}"}} {v}']
        for k, v in snap["timers"].items():
            if v.get("count"):
                n = name(k) + "_seconds"
                lines += [f"# TYPE {n} summary", f'{n}_count{{rank="{self.rank}"}} {v["count"]}',
                          f'{n}_sum{{rank="{self.rank}"}} {v["mean_ms"] * v["count"] / 1e3}']
        return "\n".join(lines) + "\n"

    def reset(self) -> None:
        with self._lock:
            self.counters.clear()
            self.gauges.clear()
            self.timers.clear()


_REG: list = [None]


def registry() -> Registry:
    if _REG[0] is None:
        _REG[0] = Registry()
    return _REG[0]


def merge_jsonl(logdir) -> list[dict]:
    """All ranks' records of a run, ordered by (step, rank)."""
    out = []
    for p in sorted(Path(logdir).glob("metrics_rank*.jsonl")):
        for line in p.read_text().splitlines():
            if line.strip():
                out.append(json.loads(line))
    return sorted(out, key=lambda r: (r.get("step", 0), r.get("rank", 0), r.get("time", 0)))
