"""Tracing, profiling and numerical health checks.

The reference profiles through the Keras TensorBoard callback ``profile_batch='5,10'``
(notebooks/ml/Experiment/Tensorflow/mnist.ipynb:172-173) and shows tfdbg NaN/Inf "health pills"
(notebooks/ml/images/tensorboard_debug.png).  The MI355X counterparts:

* :class:`StepProfiler` / :func:`profile` — ``profile_batch``-style step window around a training
  loop.  Inside the window ``torch.profiler`` (kineto + roctracer on ROCm: host ops, HIP API calls
  and every hopsx kernel by name) records and writes a Chrome/Perfetto trace JSON into
  ``<logdir>/plugins/profile/<run>/`` (the layout the TensorBoard profile plugin reads), plus a
  per-kernel summary table ``kernels.txt``.
* :func:`rocprof_command` — the command line for a ``rocprofv3`` kernel-trace / stats run or a
  counter pass (kept apart from tracing: counters never share a run with ``--sys-trace``), and
  :func:`summarize_rocprof` — per-kernel totals from its ``*_kernel_stats.csv``.
* :func:`nonfinite` / :class:`HealthCheck` — NaN/Inf counts of tensors from one fused HIP
  reduction (``hopsx_nonfinite``), graph-capturable; ``HealthCheck`` watches the parameter
  arena's gradients and weights every N steps.
"""
from __future__ import annotations

import csv
import json
import os
import shlex
import time
from pathlib import Path

import torch


# ------------------------------------------------------------------ step-window tracing
def _parse_window(profile_batch) -> tuple[int, int] | None:
    """Keras semantics: '5,10' -> steps 5..10 (inclusive), 7 -> just step 7, 0/None -> off."""
    if not profile_batch:
        return None
    if isinstance(profile_batch, int):
        return (profile_batch, profile_batch)
    if isinstance(profile_batch, (tuple, list)):
        a, b = int(profile_batch[0]), int(profile_batch[1])
    else:
        parts = [int(p) for p in str(profile_batch).split(",")]
        a, b = (parts[0], parts[0]) if len(parts) == 1 else (parts[0], parts[1])
    if a <= 0 or b < a:
        raise ValueError(f"profile_batch must be 'start,stop' with 0 < start <= stop, got {profile_batch!r}")
    return a, b


class StepProfiler:
    """``prof = StepProfiler('5,10', logdir); for step ...: prof.step()`` (call once per step,
    after the step's work).  Steps are 1-based like Keras batches."""

    def __init__(self, profile_batch="5,10", logdir: str | None = None, run_name: str | None = None,
                 record_shapes: bool = False):
        self.window = _parse_window(profile_batch)
        if logdir is None:
            from .tensorboard import logdir as _ld

            logdir = _ld()
        self.run = run_name or time.strftime("%Y_%m_%d_%H_%M_%S")
        self.out_dir = Path(logdir) / "plugins" / "profile" / self.run
        self.record_shapes = record_shapes
        self._n = 0
        self._prof = None
        self.trace_path: Path | None = None
        self.summary_path: Path | None = None
        if self.window and self.window[0] == 1:
            self._start()  # the window opens before the first step

    def _start(self):
        from torch.profiler import ProfilerActivity, profile as tprof

        acts = [ProfilerActivity.CPU]
        if torch.cuda.is_available():
            acts.append(ProfilerActivity.CUDA)  # HIP kernels via roctracer on ROCm
        self._prof = tprof(activities=acts, record_shapes=self.record_shapes)
        self._prof.__enter__()

    def _stop(self):
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        self._prof.__exit__(None, None, None)
        self.out_dir.mkdir(parents=True, exist_ok=True)
        self.trace_path = self.out_dir / "trace.json"
        self._prof.export_chrome_trace(str(self.trace_path))
        self.summary_path = self.out_dir / "kernels.txt"
        self.summary_path.write_text(format_table(trace_kernel_summary(self.trace_path)))
        self._prof = None

    def step(self):
        self._n += 1
        if self.window is None:
            return
        a, b = self.window
        if self._n == a - 1 and self._prof is None:
            self._start()
        if self._n == b and self._prof is not None:
            self._stop()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        if self._prof is not None:
            self._stop()


def profile(profile_batch="5,10", logdir: str | None = None, **kw) -> StepProfiler:
    """Context manager form: ``with hx.profiler.profile('5,10') as p: ... p.step()``."""
    return StepProfiler(profile_batch, logdir, **kw)


def trace_kernel_summary(trace_json) -> list[dict]:
    """Per-kernel totals (GPU 'kernel' events) from a Chrome trace written by the profiler."""
    with open(trace_json) as f:
        data = json.load(f)
    evs = data["traceEvents"] if isinstance(data, dict) else data
    agg: dict[str, list] = {}
    for e in evs:
        if e.get("ph") != "X" or e.get("cat") not in ("kernel", "gpu_memcpy", "gpu_memset"):
            continue
        a = agg.setdefault(e.get("name", "?"), [0, 0.0])
        a[0] += 1
        a[1] += float(e.get("dur", 0.0))
    rows = [{"name": k, "calls": v[0], "total_us": v[1], "avg_us": v[1] / max(v[0], 1)} for k, v in agg.items()]
    return sorted(rows, key=lambda r: -r["total_us"])


def format_table(rows: list[dict], top: int = 40) -> str:
    tot = sum(r["total_us"] for r in rows) or 1.0
    out = [f"{'kernel':90s} {'calls':>7s} {'avg_us':>9s} {'total_us':>10s} {'pct':>6s}"]
    for r in rows[:top]:
        out.append(f"{r['name'][:90]:90s} {r['calls']:7d} {r['avg_us']:9.2f} {r['total_us']:10.1f} "
                   f"{100.0 * r['total_us'] / tot:6.1f}")
    return "\n".join(out) + "\n"


# ------------------------------------------------------------------------- rocprofv3
def rocprof_command(cmd, out_dir, pmc: list[str] | None = None, name: str = "run") -> str:
    """rocprofv3 command line: kernel trace + stats, or ONE counter pass when ``pmc`` is given.
    Counter passes never combine with --sys-trace/--runtime-trace (collect them in runs of their
    own) and the profiled program must come straight after ``--`` (no env/bash wrappers)."""
    argv = ["rocprofv3"]
    if pmc:
        argv += ["--pmc", *pmc]
    else:
        argv += ["--kernel-trace", "--stats"]
    argv += ["-d", str(out_dir), "-o", name, "--output-format", "csv", "--"]
    argv += cmd if isinstance(cmd, (list, tuple)) else shlex.split(cmd)
    return " ".join(shlex.quote(a) for a in argv)


def summarize_rocprof(stats_csv) -> list[dict]:
    """Rows of rocprofv3 ``*_kernel_stats.csv`` as {name, calls, total_us, avg_us}, largest first."""
    rows = []
    with open(stats_csv) as f:
        for r in csv.DictReader(f):
            rows.append({"name": r["Name"], "calls": int(r["Calls"]), "total_us": float(r["TotalDurationNs"]) / 1e3,
                         "avg_us": float(r["AverageNs"]) / 1e3})
    return sorted(rows, key=lambda r: -r["total_us"])


# --------------------------------------------------------------------- health pills
def nonfinite(t: torch.Tensor) -> tuple[int, int]:
    """(#NaN, #Inf) of a tensor: the hopsx_nonfinite HIP reduction on the GPU, torch on the CPU."""
    if t.is_cuda and t.dtype in (torch.float32, torch.bfloat16):
        from .ops import kernels as K

        c = K.nonfinite_counts(t).cpu()
        return int(c[0]), int(c[1])
    f = t.detach().float()
    return int(torch.isnan(f).sum()), int(torch.isinf(f).sum())


class NonFiniteError(FloatingPointError):
    pass


class HealthCheck:
    """Check a model's parameter arena (weights and gradients) for NaN/Inf every ``every`` steps.
    ``check(step)`` returns the counts and raises NonFiniteError when ``raise_on_error``."""

    def __init__(self, model, every: int = 100, raise_on_error: bool = True, log=print):
        self.arena = getattr(model, "_hx_arena", None)
        self.model, self.every, self.raise_on_error, self.log = model, every, raise_on_error, log
        self.history: list[dict] = []

    def _tensors(self):
        if self.arena is not None:
            return {"weights": self.arena.master, "grads": self.arena.grad}
        return {n: p.detach() for n, p in self.model.named_parameters()}

    def check(self, step: int) -> dict | None:
        if self.every <= 0 or step % self.every != 0:
            return None
        rep = {"step": step}
        bad = []
        for name, t in self._tensors().items():
            n_nan, n_inf = nonfinite(t)
            rep[name] = {"nan": n_nan, "inf": n_inf}
            if n_nan or n_inf:
                bad.append(f"{name}: {n_nan} NaN, {n_inf} Inf")
        self.history.append(rep)
        if bad:
            msg = f"non-finite values at step {step}: " + "; ".join(bad)
            if self.log:
                self.log(msg)
            if self.raise_on_error:
                raise NonFiniteError(msg)
        return rep


def env_profile_batch() -> str | None:
    """HOPSX_PROFILE_BATCH='5,10' turns the step profiler on for TrainStep-driven runs."""
    return os.environ.get("HOPSX_PROFILE_BATCH") or None
