"""Worker liveness, failure detection and fault injection.

The reference's only failure handling is Spark's (executor blacklisting switched off,
jobs-client/spark/job_config.json:18) plus a 90 s poll for a Flink job to reach RUNNING
(jobs-client/flink/jobs_flink_client.py:52-69); a hung MultiWorkerMirroredStrategy worker
hangs the whole notebook.  Here every training process reports progress and the launcher
(``experiment._runner.wait_all``) watches it:

* ``beat(step)`` — called once per training step by ``TrainStep`` (and usable from any user
  loop); rate-limited to one ``os.utime`` of ``$HOPSX_LOGDIR/.hb_<rank>`` per
  ``HOPSX_HEARTBEAT_S`` seconds (default 1 s), so it costs nothing in the hot loop.  A rank
  whose file stops advancing for ``heartbeat_timeout`` seconds is declared stalled (a hung
  collective, a dead peer) and the launcher tears the job down with that rank named.
* ``HOPSX_FAULT=<rank>:<step>[:raise|exit|hang]`` — fault injection for tests: the given rank
  raises / hard-exits / stops making progress when it reaches the given step.
"""
from __future__ import annotations

import os
import time
from pathlib import Path

_last = [0.0]
_path: list = [None]
_fault: list = [None]


def _rank() -> int:
    return int(os.environ.get("RANK", "0"))


def heartbeat_path(run_dir, rank: int) -> Path:
    return Path(run_dir) / f".hb_{rank}"


def _parse_fault():
    spec = os.environ.get("HOPSX_FAULT", "")
    if not spec:
        return False
    parts = spec.split(":")
    try:
        r, s = int(parts[0]), int(parts[1])
    except (IndexError, ValueError):
        raise ValueError(f"HOPSX_FAULT must be '<rank>:<step>[:raise|exit|hang]', got {spec!r}") from None
    kind = parts[2] if len(parts) > 2 else "raise"
    if kind not in ("raise", "exit", "hang"):
        raise ValueError(f"HOPSX_FAULT kind must be raise|exit|hang, got {kind!r}")
    return (r, s, kind)


class InjectedFault(RuntimeError):
    pass


def maybe_fault(step: int) -> None:
    if _fault[0] is None:
        _fault[0] = _parse_fault()
    f = _fault[0]
    if not f or f[0] != _rank() or f[1] != step:
        return
    if os.environ.get("HOPSX_RESTART", "0") != "0" and os.environ.get("HOPSX_FAULT_ONCE", "1") == "1":
        return  # a restarted attempt runs clean (tests restart-from-checkpoint)
    kind = f[2]
    if kind == "exit":
        os._exit(13)
    if kind == "hang":
        while True:  # stop making progress; the launcher's heartbeat watchdog must catch this
            time.sleep(3600)
    raise InjectedFault(f"HOPSX_FAULT: injected failure on rank {f[0]} at step {step}")


def beat(step: int | None = None) -> None:
    """Progress heartbeat (+ fault injection hook).  Cheap enough to call every step."""
    if step is not None:
        maybe_fault(step)
    now = time.monotonic()
    if now - _last[0] < _interval():
        return
    _touch(now)


def beat_range(first: int, n: int) -> None:
    """One heartbeat for the n steps first .. first + n - 1 that ONE launch / graph replay runs (the fault
    hook still fires when its step is among them): per-step beats cost ~2 us of host time each, which at
    20 steps per launch sits inside a timed window while the GPU waits."""
    if n <= 0:
        return
    if _fault[0] is None:
        _fault[0] = _parse_fault()
    f = _fault[0]
    if f and f[0] == _rank() and first <= f[1] < first + n:
        maybe_fault(f[1])
    now = time.monotonic()
    if now - _last[0] < _interval():
        return
    _touch(now)


_IVAL: list = [None, None]  # (env string, seconds)


def _interval() -> float:
    v = os.environ.get("HOPSX_HEARTBEAT_S", "1.0")
    if _IVAL[0] != v:
        _IVAL[0], _IVAL[1] = v, float(v)
    return _IVAL[1]


def _touch(now: float) -> None:
    _last[0] = now
    if _path[0] is None:
        d = os.environ.get("HOPSX_LOGDIR")
        if not d:
            _path[0] = False
            return
        _path[0] = heartbeat_path(d, _rank())
    p = _path[0]
    if not p:
        return
    try:
        p.touch(exist_ok=True)
        os.utime(p, None)
    except OSError:
        pass


def last_beat(run_dir, rank: int) -> float | None:
    """Wall-clock mtime of a rank's heartbeat file, None before its first beat."""
    try:
        return heartbeat_path(run_dir, rank).stat().st_mtime
    except OSError:
        return None
