"""Experiment execution engine: run a user function in worker processes.

The reference ships the user's wrapper function to Spark executors (pickled
closure + YARN containers; SURVEY §1.1 "Process/device boundaries").  Here a
worker is a child Python process pinned to one GPU (``HIP_VISIBLE_DEVICES``),
started with ``subprocess`` (never fork-only, never exec from a GPU process),
receiving the function via cloudpickle and writing its return value back the
same way.  stdout/stderr go to the run directory's ``output.log`` (chief/worker
logs for distributed runs), exactly where the reference puts them.
"""
from __future__ import annotations

import dataclasses
import json
import os
import shutil
import socket
import subprocess
import sys
import time
import traceback
from pathlib import Path

import cloudpickle

from .. import config, hdfs

_APP_TS = str(int(time.time() * 1000))


def _counter_file() -> Path:
    return Path(hdfs.project_path()) / "Experiments" / ".hopsx_runs.json"


def next_app_id() -> str:
    """``application_<clusterTs>_<appSeq>_<runSeq>`` (reference format)."""
    cf = _counter_file()
    cf.parent.mkdir(parents=True, exist_ok=True)
    try:
        state = json.loads(cf.read_text())
    except Exception:
        state = {}
    key = f"{_APP_TS}_{os.getpid()}"
    app_seq = state.get("apps", {}).get(key)
    if app_seq is None:
        app_seq = len(state.get("apps", {})) + 1
        state.setdefault("apps", {})[key] = app_seq
    run = state.get("runs", {}).get(key, 0) + 1
    state.setdefault("runs", {})[key] = run
    cf.write_text(json.dumps(state))
    return f"application_{_APP_TS}_{app_seq:04d}_{run}"


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def num_gpus() -> int:
    """GPUs usable for trials. Counting devices does not initialise the GPU on ROCm."""
    env = os.environ.get("HOPSX_NUM_GPUS")
    if env is not None:
        return int(env)
    try:
        import torch

        return torch.cuda.device_count()
    except Exception:
        return 0


@dataclasses.dataclass
class Worker:
    proc: subprocess.Popen
    run_dir: Path
    result_path: Path
    log_path: Path
    logf: object
    started: float


def spawn(fn, kwargs: dict, run_dir: Path, log_name: str = "output.log", env: dict | None = None,
          gpu: int | None = None, local_logdir: bool = False) -> Worker:
    run_dir.mkdir(parents=True, exist_ok=True)
    tag = log_name.replace("_output.log", "").replace("output.log", "main")
    payload = run_dir / f".payload_{tag}.pkl"
    result = run_dir / f".result_{tag}.pkl"
    if result.exists():
        result.unlink()
    payload.write_bytes(cloudpickle.dumps((fn, kwargs)))
    e = dict(os.environ)
    c = config.get()
    e.update({
        "HOPSX_PROJECT_ROOT": str(c.project_root),
        "HOPSX_PROJECT_NAME": c.project_name,
        "HOPSX_LOGDIR": str(run_dir),
        "HOPSX_LOCAL_LOGDIR": "1" if local_logdir else "0",
        "HSA_ENABLE_IPC_MODE_LEGACY": "0",
        "PYTHONUNBUFFERED": "1",
    })
    root = str(Path(__file__).resolve().parents[2])
    e["PYTHONPATH"] = root + (os.pathsep + e["PYTHONPATH"] if e.get("PYTHONPATH") else "")
    if gpu is not None:
        e["HIP_VISIBLE_DEVICES"] = str(gpu)
        e["CUDA_VISIBLE_DEVICES"] = str(gpu)
    if env:
        e.update({k: str(v) for k, v in env.items()})
    log_path = run_dir / log_name
    logf = open(log_path, "ab")
    proc = subprocess.Popen([sys.executable, "-m", "hops_examples_amd.experiment._worker", str(payload), str(result)],
                            stdout=logf, stderr=subprocess.STDOUT, env=e, cwd=str(run_dir))
    return Worker(proc, run_dir, result, log_path, logf, time.time())


class TrialError(RuntimeError):
    pass


def collect(w: Worker, timeout: float | None = None):
    try:
        rc = w.proc.wait(timeout=timeout)
    except subprocess.TimeoutExpired:
        w.proc.kill()
        w.proc.wait()
        w.logf.close()
        raise TrialError(f"worker timed out after {timeout}s; see {w.log_path}")
    w.logf.close()
    if not w.result_path.exists():
        tail = w.log_path.read_text(errors="replace")[-3000:]
        raise TrialError(f"worker exited with code {rc} and no result; log tail:\n{tail}")
    ok, value = cloudpickle.loads(w.result_path.read_bytes())
    if not ok:
        raise TrialError(f"user function raised:\n{value}")
    return value


def _tail(w: Worker, n: int = 3000) -> str:
    try:
        return w.log_path.read_text(errors="replace")[-n:]
    except OSError:
        return ""


def wait_all(workers: list, timeout: float | None = None, heartbeat_timeout: float | None = None,
             poll_s: float = 0.2) -> list:
    """Wait for a gang of workers (one distributed job) and return their values in order.

    Unlike collecting them one by one, the FIRST failing rank ends the job: the others are
    killed at once (a rank blocked in a collective on a dead peer would otherwise wait for
    the collective timeout) and the error names that rank with its log tail.  With
    ``heartbeat_timeout`` a rank whose progress heartbeat (runtime.health.beat, written by
    TrainStep every step) stops for that long is declared stalled and the job is torn down.
    """
    from ..runtime import health

    t0 = time.time()
    pending = set(range(len(workers)))
    failure = None
    while pending and failure is None:
        for i in sorted(pending):
            rc = workers[i].proc.poll()
            if rc is None:
                continue
            pending.discard(i)
            if rc != 0 or not workers[i].result_path.exists():
                failure = (i, f"rank {i} exited with code {rc}")
                break
        if failure is not None or not pending:
            break
        now = time.time()
        if timeout is not None and now - t0 > timeout:
            failure = (min(pending), f"job timed out after {timeout}s")
            break
        if heartbeat_timeout:
            for i in sorted(pending):
                hb = health.last_beat(workers[i].run_dir, i)
                if hb is not None and now - hb > heartbeat_timeout:
                    failure = (i, f"rank {i} stalled: no progress heartbeat for {now - hb:.1f}s "
                                  f"(> heartbeat_timeout={heartbeat_timeout}s)")
                    break
        time.sleep(poll_s)
    if failure is not None:
        failure = _root_cause(workers, failure, pending)
        for w in workers:
            if w.proc.poll() is None:
                w.proc.kill()
        for w in workers:
            try:
                w.proc.wait(timeout=30)
            except subprocess.TimeoutExpired:
                pass
            w.logf.close()
        i, why = failure
        w = workers[i]
        detail = ""
        if w.result_path.exists():
            ok, value = cloudpickle.loads(w.result_path.read_bytes())
            if not ok:
                detail = f"\nuser function raised:\n{value}"
        raise TrialError(f"{why}; first failure in {w.log_path}{detail}\nlog tail:\n{_tail(w)}")
    return [collect(w) for w in workers]


# errors a rank raises because a PEER died (its collective lost the connection), not the root cause
_PEER_LOSS = ("Connection reset", "Connection closed", "Broken pipe", "gloo", "NCCL", "RCCL", "ProcessGroup",
              "Socket Timeout", "recvBytes", "sendBytes")


def _root_cause(workers, failure, pending, grace_s: float = 1.0):
    """The first rank seen failing may only be reacting to a peer's death (its all-reduce lost the
    connection).  Give the other ranks a short grace to exit, then name a rank whose own function
    raised something other than a lost-peer error, if there is one."""
    first, _ = failure
    t_end = time.time() + grace_s
    failed = [first]
    while time.time() < t_end:
        for i in sorted(pending):
            rc = workers[i].proc.poll()
            if rc is not None and (rc != 0 or not workers[i].result_path.exists()) and i not in failed:
                failed.append(i)
        if len(failed) == len(workers):
            break
        time.sleep(0.05)
    for i in failed:
        w = workers[i]
        msg = ""
        if w.result_path.exists():
            try:
                ok, value = cloudpickle.loads(w.result_path.read_bytes())
                msg = "" if ok else str(value)
            except Exception:  # noqa: BLE001 - a torn result file is no root cause either
                msg = ""
        if msg and not any(k in msg for k in _PEER_LOSS):
            return (i, f"rank {i} exited with code {w.proc.poll()}") if i != first else failure
    return failure


def run_inline(fn, kwargs: dict, run_dir: Path, log_name="output.log"):
    """In-process execution (``HOPSX_INLINE=1``): same directory/log contract, no child process."""
    import contextlib
    import io

    run_dir.mkdir(parents=True, exist_ok=True)
    old = os.environ.get("HOPSX_LOGDIR")
    os.environ["HOPSX_LOGDIR"] = str(run_dir)
    buf = io.StringIO()
    try:
        with contextlib.redirect_stdout(buf):
            try:
                return fn(**kwargs)
            except Exception:
                print(traceback.format_exc())
                raise
    finally:
        (run_dir / log_name).write_text(buf.getvalue())
        if old is None:
            os.environ.pop("HOPSX_LOGDIR", None)
        else:
            os.environ["HOPSX_LOGDIR"] = old


def rel_to_project(p: Path) -> str:
    root = Path(hdfs.project_path())
    try:
        return str(p.resolve().relative_to(root.resolve()))
    except ValueError:
        return str(p)


def finalize_result(value, run_dir: Path, log_name: str = "output.log") -> dict:
    """The reference's result-dict contract: dict returns are kept, file-valued
    entries are copied into the run dir and rewritten to project-relative paths, a
    non-dict return becomes {'metric': value}, and 'log' points at the run's log."""
    if isinstance(value, dict):
        out = {}
        for k, v in value.items():
            if isinstance(v, str) and not v.startswith("Experiments/"):
                for base in (run_dir, Path.cwd()):
                    cand = base / v
                    if cand.is_file():
                        dest = run_dir / Path(v).name
                        if cand.resolve() != dest.resolve():
                            shutil.copy2(cand, dest)
                        v = rel_to_project(dest)
                        break
            out[k] = v
    else:
        out = {"metric": value}
    out["log"] = rel_to_project(run_dir / log_name)
    return out


def write_meta(run_dir: Path, **meta) -> None:
    p = run_dir / "experiment.json"
    cur = {}
    if p.exists():
        try:
            cur = json.loads(p.read_text())
        except Exception:
            cur = {}
    cur.update(meta)
    p.write_text(json.dumps(cur, indent=2, default=str))
