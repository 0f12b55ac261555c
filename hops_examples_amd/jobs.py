"""Jobs service: named, configured programs launched as tracked executions.

Reference contract: ``jobs.create_job(name, config)`` / ``jobs.start_job(name, args)``
(jobs-client/spark/jobs_spark_client.py:50-54, config jobs-client/spark/job_config.json:1-23),
``get_executions`` polling (jobs-client/flink/jobs_flink_client.py:60-90) and the Airflow
operators that launch a job and wait for it (airflow/launch_jobs.py:79-130).

Local execution model: a job is a Python program (``appPath``; PYSPARK / PYTHON job
types both run on the pandas + GPU engine).  Each execution is a child process
started through :mod:`hops_examples_amd._job_exec`, which records its state in
``Jobs/<name>/executions/<id>/state.json`` — so state survives the launching
process.  ``spark.executor.gpus`` becomes ``HIP_VISIBLE_DEVICES`` (GPUs are handed
out round-robin), ``spark.yarn.dist.pyFiles`` zips/dirs go on ``PYTHONPATH``.
"""
from __future__ import annotations

import json
import os
import shlex
import signal
import subprocess
import sys
import time
from pathlib import Path

from . import hdfs

TERMINAL = ("FINISHED", "FAILED", "KILLED")


def _jobs_dir() -> Path:
    d = Path(hdfs.project_path()) / "Jobs"
    d.mkdir(parents=True, exist_ok=True)
    return d


def _job_dir(name: str) -> Path:
    return _jobs_dir() / name


def _resolve_app(path: str) -> str:
    return str(hdfs._resolve(path))


def create_job(name: str, job_config: dict) -> dict:
    cfg = dict(job_config)
    cfg.setdefault("appName", name)
    d = _job_dir(name)
    (d / "executions").mkdir(parents=True, exist_ok=True)
    (d / "config.json").write_text(json.dumps(cfg, indent=2))
    return {"name": name, "config": cfg, "creationTime": time.time()}


def get_job(name: str) -> dict:
    p = _job_dir(name) / "config.json"
    if not p.exists():
        raise KeyError(f"no job named {name!r}")
    return {"name": name, "config": json.loads(p.read_text())}


def get_jobs() -> list[dict]:
    return [get_job(p.name) for p in sorted(_jobs_dir().iterdir()) if (p / "config.json").exists()]


def delete_job(name: str) -> None:
    stop_job(name)
    import shutil

    shutil.rmtree(_job_dir(name), ignore_errors=True)


def _next_exec_id(name: str) -> int:
    d = _job_dir(name) / "executions"
    ids = [int(p.name) for p in d.iterdir() if p.name.isdigit()] if d.exists() else []
    return max(ids, default=0) + 1


_gpu_rr = [0]


def start_job(name: str, args: str = "", env: dict | None = None) -> dict:
    cfg = get_job(name)["config"]
    eid = _next_exec_id(name)
    ed = _job_dir(name) / "executions" / str(eid)
    ed.mkdir(parents=True)
    app = _resolve_app(cfg["appPath"])
    e = dict(os.environ)
    paths = [str(Path(__file__).resolve().parents[1])]
    for f in str(cfg.get("spark.yarn.dist.pyFiles", "") or "").split(","):
        if f.strip():
            paths.append(_resolve_app(f.strip()))
    if e.get("PYTHONPATH"):
        paths.append(e["PYTHONPATH"])
    e["PYTHONPATH"] = os.pathsep.join(paths)
    e["HOPSX_JOB_NAME"] = name
    e["HOPSX_EXECUTION_ID"] = str(eid)
    e["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    e["PYTHONUNBUFFERED"] = "1"
    gpus = int(cfg.get("spark.executor.gpus", 0) or 0)
    if gpus:
        from .experiment._runner import num_gpus

        n = max(num_gpus(), 1)
        sel = [(_gpu_rr[0] + i) % n for i in range(gpus)]
        _gpu_rr[0] += gpus
        e["HIP_VISIBLE_DEVICES"] = ",".join(map(str, sel))
    if env:
        e.update({k: str(v) for k, v in env.items()})
    cmd = [sys.executable, "-m", "hops_examples_amd._job_exec", str(ed), "--", sys.executable, app,
           *shlex.split(args or "")]
    state = {"id": eid, "job": name, "state": "INITIALIZING", "finalStatus": "UNDEFINED", "args": args,
             "submissionTime": time.time(), "stdoutPath": str(ed / "stdout.log"), "stderrPath": str(ed / "stderr.log")}
    (ed / "state.json").write_text(json.dumps(state))
    proc = subprocess.Popen(cmd, env=e, cwd=str(ed), start_new_session=True,
                            stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    state["pid"] = proc.pid
    _procs[(name, eid)] = proc
    return state


_procs: dict = {}


def _read_state(ed: Path) -> dict:
    for _ in range(5):
        try:
            return json.loads((ed / "state.json").read_text())
        except (ValueError, FileNotFoundError):
            time.sleep(0.01)
    return {"id": int(ed.name), "state": "UNKNOWN"}


def get_executions(name: str) -> list[dict]:
    d = _job_dir(name) / "executions"
    out = []
    for p in sorted((x for x in d.iterdir() if x.name.isdigit()), key=lambda x: int(x.name)) if d.exists() else []:
        s = _read_state(p)
        pr = _procs.get((name, int(p.name)))
        if pr is not None:
            pr.poll()  # reap our own children so they do not linger as zombies
        out.append(s)
    return out


def get_execution(name: str, execution_id: int) -> dict:
    return _read_state(_job_dir(name) / "executions" / str(execution_id))


def wait_for_execution(name: str, execution_id: int, timeout: float | None = None, poll: float = 0.1) -> dict:
    t0 = time.time()
    while True:
        s = get_execution(name, execution_id)
        if s.get("state") in TERMINAL:
            pr = _procs.pop((name, execution_id), None)
            if pr is not None:
                pr.wait()
            return s
        if timeout is not None and time.time() - t0 > timeout:
            raise TimeoutError(f"job {name} execution {execution_id} still {s.get('state')} after {timeout}s")
        time.sleep(poll)


def stop_job(name: str) -> None:
    """Kill running executions of this job (the process groups this module started)."""
    for s in get_executions(name) if _job_dir(name).exists() else []:
        if s.get("state") not in TERMINAL and s.get("pgid"):
            try:
                os.killpg(int(s["pgid"]), signal.SIGTERM)
            except (ProcessLookupError, PermissionError):
                pass


def get_logs(name: str, execution_id: int | None = None, stream: str = "stdout") -> str:
    ex = get_executions(name)
    if not ex:
        return ""
    s = ex[-1] if execution_id is None else get_execution(name, execution_id)
    p = Path(s["stdoutPath"] if stream == "stdout" else s["stderrPath"])
    return p.read_text(errors="replace") if p.exists() else ""
