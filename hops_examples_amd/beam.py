"""Portable-runner lifecycle and its REST client (``hops.beam.create_runner/start_runner`` and the
Flink REST calls of jobs-client/flink/jobs_flink_client.py:29-121).

A runner is a job (:mod:`hops_examples_amd.jobs`) whose program is :mod:`hops_examples_amd.beam_runner`
— a job-manager REST server with task slots that runs uploaded programs.  ``start_runner`` launches
it; ``wait_until_running`` polls the execution until it is RUNNING and has published its endpoint
(the reference waits 90 s in 5 s steps, :52-69); ``find_running`` reuses a runner that is already up
(:38-43, 70-72); ``upload_program`` / ``run_program`` are the ``/jars/upload`` and
``/jars/<id>/run`` calls, and REST failures raise :class:`~hops_examples_amd.exceptions.RestAPIError`
with the reference's message shape (:111-119).
"""
from __future__ import annotations

import json
import os
import time
import urllib.error
import urllib.parse
import urllib.request
import uuid
from pathlib import Path

from . import jobs
from .exceptions import RestAPIError

RUNNER_APP = str(Path(__file__).resolve().parent / "beam_runner.py")


def create_runner(runner_name: str, jobmanager_heap_size: int = 1024, num_of_taskmanagers: int = 1,
                  taskmanager_heap_size: int = 4096, num_task_slots: int = 1) -> dict:
    cfg = {"appPath": RUNNER_APP, "jobType": "FLINK", "jobmanager.heap.size": int(jobmanager_heap_size),
           "taskmanager.heap.size": int(taskmanager_heap_size), "numberOfTaskManagers": int(num_of_taskmanagers),
           "taskmanager.numberOfTaskSlots": int(num_task_slots),
           "defaultArgs": f"--slots {int(num_task_slots)} --taskmanagers {int(num_of_taskmanagers)}"}
    return jobs.create_job(runner_name, cfg)


def start_runner(runner_name: str) -> dict:
    """Start the runner job; returns its execution record (state INITIALIZING until it is up)."""
    cfg = jobs.get_job(runner_name)["config"]
    return jobs.start_job(runner_name, cfg.get("defaultArgs", ""))


def _endpoint_of(execution: dict) -> str | None:
    p = Path(execution["stdoutPath"]).parent / "runner.json"
    try:
        return json.loads(p.read_text())["endpoint"]
    except (FileNotFoundError, ValueError, KeyError):
        return None


def find_running(runner_name: str) -> dict | None:
    """The newest execution of the runner that is RUNNING with a published endpoint, or None."""
    try:
        ex = jobs.get_executions(runner_name)
    except KeyError:
        return None
    for e in reversed(ex):
        if e.get("state") == "RUNNING":
            ep = _endpoint_of(e)
            if ep:
                return dict(e, endpoint=ep, appId=str(e["id"]))
    return None


def wait_until_running(runner_name: str, wait: float = 90.0, step: float = 5.0) -> dict | None:
    """Poll until the runner is RUNNING and reachable (the reference's 90 s / 5 s loop); None on timeout
    or when the runner's execution ended."""
    t0 = time.time()
    while True:
        e = find_running(runner_name)
        if e is not None:
            try:
                overview(e["endpoint"])
                return e
            except RestAPIError:
                pass
        ex = jobs.get_executions(runner_name)
        if ex and ex[-1].get("state") in jobs.TERMINAL:
            return None
        if time.time() - t0 >= wait:
            return None
        time.sleep(min(step, max(0.01, wait - (time.time() - t0))))


def get_runner_state(runner_name: str) -> str:
    ex = jobs.get_executions(runner_name)
    return ex[-1]["state"] if ex else "CREATED"


def stop_runner(runner_name: str) -> None:
    jobs.stop_job(runner_name)


# ------------------------------------------------------------------ REST client
def _parse_rest_error(obj) -> tuple[str, str, str]:
    """(error code, error msg, user msg) of an error response (hops util._parse_rest_error shape)."""
    if isinstance(obj, dict):
        if "errors" in obj:
            msg = "; ".join(map(str, obj["errors"]))
            return "", msg, msg
        return str(obj.get("errorCode", "")), str(obj.get("errorMsg", "")), str(obj.get("usrMsg", ""))
    return "", "", ""


def _request(method: str, url: str, body: bytes | None = None, headers: dict | None = None) -> dict:
    req = urllib.request.Request(url, data=body, method=method, headers=headers or {})
    try:
        with urllib.request.urlopen(req, timeout=30) as r:
            data = r.read()
            return json.loads(data) if data else {}
    except urllib.error.HTTPError as e:
        try:
            obj = json.loads(e.read())
        except ValueError:
            obj = None
        code, msg, user = _parse_rest_error(obj)
        raise RestAPIError("Could not execute HTTP request (url: {}), server response: \n HTTP code: {}, HTTP reason: {}, "
                           "error code: {}, error msg: {}, user msg: {}".format(url, e.code, e.reason, code, msg, user),
                           status=e.code) from None
    except urllib.error.URLError as e:
        raise RestAPIError(f"Could not execute HTTP request (url: {url}): {e.reason}") from None


def overview(endpoint: str) -> dict:
    return _request("GET", endpoint + "/overview")


def upload_program(endpoint: str, path: str) -> str:
    """``POST /jars/upload`` (multipart ``jarfile`` part, as the reference's requests call); returns the
    program id to run."""
    name = os.path.basename(path)
    boundary = uuid.uuid4().hex
    data = Path(path).read_bytes()
    body = (f"--{boundary}\r\nContent-Disposition: form-data; name=\"jarfile\"; filename=\"{name}\"\r\n"
            f"Content-Type: application/octet-stream\r\n\r\n").encode() + data + f"\r\n--{boundary}--\r\n".encode()
    r = _request("POST", endpoint + "/jars/upload", body, {"Content-Type": f"multipart/form-data; boundary={boundary}"})
    return r["filename"].split("/")[-1]


def run_program(endpoint: str, program_id: str, entry_class: str = "", args: str = "") -> str:
    q = urllib.parse.urlencode({"entry-class": entry_class, "program-args": args})
    return _request("POST", f"{endpoint}/jars/{program_id}/run?{q}", b"", {"Content-Type": "application/json"})["jobid"]


def job_status(endpoint: str, job_id: str) -> dict:
    return _request("GET", f"{endpoint}/jobs/{job_id}")


def wait_job(endpoint: str, job_id: str, timeout: float = 300.0, poll: float = 0.1) -> dict:
    t0 = time.time()
    while True:
        s = job_status(endpoint, job_id)
        if s["state"] != "RUNNING":
            return s
        if time.time() - t0 > timeout:
            raise TimeoutError(f"job {job_id} still running after {timeout}s")
        time.sleep(poll)


def run_pipeline(runner_name: str, app_path: str, args: str = "", entry_class: str = "") -> dict:
    """Submit a pipeline program to a RUNNING runner; returns {'jobid', 'endpoint'}."""
    e = find_running(runner_name)
    if e is None:
        raise RuntimeError(f"runner {runner_name} is not running")
    pid = upload_program(e["endpoint"], app_path)
    return {"jobid": run_program(e["endpoint"], pid, entry_class, args), "endpoint": e["endpoint"]}
