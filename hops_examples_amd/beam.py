"""Portable-runner lifecycle (``hops.beam.create_runner/start_runner``,
jobs-client/flink/jobs_flink_client.py:45-51).

Beam/Flink are not in the image; a "runner" here is a named job-server record whose
pipelines execute as jobs through :mod:`hops_examples_amd.jobs` (so they get the
same execution tracking, logs and GPU assignment).
"""
from __future__ import annotations

import json
from pathlib import Path

from . import hdfs, jobs


def _rdir() -> Path:
    d = Path(hdfs.project_path()) / "Jobs" / "_runners"
    d.mkdir(parents=True, exist_ok=True)
    return d


def create_runner(runner_name: str, jobmanager_heap_size: int = 1024, num_of_taskmanagers: int = 1,
                  taskmanager_heap_size: int = 4096, num_task_slots: int = 1) -> dict:
    cfg = {"name": runner_name, "state": "CREATED", "taskmanagers": num_of_taskmanagers,
           "slots": num_task_slots, "jobmanager_heap": jobmanager_heap_size, "taskmanager_heap": taskmanager_heap_size}
    (_rdir() / f"{runner_name}.json").write_text(json.dumps(cfg))
    return cfg


def start_runner(runner_name: str) -> dict:
    p = _rdir() / f"{runner_name}.json"
    cfg = json.loads(p.read_text())
    cfg["state"] = "RUNNING"
    p.write_text(json.dumps(cfg))
    return cfg


def get_runner_state(runner_name: str) -> str:
    return json.loads((_rdir() / f"{runner_name}.json").read_text())["state"]


def stop_runner(runner_name: str) -> dict:
    p = _rdir() / f"{runner_name}.json"
    cfg = json.loads(p.read_text())
    cfg["state"] = "STOPPED"
    p.write_text(json.dumps(cfg))
    return cfg


def run_pipeline(runner_name: str, app_path: str, args: str = "") -> dict:
    """Submit a pipeline program to a RUNNING runner; returns the job execution record."""
    if get_runner_state(runner_name) != "RUNNING":
        raise RuntimeError(f"runner {runner_name} is not running")
    name = f"{runner_name}-pipeline"
    jobs.create_job(name, {"appPath": app_path, "jobType": "PYTHON"})
    return jobs.start_job(name, args)
