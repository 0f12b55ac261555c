"""Project context (``project.connect`` in jobs-client/spark/jobs_spark_client.py:45-47).

A project is a directory (the HopsFS project root stand-in); connecting selects it
for every other module (hdfs, jobs, featurestore, model registry).  API keys are
accepted for signature compatibility but never stored or printed.
"""
from __future__ import annotations

from pathlib import Path

from . import config


def connect(project: str, host: str | None = None, port: int | str = 443, api_key: str | None = None,
            region_name: str | None = None, secrets_store: str | None = None, hostname_verification: bool = True,
            trust_store_path: str | None = None, project_root: str | None = None) -> dict:
    cur = config.get()
    root = Path(project_root) if project_root else (cur.project_root.parent / project
                                                    if project != cur.project_name else cur.project_root)
    config.set(project_name=project, project_root=str(root))
    root.mkdir(parents=True, exist_ok=True)
    for d in ("Resources", "Jobs", "Experiments", "Models", "Logs", "DataValidation"):
        (root / d).mkdir(exist_ok=True)
    return get_project_info(project)


def create(project: str, description: str = "") -> dict:
    return connect(project)


def get_project_info(project: str | None = None) -> dict:
    c = config.get()
    return {"projectName": project or c.project_name, "projectPath": str(c.project_root), "owner": c.user}
