"""``hops.util`` helpers used by the notebooks."""
from __future__ import annotations

import os

from . import config


def num_executors() -> int:
    """Parallel workers available to a job on this node (one per GPU, or CPU slots)."""
    from .experiment._runner import num_gpus

    n = num_gpus()
    return n if n else max(1, (os.cpu_count() or 2) // 2)


def num_param_servers() -> int:
    return config.get().num_ps


def get_job_name() -> str:
    return os.environ.get("HOPSX_JOB_NAME", "notebook")


def project_name() -> str:
    return config.get().project_name
