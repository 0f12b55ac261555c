"""Dataset upload/download into the project (``dataset.upload`` in
jobs-client/spark/jobs_spark_client.py:49-50)."""
from __future__ import annotations

import shutil
from pathlib import Path

from . import hdfs


def upload(local_path: str, dataset_path: str, overwrite: bool = True) -> str:
    src = Path(local_path)
    dst_dir = Path(hdfs._resolve(dataset_path))
    dst_dir.mkdir(parents=True, exist_ok=True)
    dst = dst_dir / src.name
    if dst.exists() and not overwrite:
        raise FileExistsError(dst)
    if src.is_dir():
        shutil.copytree(src, dst, dirs_exist_ok=True)
    else:
        shutil.copy2(src, dst)
    return str(dst)


def download(dataset_path: str, local_path: str = ".") -> str:
    src = Path(hdfs._resolve(dataset_path))
    dst = Path(local_path) / src.name
    if src.is_dir():
        shutil.copytree(src, dst, dirs_exist_ok=True)
    else:
        dst.parent.mkdir(parents=True, exist_ok=True)
        shutil.copy2(src, dst)
    return str(dst)


def delete(dataset_path: str) -> None:
    hdfs.rmr(dataset_path)


def sample_data(name: str = "") -> str:
    """Local path of a bundled sample dataset: the data files the reference notebooks ship
    (notebooks/featurestore/aws/s3/data/telco_customer_churn.csv and its ``telco-delta`` Delta
    table, notebooks/featurestore/aws/data/Sacramentorealestatetransactions.csv, the retail
    ``hsfs/archive`` CSVs), copied into ``tests/fixtures``.  ``HOPSX_SAMPLE_DATA`` overrides the
    directory."""
    import os

    base = os.environ.get("HOPSX_SAMPLE_DATA")
    root = Path(base) if base else Path(os.environ.get("HOPSX_REPO", Path(__file__).resolve().parent.parent)) / \
        "tests" / "fixtures"
    p = root / name
    if not p.exists():
        raise FileNotFoundError(f"sample dataset {name!r} not found under {root}")
    return str(p)
