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
