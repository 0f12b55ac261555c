"""``hops.pandas_helper``: pandas CSV/Parquet IO with project-relative paths
(notebooks/ml/pandas/pandas-hdfs.ipynb:58-69)."""
from __future__ import annotations

import os

import pandas as pd

from . import hdfs


def read_csv(path: str, **kw) -> pd.DataFrame:
    return pd.read_csv(hdfs.abs_path(path), **kw)


def write_csv(path: str, df: pd.DataFrame, index: bool = False, **kw) -> None:
    p = hdfs.abs_path(path)
    os.makedirs(os.path.dirname(p) or ".", exist_ok=True)
    df.to_csv(p, index=index, **kw)


def read_parquet(path: str, **kw) -> pd.DataFrame:
    return pd.read_parquet(hdfs.abs_path(path), **kw)


def write_parquet(path: str, df: pd.DataFrame, **kw) -> None:
    p = hdfs.abs_path(path)
    os.makedirs(os.path.dirname(p) or ".", exist_ok=True)
    df.to_parquet(p, **kw)
