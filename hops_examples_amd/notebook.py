"""Notebook <-> cluster boundary helpers (Livy / sparkmagic).

The reference's notebooks run PySpark through a Livy session and move results to the notebook
kernel with sparkmagic cell magics: ``%%sql -o df`` runs SQL on the cluster and binds the result as
a local pandas DataFrame, ``%%spark -o df`` exports a Spark DataFrame, ``%%local`` runs a cell on
the notebook host (notebooks/ml/Plotting/matplotlib_sparkmagic.ipynb:176,301-403).  With hopsx the
"cluster" is this node, so the boundary collapses to functions:

* :func:`sql` — run SQL against the Hive warehouse (``hive``) or the feature store (``fs.sql``)
  and optionally bind the pandas result under ``output`` in a namespace (the ``-o`` flag);
* :func:`local` — run a callable "locally" (a no-op boundary, kept so notebook code ports 1:1);
* :class:`Session` — the Livy session table of the reference (id, kind, state, driver log link).
"""
from __future__ import annotations

import itertools
import time

import pandas as pd

_ids = itertools.count()
NAMESPACE: dict = {}


def sql(query: str, output: str | None = None, engine: str = "hive", namespace: dict | None = None,
        max_rows: int | None = None) -> pd.DataFrame:
    """``%%sql -o <output>``: run ``query`` and return (and bind) a pandas DataFrame."""
    if engine == "hive":
        from . import hive

        df = hive.sql(query)
    elif engine in ("featurestore", "hsfs"):
        from .featurestore import connection

        df = connection().get_feature_store().sql(query)
    else:
        raise ValueError(f"engine must be 'hive' or 'featurestore', got {engine!r}")
    if df is None:
        df = pd.DataFrame()
    if max_rows is not None:
        df = df.head(max_rows)
    if output:
        (NAMESPACE if namespace is None else namespace)[output] = df
    return df


def local(fn, *args, **kwargs):
    """``%%local``: the cell runs on this host (it always does here)."""
    return fn(*args, **kwargs)


class Session:
    """A Livy-style session record (the table the reference prints when a session starts)."""

    def __init__(self, kind: str = "pyspark"):
        self.id = next(_ids)
        self.kind = kind
        self.state = "idle"
        self.started = time.time()

    def info(self) -> dict:
        from .experiment import _runner

        return {"ID": self.id, "Kind": self.kind, "State": self.state, "Spark UI": None,
                "Driver log": None, "Executors": _runner.num_gpus() or 1}
