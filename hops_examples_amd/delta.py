"""Versioned tables with a Delta-style transaction log (notebooks/featurestore/delta/DeltaOnHops.ipynb:
``write.format("delta").save`` / ``mode("overwrite")``, ``read.option("versionAsOf", v)``,
``DeltaTable.forPath(...).merge(src, "old.id = new.id").whenMatched.update(...).whenNotMatched.insert(...)
.execute()``).

Layout (compatible in spirit with Delta Lake): ``<path>/part-<uuid>.parquet`` data files and
``<path>/_delta_log/<version:020d>.json`` commits holding ``add`` / ``remove`` actions plus
``commitInfo``.  A version's snapshot = files added and not yet removed up to that commit, so
time travel never rewrites data.  pandas + pyarrow only (no Spark).
"""
from __future__ import annotations

import json
import re
import time
import uuid
from pathlib import Path

import pandas as pd
import pyarrow as pa
import pyarrow.parquet as pq

from . import hdfs


def _root(path: str) -> Path:
    return Path(hdfs._resolve(path))


def _log(p: Path) -> Path:
    return p / "_delta_log"


def _versions(p: Path) -> list[int]:
    d = _log(p)
    return sorted(int(f.stem) for f in d.glob("*.json")) if d.exists() else []


def _commit(p: Path, actions: list[dict], operation: str, params: dict | None = None) -> int:
    vs = _versions(p)
    v = vs[-1] + 1 if vs else 0
    _log(p).mkdir(parents=True, exist_ok=True)
    info = {"commitInfo": {"timestamp": int(time.time() * 1000), "operation": operation,
                           "operationParameters": params or {}, "version": v}}
    tmp = _log(p) / f".{v:020d}.json.tmp"
    tmp.write_text("\n".join(json.dumps(a) for a in [info] + actions) + "\n")
    target = _log(p) / f"{v:020d}.json"
    if target.exists():
        raise RuntimeError(f"concurrent commit to version {v}")
    tmp.rename(target)
    return v


def _actions(p: Path, v: int) -> list[dict]:
    return [json.loads(l) for l in (_log(p) / f"{v:020d}.json").read_text().splitlines() if l]


def _snapshot_files(p: Path, version: int | None = None) -> list[str]:
    vs = _versions(p)
    if not vs:
        raise FileNotFoundError(f"{p} is not a delta table")
    if version is None:
        version = vs[-1]
    if version not in vs:
        raise ValueError(f"version {version} does not exist (have {vs[0]}..{vs[-1]})")
    live: dict[str, None] = {}
    for v in vs:
        if v > version:
            break
        for a in _actions(p, v):
            if "add" in a:
                live[a["add"]["path"]] = None
            elif "remove" in a:
                live.pop(a["remove"]["path"], None)
    return list(live)


def _write_file(p: Path, df: pd.DataFrame) -> dict:
    name = f"part-{uuid.uuid4().hex}.parquet"
    pq.write_table(pa.Table.from_pandas(df, preserve_index=False), str(p / name))
    return {"add": {"path": name, "size": (p / name).stat().st_size, "numRecords": len(df),
                    "modificationTime": int(time.time() * 1000), "dataChange": True}}


def write(df: pd.DataFrame, path: str, mode: str = "errorifexists") -> int:
    """Append / overwrite a delta table; returns the committed version."""
    p = _root(path)
    exists = bool(_versions(p))
    if exists and mode in ("error", "errorifexists"):
        raise FileExistsError(f"delta table {path} exists (mode={mode})")
    if exists and mode == "ignore":
        return _versions(p)[-1]
    p.mkdir(parents=True, exist_ok=True)
    acts = []
    if exists and mode == "overwrite":
        acts += [{"remove": {"path": f, "deletionTimestamp": int(time.time() * 1000), "dataChange": True}}
                 for f in _snapshot_files(p)]
    acts.append(_write_file(p, df))
    return _commit(p, acts, "WRITE", {"mode": "Overwrite" if mode == "overwrite" else "Append"})


def read(path: str, version_as_of: int | None = None, timestamp_as_of: float | None = None) -> pd.DataFrame:
    p = _root(path)
    if timestamp_as_of is not None:
        ts = int(timestamp_as_of * 1000)
        cands = [v for v in _versions(p) if _actions(p, v)[0]["commitInfo"]["timestamp"] <= ts]
        if not cands:
            raise ValueError("no version at or before that timestamp")
        version_as_of = cands[-1]
    files = _snapshot_files(p, version_as_of)
    frames = [pq.read_table(str(p / f)).to_pandas() for f in files]
    return pd.concat(frames, ignore_index=True) if frames else pd.DataFrame()


def history(path: str) -> pd.DataFrame:
    p = _root(path)
    rows = []
    for v in reversed(_versions(p)):
        ci = _actions(p, v)[0]["commitInfo"]
        rows.append({"version": v, "timestamp": pd.Timestamp(ci["timestamp"], unit="ms"),
                     "operation": ci["operation"], "operationParameters": ci["operationParameters"]})
    return pd.DataFrame(rows)


_COND = re.compile(r"^\s*(\w+)\.(\w+)\s*=\s*(\w+)\.(\w+)\s*$")


class _Merge:
    def __init__(self, table: "DeltaTable", source: pd.DataFrame, condition: str, src_alias: str | None):
        self.t, self.src, self.cond = table, source, condition
        self.src_alias = src_alias
        self.matched_update: dict | None = None
        self.matched_delete = False
        self.insert_values: dict | None = None

    @property
    def whenMatched(self):  # noqa: N802 (Delta API spelling)
        return self

    @property
    def whenNotMatched(self):  # noqa: N802
        return self

    def whenMatchedUpdate(self, set: dict):  # noqa: N802,A002
        return self.update(set)

    def whenMatchedUpdateAll(self):  # noqa: N802
        self.matched_update = {c: c for c in self.src.columns}
        return self

    def whenMatchedDelete(self):  # noqa: N802
        self.matched_delete = True
        return self

    def whenNotMatchedInsert(self, values: dict):  # noqa: N802
        return self.insert(values)

    def whenNotMatchedInsertAll(self):  # noqa: N802
        self.insert_values = {c: c for c in self.src.columns}
        return self

    @staticmethod
    def _col(expr: str) -> str:
        return expr.split(".", 1)[1] if "." in expr else expr

    def update(self, set: dict):  # noqa: A002
        self.matched_update = {k: self._col(v) for k, v in set.items()}
        return self

    def insert(self, values: dict):
        self.insert_values = {k: self._col(v) for k, v in values.items()}
        return self

    def execute(self) -> int:
        m = _COND.match(self.cond)
        if not m:
            raise ValueError(f"merge condition must be '<t>.<col> = <s>.<col>', got {self.cond!r}")
        a1, c1, a2, c2 = m.groups()
        tcol, scol = (c1, c2) if a1 == self.t._alias else (c2, c1)
        cur = self.t.toDF()
        src = self.src
        matched = src[scol].isin(cur[tcol])
        out = cur.copy()
        if self.matched_delete:
            out = out[~out[tcol].isin(src[scol])]
        elif self.matched_update:
            s = src[matched].drop_duplicates(scol, keep="last")
            s.index = s[scol].values
            idx = out[tcol].isin(s.index)
            for tc, sc in self.matched_update.items():
                out.loc[idx, tc] = out.loc[idx, tcol].map(s[sc]).values
        n_ins = 0
        if self.insert_values:
            new = src[~matched]
            ins = pd.DataFrame({tc: new[sc].values for tc, sc in self.insert_values.items()})
            n_ins = len(ins)
            out = pd.concat([out, ins], ignore_index=True)
        p = self.t.p
        acts = [{"remove": {"path": f, "deletionTimestamp": int(time.time() * 1000), "dataChange": True}}
                for f in _snapshot_files(p)]
        acts.append(_write_file(p, out.reset_index(drop=True)))
        return _commit(p, acts, "MERGE", {"predicate": self.cond, "numTargetRowsUpdated": int(matched.sum()),
                                          "numTargetRowsInserted": n_ins})


class DeltaTable:
    def __init__(self, path: str, alias: str | None = None):
        self.path, self.p, self._alias = path, _root(path), alias

    @staticmethod
    def forPath(path: str, spark=None) -> "DeltaTable":  # noqa: N802
        if not _versions(_root(path)):
            raise FileNotFoundError(f"{path} is not a delta table")
        return DeltaTable(path)

    @staticmethod
    def isDeltaTable(path: str, spark=None) -> bool:  # noqa: N802
        return bool(_versions(_root(path)))

    def alias(self, name: str) -> "DeltaTable":
        return DeltaTable(self.path, name)

    as_ = alias

    def toDF(self) -> pd.DataFrame:  # noqa: N802
        return read(self.path)

    def history(self) -> pd.DataFrame:
        return history(self.path)

    def merge(self, source: pd.DataFrame, condition: str, source_alias: str | None = None) -> _Merge:
        return _Merge(self, source, condition, source_alias)

    def delete(self, condition=None) -> int:
        cur = self.toDF()
        keep = cur[~condition(cur)] if callable(condition) else cur.iloc[0:0]
        acts = [{"remove": {"path": f, "deletionTimestamp": int(time.time() * 1000), "dataChange": True}}
                for f in _snapshot_files(self.p)]
        acts.append(_write_file(self.p, keep))
        return _commit(self.p, acts, "DELETE")

    def vacuum(self, retain_versions: int = 1) -> int:
        """Delete data files no snapshot among the last ``retain_versions`` versions references."""
        vs = _versions(self.p)
        keep = set()
        for v in vs[-retain_versions:]:
            keep.update(_snapshot_files(self.p, v))
        n = 0
        for f in self.p.glob("part-*.parquet"):
            if f.name not in keep:
                f.unlink()
                n += 1
        return n
