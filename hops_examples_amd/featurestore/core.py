"""hsfs-compatible feature store on a local engine (pandas + Parquet commit logs +
SQLite for SQL and the online store) with GPU-accelerated statistics.

Surface and output contracts re-provided from the reference notebooks:
  connection / get_feature_store ........ hsfs/basics/feature_engineering.ipynb:90-94
  create_feature_group / save / insert .. feature_engineering.ipynb:177-206, 289-346, 400-442
  get_feature_group + VersionWarning .... hsfs/basics/feature_exploration.ipynb:93
  select / filter / join / to_string .... feature_exploration.ipynb:389-396, 533-611
  HUDI time travel, commit_details ....... hsfs/time_travel/time_travel_python.ipynb:284-1281
  training datasets, splits, tf_data .... hsfs/basics/training_datasets.ipynb:108-526
  online serving vectors ................ hsfs/serving/feature_vector_model_serving.ipynb:61-254
  tags .................................. hsfs/tags/feature_store_tags.ipynb
  validation ............................ hsfs/data_validation/feature_validation_python.ipynb
The engine is pandas in-process instead of Spark; HUDI upserts/time travel are
an append-only Parquet commit log per feature group version; SQL (queries and
``fs.sql``) runs on SQLite with the feature store attached as a schema, so the
generated SQL is executed verbatim.
"""
from __future__ import annotations

import datetime as _dt
import json
import os
import random
import sqlite3
import time
import warnings
from pathlib import Path

import numpy as np
import pandas as pd

from .. import config, hdfs
from . import rules as R
from . import statistics as ST


def _camel_to_snake(name: str) -> str:
    import re

    return re.sub(r"(?<!^)(?=[A-Z])", "_", name).lower()


class VersionWarning(Warning):
    pass


class FeatureStoreException(Exception):
    pass


def _warn_version(kind: str, name: str):
    msg = f"VersionWarning: No version provided for getting {kind} `{name}`, defaulting to `1`."
    print(msg)
    warnings.warn(msg[len("VersionWarning: "):], VersionWarning, stacklevel=3)


# ---------------------------------------------------------------- type mapping
def _hsfs_type(dtype) -> str:
    k = np.dtype(dtype).kind if not isinstance(dtype, pd.CategoricalDtype) else "O"
    if str(dtype).startswith("datetime64"):
        return "timestamp"
    if k == "b":
        return "boolean"
    if k in "iu":
        return "bigint" if np.dtype(dtype).itemsize == 8 else "int"
    if k == "f":
        return "double" if np.dtype(dtype).itemsize == 8 else "float"
    return "string"


def _to_pandas(df) -> pd.DataFrame:
    if isinstance(df, pd.DataFrame):
        return df.copy()
    if hasattr(df, "toPandas"):
        return df.toPandas()
    if hasattr(df, "to_pandas"):
        return df.to_pandas()
    if isinstance(df, dict):
        return pd.DataFrame(df)
    if isinstance(df, np.ndarray):
        return pd.DataFrame(df, columns=[f"f{i}" for i in range(df.shape[1])])
    raise TypeError(f"unsupported dataframe type {type(df)}")


def _spark_show(df: pd.DataFrame, n: int) -> None:
    """Print like Spark's DataFrame.show (the format of the reference notebook outputs)."""
    head = df.head(n)
    cols = [str(c) for c in head.columns]
    rows = [[("null" if (isinstance(v, float) and np.isnan(v)) or v is None else str(v)) for v in r]
            for r in head.itertuples(index=False)]
    widths = [max([len(c)] + [len(r[i]) for r in rows]) for i, c in enumerate(cols)]
    sep = "+" + "+".join("-" * w for w in widths) + "+"
    print(sep)
    print("|" + "|".join(c.rjust(w) for c, w in zip(cols, widths)) + "|")
    print(sep)
    for r in rows:
        print("|" + "|".join(v.rjust(w) for v, w in zip(r, widths)) + "|")
    print(sep)
    if len(df) > n:
        print(f"only showing top {n} rows")


def _commit_time(ts) -> int:
    """Accept ms epoch, 'YYYYMMDDhhmmss' (committedOn), 'YYYY-MM-DD hh:mm:ss' or datetime -> ms."""
    if ts is None:
        return 2 ** 62
    if isinstance(ts, _dt.datetime):
        return int(ts.timestamp() * 1000)
    if isinstance(ts, (int, np.integer)) and ts > 10 ** 11:
        return int(ts)
    s = str(ts)
    for fmt in ("%Y%m%d%H%M%S", "%Y%m%d%H%M%S%f", "%Y-%m-%d %H:%M:%S", "%Y-%m-%d", "%Y%m%d"):
        try:
            return int(_dt.datetime.strptime(s, fmt).timestamp() * 1000)
        except ValueError:
            continue
    raise ValueError(f"unrecognised commit time {ts!r}")


# ======================================================================= Feature
class Feature:
    def __init__(self, name: str, type: str = "double", description: str = "", primary: bool = False,
                 partition: bool = False, hudi_precombine_key: bool = False, default_value=None, fg=None):
        self.name, self.type, self.description = name, type, description
        self.primary, self.partition, self.hudi_precombine_key = primary, partition, hudi_precombine_key
        self.default_value = default_value
        self._fg = fg

    # comparison operators build filters
    def _f(self, op, v):
        return Filter(self, op, v)

    def __lt__(self, v):
        return self._f("<", v)

    def __le__(self, v):
        return self._f("<=", v)

    def __gt__(self, v):
        return self._f(">", v)

    def __ge__(self, v):
        return self._f(">=", v)

    def __eq__(self, v):  # noqa: D105
        if isinstance(v, Feature):
            return self is v
        return self._f("=", v)

    def __ne__(self, v):
        return self._f("!=", v)

    def __hash__(self):
        return hash((self.name, id(self._fg)))

    def like(self, pattern):
        return self._f("LIKE", pattern)

    def isin(self, values):
        return self._f("IN", list(values))

    def to_dict(self):
        return {"name": self.name, "type": self.type, "description": self.description, "primary": self.primary,
                "partition": self.partition, "hudiPrecombineKey": self.hudi_precombine_key,
                "defaultValue": self.default_value}

    def __repr__(self):
        return f"Feature({self.name!r}, {self.type!r}, primary={self.primary}, partition={self.partition})"


def _lit(v) -> str:
    if isinstance(v, str):
        return "'" + v.replace("'", "''") + "'"
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, (list, tuple)):
        return "(" + ", ".join(_lit(x) for x in v) + ")"
    return str(v)


class Filter:
    def __init__(self, feature: Feature, op: str, value):
        self.feature, self.op, self.value = feature, op, value

    def __and__(self, o):
        return Logic("AND", self, o)

    def __or__(self, o):
        return Logic("OR", self, o)

    def sql(self, alias_of) -> str:
        return f"`{alias_of(self.feature._fg)}`.`{self.feature.name}` {self.op} {_lit(self.value)}"

    def mask(self, df: pd.DataFrame) -> pd.Series:
        s = df[self.feature.name]
        v = self.value
        return {
            "<": lambda: s < v, "<=": lambda: s <= v, ">": lambda: s > v, ">=": lambda: s >= v,
            "=": lambda: s == v, "!=": lambda: s != v, "IN": lambda: s.isin(v),
            "LIKE": lambda: s.astype(str).str.match("^" + str(v).replace("%", ".*").replace("_", ".") + "$"),
        }[self.op]()


class Logic:
    def __init__(self, op: str, left, right):
        self.op, self.left, self.right = op, left, right

    def __and__(self, o):
        return Logic("AND", self, o)

    def __or__(self, o):
        return Logic("OR", self, o)

    def sql(self, alias_of) -> str:
        l, r = self.left.sql(alias_of), self.right.sql(alias_of)
        return f"{l} AND {r}" if self.op == "AND" else f"({l} OR {r})"

    def mask(self, df):
        a, b = self.left.mask(df), self.right.mask(df)
        return a & b if self.op == "AND" else a | b


# ========================================================================= Query
class JoinType:
    INNER, LEFT, RIGHT, FULL, CROSS, LEFT_SEMI_JOIN, COMMA = "INNER", "LEFT", "RIGHT", "FULL", "CROSS", \
        "LEFT_SEMI_JOIN", "COMMA"


_JOIN_SQL = {"INNER": "INNER JOIN", "LEFT": "LEFT JOIN", "RIGHT": "RIGHT JOIN", "FULL": "FULL JOIN",
             "CROSS": "CROSS JOIN", "LEFT_SEMI_JOIN": "LEFT SEMI JOIN", "COMMA": ","}


class Join:
    def __init__(self, query, on, left_on, right_on, join_type):
        self.query, self.on, self.left_on, self.right_on, self.join_type = query, on, left_on, right_on, join_type


class Query:
    def __getattr__(self, name):  # JVM-style camelCase (asOf, selectAll ...)
        if name.startswith("_") or not any(c.isupper() for c in name):
            raise AttributeError(name)
        return object.__getattribute__(self, _camel_to_snake(name))

    def __init__(self, fg, features: list[Feature]):
        self._left_fg = fg
        self._left_features = features
        self._joins: list[Join] = []
        self._filter = None
        self._as_of = None

    # ------------------------------------------------------------ building
    def join(self, sub_query: "Query", on: list | None = None, left_on: list | None = None,
             right_on: list | None = None, join_type: str = "inner", prefix=None) -> "Query":
        if sub_query._joins:
            raise FeatureStoreException("Nested joins are not supported")
        if isinstance(on, str):
            on = [on]
        jt = str(join_type).upper()
        if on is None and left_on is None:
            on = [k for k in self._left_fg.primary_key if k in sub_query._left_fg.primary_key]
            if not on:
                raise FeatureStoreException("Cannot join feature groups without common primary keys; "
                                            "pass on= or left_on=/right_on=")
            # the order Hopsworks' query constructor emits the implicit keys in: the left feature group's
            # primary-key order for the first join, reversed for every later one — feature_exploration.ipynb
            # prints `store` AND `date` for sales <> exogenous (:535) but `date` AND `store` when that join
            # follows sales <> store (:574, :610)
            if self._joins:
                on = on[::-1]
        self._joins.append(Join(sub_query, on or [], left_on or [], right_on or [], jt))
        return self

    def filter(self, f) -> "Query":
        self._filter = f if self._filter is None else Logic("AND", self._filter, f)
        return self

    def as_of(self, wallclock_time) -> "Query":
        self._as_of = wallclock_time
        for j in self._joins:
            j.query._as_of = wallclock_time
        return self

    # ------------------------------------------------------------ SQL
    def _fgs(self):
        return [j.query._left_fg for j in self._joins] + [self._left_fg]

    def _alias_of(self, fg):
        order = self._fgs()
        for i, g in enumerate(order):
            if g is fg or (g.name == fg.name and g.version == fg.version):
                return f"fg{i}"
        raise FeatureStoreException(f"feature group {fg.name} is not part of the query")

    def _select_cols(self, fg, feats, drop: set):
        out = []
        for f in feats:
            if f.name in drop:
                continue
            a = self._alias_of(fg)
            if f.default_value is not None:
                out.append(f"CASE WHEN `{a}`.`{f.name}` IS NULL THEN {_lit(f.default_value)} ELSE "
                           f"`{a}`.`{f.name}` END `{f.name}`")
            else:
                out.append(f"`{a}`.`{f.name}`")
        return out

    def to_string(self, online: bool = False) -> str:
        db = self._left_fg._fs.name
        cols = self._select_cols(self._left_fg, self._left_features, set())
        for j in self._joins:
            drop = set(j.on) | set(j.right_on)
            cols += self._select_cols(j.query._left_fg, j.query._left_features, drop)
        la = self._alias_of(self._left_fg)
        sql = "SELECT " + ", ".join(cols) + f"\nFROM `{db}`.`{self._left_fg._table}` `{la}`"
        for j in self._joins:
            ra = self._alias_of(j.query._left_fg)
            if j.on:
                cond = " AND ".join(f"`{la}`.`{k}` = `{ra}`.`{k}`" for k in j.on)
            else:
                cond = " AND ".join(f"`{la}`.`{a}` = `{ra}`.`{b}`" for a, b in zip(j.left_on, j.right_on))
            if j.join_type in ("CROSS", "COMMA"):
                sql += f"\n{_JOIN_SQL[j.join_type]} `{db}`.`{j.query._left_fg._table}` `{ra}`"
            else:
                sql += f"\n{_JOIN_SQL.get(j.join_type, 'INNER JOIN')} `{db}`.`{j.query._left_fg._table}` `{ra}` ON {cond}"
        filters = []
        if self._filter is not None:
            filters.append(self._filter.sql(self._alias_of))
        for j in self._joins:
            if j.query._filter is not None:
                filters.append(j.query._filter.sql(self._alias_of))
        if filters:
            sql += "\nWHERE " + " AND ".join(filters)
        return sql

    # ------------------------------------------------------------ execution
    def read(self, online: bool = False, dataframe_type: str = "default", read_options=None) -> pd.DataFrame:
        fs = self._left_fg._fs
        frames = {}
        for fg in self._fgs():
            q = self if fg is self._left_fg else next(j.query for j in self._joins if j.query._left_fg is fg)
            frames[fg._table] = fg._read_df(online=online, as_of=q._as_of)
        return fs._run_sql(self.to_string(online), frames)

    def show(self, n: int = 20, online: bool = False) -> None:
        _spark_show(self.read(online), n)

    def __str__(self):
        return self.to_string()

    @property
    def features(self):
        out = list(self._left_features)
        for j in self._joins:
            out += [f for f in j.query._left_features if f.name not in set(j.on) | set(j.right_on)]
        return out


# ================================================================== FeatureGroup
class FeatureGroupBase:
    def __getattr__(self, name):
        if name.startswith("_"):
            raise AttributeError(name)
        for f in self.__dict__.get("_features", []):
            if f.name == name:
                return f
        if any(c.isupper() for c in name):  # JVM-style camelCase method (builders.CamelCaseAPI)
            sn = _camel_to_snake(name)
            if sn != name:
                try:
                    return object.__getattribute__(self, sn)
                except AttributeError:
                    pass
        raise AttributeError(f"'{type(self).__name__}' has no feature or attribute {name!r}")

    def getValidation(self, time, time_type="VALIDATION_TIME"):  # noqa: N802 (JVM API)
        """``fg.getValidation(ts, ValidationTimeType.COMMIT_TIME)`` (feature_validation_scala.ipynb:741-765)."""
        if str(time_type).upper() == "COMMIT_TIME":
            return self.get_validations(commit_time=time)
        return self.get_validations(validation_time=time)

    def __getitem__(self, name):
        return self.__getattr__(name)

    @property
    def features(self):
        return self._features

    @property
    def schema(self):
        return self._features

    def get_feature(self, name):
        return self.__getattr__(name)

    def select_all(self) -> Query:
        return Query(self, list(self._features))

    def select(self, features: list) -> Query:
        names = [f if isinstance(f, str) else f.name for f in features]
        lookup = {f.name: f for f in self._features}
        missing = [n for n in names if n not in lookup]
        if missing:
            raise FeatureStoreException(f"features {missing} not in feature group {self.name}")
        return Query(self, [lookup[n] for n in names])

    def select_except(self, features: list) -> Query:
        ex = {f if isinstance(f, str) else f.name for f in features}
        return Query(self, [f for f in self._features if f.name not in ex])

    def filter(self, f) -> Query:
        return self.select_all().filter(f)

    # ---- tags (JSON-schema typed tags, feature_store_tags.ipynb)
    def add_tag(self, name: str, value) -> None:
        self._fs._tags.check(name, value)
        self._meta.setdefault("tags", {})[name] = value
        self._persist()

    def get_tag(self, name: str):
        return self._meta.get("tags", {}).get(name)

    def get_tags(self) -> dict:
        return dict(self._meta.get("tags", {}))

    def delete_tag(self, name: str) -> None:
        self._meta.get("tags", {}).pop(name, None)
        self._persist()


class FeatureGroup(FeatureGroupBase):
    ENTITY_TYPE = "featuregroups"

    def __init__(self, fs, name, version, description="", primary_key=None, partition_key=None,
                 online_enabled=False, time_travel_format=None, statistics_config=None, hudi_precombine_key=None,
                 validation_type="NONE", expectations=None, features=None, meta=None):
        self._fs = fs
        self.name, self.version, self.description = name, int(version), description or ""
        self.primary_key = list(primary_key or [])
        self.partition_key = list(partition_key or [])
        self.online_enabled = bool(online_enabled)
        self.time_travel_format = (time_travel_format or "NONE").upper() if time_travel_format else None
        self.hudi_precombine_key = hudi_precombine_key or (self.primary_key[0] if self.time_travel_format == "HUDI"
                                                           and self.primary_key else None)
        self.statistics_config = ST.StatisticsConfig.parse(statistics_config)
        self._validation_type = (validation_type or "NONE").upper()
        self._features = features or []
        for f in self._features:
            f._fg = self
        self._meta = meta or {"tags": {}, "expectations": [e if isinstance(e, str) else e.name
                                                           for e in (expectations or [])]}
        for e in expectations or []:
            if not isinstance(e, str):
                fs._save_expectation(e)
        self.created = self._meta.get("created")
        self.id = self._meta.get("id")

    # ------------------------------------------------------------- paths
    @property
    def _table(self):
        return f"{self.name}_{self.version}"

    @property
    def _dir(self) -> Path:
        return self._fs._root / self._table

    @property
    def location(self):
        return str(self._dir)

    def _commits(self) -> list[dict]:
        p = self._dir / "commits.json"
        return json.loads(p.read_text()) if p.exists() else []

    def _persist(self):
        self._meta.update({
            "name": self.name, "version": self.version, "description": self.description,
            "primary_key": self.primary_key, "partition_key": self.partition_key,
            "online_enabled": self.online_enabled, "time_travel_format": self.time_travel_format,
            "hudi_precombine_key": self.hudi_precombine_key, "statistics_config": self.statistics_config.to_dict(),
            "validation_type": self._validation_type, "features": [f.to_dict() for f in self._features],
            "type": "cached",
        })
        self._fs._write_meta(self.ENTITY_TYPE, self._table, self._meta)

    # ------------------------------------------------------------- writes
    def _schema_from(self, df: pd.DataFrame):
        if not self._features:
            self._features = [Feature(c, _hsfs_type(df[c].dtype), primary=c in self.primary_key,
                                      partition=c in self.partition_key,
                                      hudi_precombine_key=c == self.hudi_precombine_key, fg=self)
                              for c in df.columns]
        else:
            names = {f.name for f in self._features}
            extra = [c for c in df.columns if c not in names]
            if extra:
                raise FeatureStoreException(f"dataframe has features {extra} not in the schema of {self.name}; "
                                            "use append_features() first")

    def save(self, features, write_options: dict | None = None):
        """Create the feature group (first commit = bulk insert)."""
        df = _to_pandas(features)
        if self._commits():
            raise FeatureStoreException(f"feature group {self.name} v{self.version} already exists; use insert()")
        if self.id is None:
            self.id = self._fs._next_id()
            self._meta["id"] = self.id
            self.created = time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime())
            self._meta["created"] = self.created
        self._schema_from(df)
        self._persist()
        self._write(df, "bulk_insert", write_options)
        return self

    def insert(self, features, overwrite: bool = False, operation: str = "upsert", storage: str | None = None,
               write_options: dict | None = None):
        df = _to_pandas(features)
        if not self._commits() and self.id is None:
            return self.save(df, write_options)
        self._schema_from(df)
        self._write(df, "overwrite" if overwrite else operation, write_options, storage)

    def _write(self, df: pd.DataFrame, op: str, write_options, storage=None):
        for f in self._features:
            if f.name not in df.columns and f.default_value is not None:
                df[f.name] = f.default_value
        # -- validation gate (STRICT / WARNING / ALL / NONE)
        if self._validation_type != "NONE" and self.get_expectations():
            v = self.validate(df, _persist=False)
            allowed = {"STRICT": ("SUCCESS",), "WARNING": ("SUCCESS", "WARNING"),
                       "ALL": ("SUCCESS", "WARNING", "FAILURE")}[self._validation_type]
            if v.status not in allowed:
                raise R.ValidationError(v)
        commits = self._commits()
        now = int(time.time()) * 1000
        if commits and now <= commits[-1]["ts"]:
            now = commits[-1]["ts"] + 1000  # strictly increasing commit times (second resolution)
        self._dir.mkdir(parents=True, exist_ok=True)
        if storage != "online":
            prev = self._read_df(as_of=None) if commits else pd.DataFrame(columns=df.columns)
            inserted, updated = len(df), 0
            if self.time_travel_format == "HUDI" and self.primary_key and len(prev):
                keys = set(map(tuple, prev[self.primary_key].astype(str).to_numpy()))
                upd = np.array([tuple(r) in keys for r in df[self.primary_key].astype(str).to_numpy()])
                updated = int(upd.sum())
                inserted = len(df) - updated
            fname = f"commit_{now}.parquet"
            df.to_parquet(self._dir / fname, index=False)
            ct = time.strftime("%Y%m%d%H%M%S", time.localtime(now / 1000))
            commits.append({"ts": now, "committedOn": ct, "rowsInserted": inserted, "rowsUpdated": updated,
                            "rowsDeleted": 0, "file": fname, "op": op})
            (self._dir / "commits.json").write_text(json.dumps(commits))
        if self.online_enabled and storage != "offline":
            self._fs._online.upsert(self, df)
        if self.statistics_config.enabled and storage != "online":
            try:
                self.compute_statistics()
            except Exception:  # statistics never block ingestion
                pass
        if self._validation_type != "NONE" and self.get_expectations():
            self.validate(df, commit_time=now)

    def _read_df(self, online: bool = False, as_of=None, wallclock_time=None) -> pd.DataFrame:
        if online:
            if not self.online_enabled:
                raise FeatureStoreException(f"feature group {self.name} is not online enabled")
            return self._fs._online.read(self)
        limit = _commit_time(as_of if as_of is not None else wallclock_time)
        frames = []
        for c in self._commits():
            if c["ts"] > limit:
                break
            d = pd.read_parquet(self._dir / c["file"])
            if c["op"] == "overwrite":
                frames = []
            frames.append(d)
        cols = [f.name for f in self._features]
        if not frames:
            return pd.DataFrame(columns=cols)
        df = pd.concat(frames, ignore_index=True)
        if self.time_travel_format == "HUDI" and self.primary_key:
            df = df.drop_duplicates(subset=self.primary_key, keep="last")
        for f in self._features:
            if f.name not in df.columns:
                df[f.name] = f.default_value
            elif f.default_value is not None:
                df[f.name] = df[f.name].fillna(f.default_value)
        return df[cols].reset_index(drop=True)

    # ------------------------------------------------------------- reads
    def read(self, wallclock_time=None, online: bool = False, dataframe_type: str = "default", read_options=None):
        return self._read_df(online=online, as_of=wallclock_time)

    def show(self, n: int = 20, online: bool = False) -> None:
        _spark_show(self.read(online=online), n)

    def read_changes(self, start_wallclock_time, end_wallclock_time, read_options=None) -> pd.DataFrame:
        t0, t1 = _commit_time(start_wallclock_time), _commit_time(end_wallclock_time)
        frames = [pd.read_parquet(self._dir / c["file"]) for c in self._commits() if t0 < c["ts"] <= t1]
        if not frames:
            return pd.DataFrame(columns=[f.name for f in self._features])
        df = pd.concat(frames, ignore_index=True)
        if self.primary_key:
            df = df.drop_duplicates(subset=self.primary_key, keep="last")
        return df.reset_index(drop=True)

    def commit_details(self, wallclock_time=None, limit: int | None = None) -> dict:
        limit_t = _commit_time(wallclock_time)
        out = {}
        for c in reversed(self._commits()):
            if c["ts"] > limit_t:
                continue
            out[c["ts"]] = {"committedOn": c["committedOn"], "rowsUpdated": c["rowsUpdated"],
                            "rowsInserted": c["rowsInserted"], "rowsDeleted": c["rowsDeleted"]}
            if limit and len(out) >= limit:
                break
        return out

    # ------------------------------------------------------------- schema ops
    def append_features(self, features) -> "FeatureGroup":
        feats = features if isinstance(features, list) else [features]
        for f in feats:
            f._fg = self
            self._features.append(f)
        self._persist()
        return self

    def update_description(self, description: str):
        self.description = description
        self._persist()
        return self

    def delete(self) -> None:
        import shutil

        shutil.rmtree(self._dir, ignore_errors=True)
        self._fs._delete_meta(self.ENTITY_TYPE, self._table)
        if self.online_enabled:
            self._fs._online.drop(self)

    # ------------------------------------------------------------- statistics
    def compute_statistics(self, wallclock_time=None):
        st = ST.compute(self._read_df(as_of=wallclock_time), self.statistics_config)
        (self._dir).mkdir(parents=True, exist_ok=True)
        (self._dir / "statistics.json").write_text(json.dumps(st, default=float))
        return st

    def get_statistics(self, commit_time=None):
        p = self._dir / "statistics.json"
        return json.loads(p.read_text()) if p.exists() else self.compute_statistics()

    @property
    def statistics(self):
        return self.get_statistics()

    # ------------------------------------------------------------- validation
    @property
    def validation_type(self):
        return self._validation_type

    @validation_type.setter
    def validation_type(self, v):
        self._validation_type = str(v).upper()
        self._persist()

    def get_expectations(self) -> list:
        return [self._fs.get_expectation(n) for n in self._meta.get("expectations", [])]

    def get_expectation(self, name):
        if name not in self._meta.get("expectations", []):
            raise FeatureStoreException(f"expectation {name} not attached")
        return self._fs.get_expectation(name)

    def attach_expectation(self, expectation):
        n = expectation if isinstance(expectation, str) else expectation.name
        if n not in self._meta.setdefault("expectations", []):
            self._meta["expectations"].append(n)
        self._persist()

    def detach_expectation(self, expectation):
        n = expectation if isinstance(expectation, str) else expectation.name
        if n in self._meta.get("expectations", []):
            self._meta["expectations"].remove(n)
        self._persist()

    def validate(self, dataframe=None, _persist: bool = True, commit_time=None) -> R.FeatureGroupValidation:
        df = self.read() if dataframe is None else _to_pandas(dataframe)
        v = R.validate(df, self.get_expectations(), self._fs._next_id("validation"), commit_time)
        if _persist:
            vals = self._meta.setdefault("validations", [])
            vals.append(v.to_dict())
            self._persist()
        return v

    def get_validations(self, validation_time=None, commit_time=None) -> list:
        out = []
        for d in self._meta.get("validations", []):
            if validation_time is not None and d["validationTime"] != _commit_time(validation_time) and \
                    d["validationTime"] != validation_time:
                continue
            if commit_time is not None and d.get("commitTime") != _commit_time(commit_time) and \
                    d.get("commitTime") != commit_time:
                continue
            exps = [R.ExpectationResult(R.Expectation.from_dict(e["expectation"]),
                                        [R.ValidationResult(r["status"], r["message"], r["value"], r["feature"],
                                                            R.Rule.from_dict(r["rule"])) for r in e["results"]])
                    for e in d["expectationResults"]]
            out.append(R.FeatureGroupValidation(d["validationId"], d["validationTime"], exps, d.get("commitTime")))
        return out

    def __repr__(self):
        return f"FeatureGroup({self.name!r}, {self.version}, {self.description!r}, {self.primary_key})"


class OnDemandFeatureGroup(FeatureGroupBase):
    """External feature group: a SQL query over a storage connector, run at read time."""

    ENTITY_TYPE = "featuregroups"

    def __init__(self, fs, name, version, query, storage_connector, description="", features=None,
                 statistics_config=None, meta=None):
        self._fs = fs
        self.name, self.version, self.query, self.description = name, int(version), query, description or ""
        self.storage_connector = storage_connector
        self.primary_key, self.partition_key = [], []
        self.online_enabled, self.time_travel_format = False, None
        self.statistics_config = ST.StatisticsConfig.parse(statistics_config)
        self._meta = meta or {"tags": {}}
        self._features = features or []
        self.id = self._meta.get("id")

    @property
    def _table(self):
        return f"{self.name}_{self.version}"

    def _persist(self):
        self._meta.update({"name": self.name, "version": self.version, "description": self.description,
                           "query": self.query, "storage_connector": self.storage_connector.name,
                           "features": [f.to_dict() for f in self._features], "type": "on_demand"})
        self._fs._write_meta(self.ENTITY_TYPE, self._table, self._meta)

    def save(self):
        df = self.storage_connector.read(self.query)
        self._features = [Feature(c, _hsfs_type(df[c].dtype), fg=self) for c in df.columns]
        if self.id is None:
            self.id = self._fs._next_id()
            self._meta["id"] = self.id
        self._persist()
        return self

    def _read_df(self, online=False, as_of=None):
        return self.storage_connector.read(self.query)

    def read(self, dataframe_type="default"):
        return self._read_df()

    def show(self, n=20):
        _spark_show(self.read(), n)
