"""Connection, FeatureStore, online store (SQLite), storage connectors and tag schemas."""
from __future__ import annotations

import json
import os
import sqlite3
import threading
from pathlib import Path

import numpy as np
import pandas as pd

from .builders import (CamelCaseAPI, ExpectationBuilder, FeatureGroupBuilder, OnDemandFeatureGroupBuilder,
                       TrainingDatasetBuilder)
from .. import config, hdfs
from . import rules as R
from .core import (Feature, FeatureGroup, FeatureStoreException, OnDemandFeatureGroup, Query, _hsfs_type,
                   _to_pandas, _warn_version)
from .training_dataset import TrainingDataset


# ====================================================================== online store
class OnlineStore:
    """Key-value online feature store (the MySQL-NDB role) on SQLite; point lookups by
    primary key through prepared statements, as ``get_serving_vector`` does."""

    def __init__(self, path: Path):
        self.path = path
        self._lock = threading.Lock()

    def _conn(self):
        c = sqlite3.connect(self.path, check_same_thread=False)
        return c

    @staticmethod
    def _tname(fg):
        return f"{fg.name}_{fg.version}"

    def upsert(self, fg, df: pd.DataFrame):
        with self._lock, self._conn() as c:
            t = self._tname(fg)
            cols = list(df.columns)
            pk = fg.primary_key or cols[:1]
            c.execute(f'CREATE TABLE IF NOT EXISTS "{t}" (' + ", ".join(f'"{x}"' for x in cols) +
                      ", PRIMARY KEY (" + ", ".join(f'"{k}"' for k in pk) + "))")
            rows = [tuple(None if (isinstance(v, float) and np.isnan(v)) else (v.item() if hasattr(v, "item") else v)
                          for v in r) for r in df.itertuples(index=False)]
            c.executemany(f'INSERT OR REPLACE INTO "{t}" (' + ", ".join(f'"{x}"' for x in cols) + ") VALUES (" +
                          ", ".join("?" * len(cols)) + ")", rows)

    def read(self, fg) -> pd.DataFrame:
        with self._lock, self._conn() as c:
            try:
                return pd.read_sql_query(f'SELECT * FROM "{self._tname(fg)}"', c)
            except Exception:
                return pd.DataFrame(columns=[f.name for f in fg.features])

    def drop(self, fg):
        with self._lock, self._conn() as c:
            c.execute(f'DROP TABLE IF EXISTS "{self._tname(fg)}"')

    def prepare(self, query: Query, exclude: set) -> dict:
        stmts, keys = [], []
        fgs = [(query._left_fg, query._left_features)] + [(j.query._left_fg, [f for f in j.query._left_features
                                                                             if f.name not in set(j.on)])
                                                           for j in query._joins]
        for fg, feats in fgs:
            if not fg.online_enabled:
                raise FeatureStoreException(f"feature group {fg.name} is not online enabled")
            cols = [f.name for f in feats if f.name not in exclude]
            pk = fg.primary_key
            for k in pk:
                if k not in keys:
                    keys.append(k)
            sql = ('SELECT ' + ", ".join(f'"{c}"' for c in cols) + f' FROM "{self._tname(fg)}" WHERE ' +
                   " AND ".join(f'"{k}" = ?' for k in pk))
            stmts.append((sql, pk, cols))
        return {"stmts": stmts, "keys": keys}

    def vector(self, prepared: dict, entry: dict) -> list:
        out = []
        with self._lock, self._conn() as c:
            for sql, pk, cols in prepared["stmts"]:
                missing = [k for k in pk if k not in entry]
                if missing:
                    raise FeatureStoreException(f"serving key(s) {missing} missing from entry")
                row = c.execute(sql, [entry[k] for k in pk]).fetchone()
                out.extend(list(row) if row is not None else [None] * len(cols))
        return out


# ================================================================ storage connectors
class StorageConnector:
    """Storage connectors (S3 / HopsFS / JDBC / Redshift / Snowflake).  Cloud and
    JDBC endpoints map to local equivalents: S3 buckets/HopsFS paths to project
    directories, JDBC/Redshift/Snowflake to SQLite database files."""

    def __init__(self, name, connector_type="HOPSFS", path=None, bucket=None, connection_string=None,
                 options=None, **kw):
        self.name, self.connector_type = name, connector_type.upper()
        self.bucket = bucket
        self.path = path or (hdfs.abs_path(f"Resources/{bucket}") if bucket else None)
        self.connection_string = connection_string
        self.options = dict(options or {})
        self.__dict__.update(kw)

    def _sf(self, key: str):
        if key == "password":  # credentials never live in connector metadata written by examples
            return self.options.get("password") or os.environ.get("SNOWFLAKE_PASSWORD")
        return self.options.get(key, getattr(self, key, None))

    def spark_options(self) -> dict:
        """Options for ``spark.read.format(...)``: the Snowflake Spark connector's ``sf*`` keys for a
        SNOWFLAKE connector (pyspark.ipynb:92-120), JDBC url/dbtable otherwise."""
        if self.connector_type == "SNOWFLAKE":
            o = {"sfURL": self._sf("url"), "sfUser": self._sf("user"), "sfPassword": self._sf("password"),
                 "sfDatabase": self._sf("database"), "sfSchema": self._sf("schema"),
                 "sfWarehouse": self._sf("warehouse"), "sfRole": self._sf("role"), "dbtable": self._sf("table")}
            return {k: v for k, v in o.items() if v is not None}
        o = {"url": self.connection_string or f"jdbc:sqlite:{self.path}", "dbtable": self.options.get("table")}
        o.update(self.options)
        return {k: v for k, v in o.items() if v is not None}

    def snowflake_connector_options(self) -> dict:
        """kwargs of ``snowflake.connector.connect`` (python.ipynb:51-75)."""
        o = {"account": self._sf("account") or (self._sf("url") or "").split("//")[-1].split(".")[0] or None,
             "user": self._sf("user"), "password": self._sf("password"), "database": self._sf("database"),
             "schema": self._sf("schema"), "warehouse": self._sf("warehouse"), "role": self._sf("role")}
        return {k: v for k, v in o.items() if v is not None}

    def read(self, query: str | None = None, data_format: str | None = None, path: str | None = None):
        if self.connector_type == "SNOWFLAKE":
            from .. import snowflake

            q = query or f"SELECT * FROM {self._sf('table')}"
            with snowflake.connect(**self.snowflake_connector_options()) as ctx:
                df = ctx.cursor().execute(q).fetch_pandas_all()
            return df.rename(columns=str.lower)  # feature names are lower-case in the feature store
        if self.connector_type in ("JDBC", "REDSHIFT", "SQLITE"):
            db = self.connection_string or self.path
            for pre in ("jdbc:sqlite:", "sqlite:///"):
                if db and db.startswith(pre):
                    db = db[len(pre):]
            with sqlite3.connect(db) as c:
                return pd.read_sql_query(query, c)
        p = Path(path or self.path)
        fmt = (data_format or p.suffix.lstrip(".") or "parquet").lower()
        if fmt == "csv":
            return pd.read_csv(p)
        return pd.read_parquet(p)

    def __repr__(self):
        return f"StorageConnector({self.name!r}, {self.connector_type!r})"


# ================================================================== tag schemas
class TagRegistry:
    """Project tag schemas (JSON-schema subset: type / properties / required)."""

    def __init__(self, path: Path):
        self.path = path

    def _load(self):
        return json.loads(self.path.read_text()) if self.path.exists() else {}

    def create(self, name: str, schema: dict | None = None):
        d = self._load()
        d[name] = schema or {"type": "string"}
        self.path.write_text(json.dumps(d, indent=2))

    def check(self, name, value):
        d = self._load()
        if name not in d:  # undeclared tags are accepted as free-form values
            return
        _check_schema(d[name], value, name)


_TYPES = {"string": str, "integer": int, "number": (int, float), "boolean": bool, "object": dict, "array": list}


def _check_schema(schema, value, path):
    t = schema.get("type")
    if t and not isinstance(value, _TYPES.get(t, object)):
        raise FeatureStoreException(f"tag {path}: expected {t}, got {type(value).__name__}")
    if t == "object":
        for r in schema.get("required", []):
            if r not in value:
                raise FeatureStoreException(f"tag {path}: missing required property {r!r}")
        for k, sub in schema.get("properties", {}).items():
            if k in value:
                _check_schema(sub, value[k], f"{path}.{k}")
    if t == "array" and "items" in schema:
        for i, v in enumerate(value):
            _check_schema(schema["items"], v, f"{path}[{i}]")


# ===================================================================== FeatureStore
class FeatureStore(CamelCaseAPI):
    # ---- JVM builder API (featurestore/builders.py): fs.createFeatureGroup().name(..)...build()
    def createFeatureGroup(self):  # noqa: N802
        return FeatureGroupBuilder(self)

    def createOnDemandFeatureGroup(self):  # noqa: N802
        return OnDemandFeatureGroupBuilder(self)

    def createTrainingDataset(self):  # noqa: N802
        return TrainingDatasetBuilder(self)

    def createExpectation(self):  # noqa: N802
        return ExpectationBuilder(self)

    def getName(self):  # noqa: N802
        return self.name

    def getOnlineStorageConnector(self):  # noqa: N802
        return self.get_storage_connector(f"{self.name}_onlinefeaturestore")

    def __init__(self, name: str, project_root: Path):
        self.name = name
        self._root = project_root / "Featurestore" / name
        self._root.mkdir(parents=True, exist_ok=True)
        self._meta_root = self._root / "_meta"
        self._meta_root.mkdir(exist_ok=True)
        self._td_root = project_root / "Training_Datasets"
        self._online = OnlineStore(self._root / "online.sqlite")
        self._tags = TagRegistry(self._meta_root / "tag_schemas.json")
        self.id = abs(hash(name)) % 1000

    # ------------------------------------------------------------- metadata
    def _meta_path(self, kind, key) -> Path:
        d = self._meta_root / kind
        d.mkdir(exist_ok=True)
        return d / f"{key}.json"

    def _write_meta(self, kind, key, meta):
        self._meta_path(kind, key).write_text(json.dumps(meta, indent=2, default=str))

    def _read_meta(self, kind, key):
        p = self._meta_path(kind, key)
        return json.loads(p.read_text()) if p.exists() else None

    def _delete_meta(self, kind, key):
        p = self._meta_path(kind, key)
        if p.exists():
            p.unlink()

    def _next_id(self, kind="entity") -> int:
        p = self._meta_root / "ids.json"
        d = json.loads(p.read_text()) if p.exists() else {}
        d[kind] = d.get(kind, 0) + 1
        p.write_text(json.dumps(d))
        return d[kind]

    def _versions(self, kind, name):
        d = self._meta_root / kind
        if not d.exists():
            return []
        out = []
        for p in d.glob(f"{name}_*.json"):
            v = p.stem[len(name) + 1:]
            if v.isdigit():
                out.append(int(v))
        return sorted(out)

    # ------------------------------------------------------------- feature groups
    def create_feature_group(self, name: str, version: int | None = None, description: str = "",
                             online_enabled: bool = False, time_travel_format: str | None = None,
                             partition_key: list | None = None, primary_key: list | None = None,
                             hudi_precombine_key: str | None = None, features: list | None = None,
                             statistics_config=None, validation_type: str = "NONE", expectations: list | None = None,
                             event_time=None):
        if version is None:
            vs = self._versions("featuregroups", name)
            version = (vs[-1] + 1) if vs else 1
        return FeatureGroup(self, name, version, description, primary_key, partition_key, online_enabled,
                            time_travel_format, statistics_config, hudi_precombine_key, validation_type,
                            expectations, features)

    def get_or_create_feature_group(self, name, version, **kw):
        try:
            return self.get_feature_group(name, version)
        except FeatureStoreException:
            return self.create_feature_group(name, version, **kw)

    def _fg_from_meta(self, m):
        if m.get("type") == "on_demand":
            sc = self.get_storage_connector(m["storage_connector"])
            fg = OnDemandFeatureGroup(self, m["name"], m["version"], m["query"], sc, m.get("description", ""),
                                      meta=m)
            fg._features = [Feature(f["name"], f["type"], fg=fg) for f in m["features"]]
            return fg
        feats = [Feature(f["name"], f["type"], f.get("description", ""), f["primary"], f["partition"],
                         f.get("hudiPrecombineKey", False), f.get("defaultValue")) for f in m["features"]]
        fg = FeatureGroup(self, m["name"], m["version"], m.get("description", ""), m["primary_key"],
                          m["partition_key"], m["online_enabled"], m["time_travel_format"], m["statistics_config"],
                          m["hudi_precombine_key"], m.get("validation_type", "NONE"), None, feats, meta=m)
        return fg

    def get_feature_group(self, name: str, version: int | None = None):
        if version is None:
            _warn_version("feature group", name)
            version = 1
        m = self._read_meta("featuregroups", f"{name}_{version}")
        if m is None:
            raise FeatureStoreException(f"Feature group {name} version {version} does not exist")
        return self._fg_from_meta(m)

    def get_feature_groups(self, name: str) -> list:
        return [self.get_feature_group(name, v) for v in self._versions("featuregroups", name)]

    def create_on_demand_feature_group(self, name: str, storage_connector, query: str | None = None,
                                       version: int | None = None, description: str = "", features=None,
                                       statistics_config=None, data_format=None, path=None):
        if version is None:
            vs = self._versions("featuregroups", name)
            version = (vs[-1] + 1) if vs else 1
        return OnDemandFeatureGroup(self, name, version, query, storage_connector, description, features,
                                    statistics_config)

    def get_on_demand_feature_group(self, name, version=None):
        return self.get_feature_group(name, version)

    # ------------------------------------------------------------- training datasets
    def create_training_dataset(self, name: str, version: int | None = None, description: str = "",
                                data_format: str = "tfrecords", coalesce: bool = False, storage_connector=None,
                                splits: dict | None = None, location: str = "", seed: int | None = None,
                                statistics_config=None, label: list | None = None):
        if version is None:
            vs = self._versions("trainingdatasets", name)
            version = (vs[-1] + 1) if vs else 1
        return TrainingDataset(self, name, version, description, data_format, coalesce, storage_connector, splits,
                               location, seed, statistics_config, label)

    def get_training_dataset(self, name: str, version: int | None = None):
        if version is None:
            _warn_version("training dataset", name)
            version = 1
        m = self._read_meta("trainingdatasets", f"{name}_{version}")
        if m is None:
            raise FeatureStoreException(f"Training dataset {name} version {version} does not exist")
        sc = self.get_storage_connector(m["storage_connector"]) if m.get("storage_connector") else None
        return TrainingDataset(self, m["name"], m["version"], m.get("description", ""), m["data_format"],
                               m.get("coalesce", False), sc, m.get("splits"), m.get("location", ""), m.get("seed"),
                               m.get("statistics_config"), m.get("label"), meta=m)

    def _rebuild_query(self, td) -> Query:
        fgs = td._meta.get("query_fgs")
        if not fgs:
            raise FeatureStoreException("training dataset was not created from a query")
        q = self.get_feature_group(*fgs[-1]).select_all()
        for n, v in fgs[:-1]:
            q = q.join(self.get_feature_group(n, v).select_all())
        return q

    # ------------------------------------------------------------- connectors
    def create_storage_connector(self, name, connector_type="HOPSFS", **kw) -> StorageConnector:
        sc = StorageConnector(name, connector_type, **kw)
        self._write_meta("connectors", name, {"name": name, "connector_type": sc.connector_type,
                                              **{k: v for k, v in sc.__dict__.items()
                                                 if k not in ("name", "connector_type")}})
        return sc

    def get_storage_connector(self, name: str, connector_type: str | None = None) -> StorageConnector:
        m = self._read_meta("connectors", name)
        if m is None:
            if name.endswith("_Training_Datasets") or name == "default":
                return StorageConnector(name, "HOPSFS", path=str(self._td_root))
            if name.endswith("_onlinefeaturestore"):
                return StorageConnector(name, "JDBC", path=str(self._online.path))
            raise FeatureStoreException(f"storage connector {name} does not exist")
        m = dict(m)
        return StorageConnector(m.pop("name"), m.pop("connector_type"), **m)

    # ------------------------------------------------------------- SQL
    def _run_sql(self, sql: str, frames: dict) -> pd.DataFrame:
        c = sqlite3.connect(":memory:")
        try:
            c.execute(f"ATTACH DATABASE ':memory:' AS `{self.name}`")
            for t, df in frames.items():
                d = df.copy()
                for col in d.columns:
                    if str(d[col].dtype).startswith("datetime"):
                        d[col] = d[col].astype(str)
                cols = [str(x) for x in d.columns]
                c.execute(f'CREATE TABLE `{self.name}`.`{t}` (' + ", ".join(f'"{x}"' for x in cols) + ")")
                rows = [tuple(None if (isinstance(v, float) and np.isnan(v)) else
                              (v.item() if hasattr(v, "item") else v) for v in r) for r in d.itertuples(index=False)]
                if rows:
                    c.executemany(f'INSERT INTO `{self.name}`.`{t}` VALUES (' + ", ".join("?" * len(cols)) + ")",
                                  rows)
            return pd.read_sql_query(sql, c)
        finally:
            c.close()

    def sql(self, query: str, dataframe_type: str = "default", online: bool = False) -> pd.DataFrame:
        """Run SQL over the offline feature groups (tables ``<fg>_<version>``)."""
        import re

        tables = set(re.findall(r"`?([A-Za-z0-9_]+_\d+)`?", query))
        frames = {}
        for t in tables:
            m = self._read_meta("featuregroups", t)
            if m is not None:
                frames[t] = self._fg_from_meta(m)._read_df(online=online)
        q = re.sub(r"(?<![`.\w])([A-Za-z0-9_]+_\d+)(?![`\w])", lambda mm: f"`{self.name}`.`{mm.group(1)}`"
                   if mm.group(1) in frames else mm.group(1), query)
        return self._run_sql(q, frames)

    # ------------------------------------------------------------- expectations
    def _save_expectation(self, e: R.Expectation):
        e._store = self
        self._write_meta("expectations", e.name, e.to_dict())

    def create_expectation(self, name, description="", features=None, rules=None) -> R.Expectation:
        return R.Expectation(name, features or [], rules or [], description, store=self)

    def get_expectation(self, name) -> R.Expectation:
        m = self._read_meta("expectations", name)
        if m is None:
            raise FeatureStoreException(f"expectation {name} does not exist")
        return R.Expectation.from_dict(m, self)

    def get_expectations(self) -> list:
        d = self._meta_root / "expectations"
        return [self.get_expectation(p.stem) for p in sorted(d.glob("*.json"))] if d.exists() else []

    def delete_expectation(self, name):
        self._delete_meta("expectations", name)

    # ------------------------------------------------------------- tags
    def create_tag_schema(self, name, schema=None):
        self._tags.create(name, schema)

    def __repr__(self):
        return f"FeatureStore({self.name!r})"


# ======================================================================= Connection
class _ConnectionBuilder(CamelCaseAPI):
    """``HopsworksConnection.builder.host(..).project(..).build()`` (ComputeFeatures.scala:91)."""

    def __init__(self):
        self._kw = {}

    def __getattr__(self, name):
        if name.startswith("_"):
            raise AttributeError(name)
        key = {"hostname": "host", "apiKeyValue": "api_key_value", "apiKeyFile": "api_key_file"}.get(name, name)

        def setter(v):
            self._kw[key] = v
            return self

        return setter

    def build(self):
        kw = {k: v for k, v in self._kw.items() if k in ("host", "port", "project", "engine", "region_name",
                                                          "api_key_value", "api_key_file")}
        return connection(**kw)


class _BuilderDescriptor:
    def __get__(self, obj, cls):
        return _ConnectionBuilder()


class Connection(CamelCaseAPI):
    builder = _BuilderDescriptor()

    def __init__(self, host=None, port=443, project=None, engine=None, region_name=None,
                 secrets_store=None, hostname_verification=True, trust_store_path=None, cert_folder=None,
                 api_key_file=None, api_key_value=None):
        # credentials are never needed locally; never echo them
        self.host, self.port, self.engine = host, port, engine or "python"
        if project:
            config.set(project_name=project, project_root=str(config.get().project_root.parent / project)) \
                if project != config.get().project_name else None
        self._connected = True
        print("Connected. Call `.close()` to terminate connection gracefully.")

    def getFeatureStore(self, name: str | None = None) -> FeatureStore:  # noqa: N802
        return self.get_feature_store(name)

    def get_feature_store(self, name: str | None = None) -> FeatureStore:
        name = name or f"{config.get().project_name}_featurestore"
        return FeatureStore(name, Path(hdfs.project_path()))

    def get_rules(self) -> list:
        return list(R.RULES.values())

    def get_rule(self, name: str):
        return R.RULES[name.upper()]

    def close(self):
        self._connected = False
        print("Connection closed.")

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


def connection(host=None, port=443, project=None, engine=None, region_name=None, secrets_store=None,
               hostname_verification=True, trust_store_path=None, cert_folder=None, api_key_file=None,
               api_key_value=None) -> Connection:
    return Connection(host, port, project, engine, region_name, secrets_store, hostname_verification,
                      trust_store_path, cert_folder, api_key_file, api_key_value)


def connection_quiet() -> Connection:
    """A connection for library code (trial workers, loaders) that prints nothing."""
    c = Connection.__new__(Connection)
    c.host, c.port, c.engine, c._connected = None, 443, "python", True
    return c
