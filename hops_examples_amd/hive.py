"""A HiveQL-subset warehouse for notebooks that use ``hops.hive`` / PySpark+Hive
(notebooks/hive/PyHive.ipynb:44-757, notebooks/spark/PySparkWithHive.ipynb:88-757,
hive/src/main/java/io/hops/examples/hive/HiveJDBCClient.java:49-158).

Supported statements (everything else is passed to the SQL engine unchanged):
  CREATE [EXTERNAL] TABLE t (cols) [PARTITIONED BY (cols)] [ROW FORMAT DELIMITED
      FIELDS TERMINATED BY ','] [STORED AS ORC|PARQUET|TEXTFILE] [LOCATION 'path']
  INSERT OVERWRITE|INTO TABLE t [PARTITION (p[=v], ...)] SELECT ...   (dynamic partitions:
      overwrite replaces only the partitions present in the result, as Hive does)
  SHOW TABLES | SHOW DATABASES | DESCRIBE t | SET k=v | DROP TABLE [IF EXISTS] t
  CREATE DATABASE / USE db
Query execution runs on SQLite; managed ORC/Parquet tables are also materialised as
partitioned files under ``Hive/warehouse/<db>.db/<table>/<p>=<v>/`` (pyarrow), external
CSV tables are loaded from their LOCATION on first use.
"""
from __future__ import annotations

import json
import re
import sqlite3
from pathlib import Path

import pandas as pd

from . import hdfs

_TYPES = {"string": "TEXT", "varchar": "TEXT", "char": "TEXT", "int": "INTEGER", "bigint": "INTEGER",
          "smallint": "INTEGER", "tinyint": "INTEGER", "boolean": "INTEGER", "float": "REAL", "double": "REAL",
          "decimal": "REAL", "date": "TEXT", "timestamp": "TEXT"}
_PD = {"TEXT": "string", "INTEGER": "Int64", "REAL": "float64"}


def _cols(spec: str) -> list[tuple[str, str]]:
    out = []
    for part in re.split(r",(?![^()]*\))", spec):
        part = part.strip()
        if not part:
            continue
        name, typ = part.split(None, 1)
        base = typ.strip().split("(")[0].lower()
        out.append((name.strip("`"), _TYPES.get(base, "TEXT")))
    return out


def _path_of(loc: str) -> Path:
    loc = loc.split("://", 1)[-1]
    m = re.match(r"/Projects/[^/]+/(.*)", loc)
    return Path(hdfs._resolve(m.group(1) if m else loc))


class HiveConnection:
    def __init__(self, database: str = "default"):
        self.root = Path(hdfs.project_path()) / "Hive"
        self.root.mkdir(parents=True, exist_ok=True)
        self.db = database
        self._meta_path = self.root / "metastore.json"
        self.meta = json.loads(self._meta_path.read_text()) if self._meta_path.exists() else {"databases": ["default"],
                                                                                                "tables": {}}
        self.conf: dict[str, str] = {}
        self._conns: dict[str, sqlite3.Connection] = {}

    # ------------------------------------------------------------------ plumbing
    def _conn(self, db=None) -> sqlite3.Connection:
        db = db or self.db
        if db not in self._conns:
            self._conns[db] = sqlite3.connect(str(self.root / f"{db}.sqlite"))
        return self._conns[db]

    def _save(self):
        self._meta_path.write_text(json.dumps(self.meta, indent=2))

    def _key(self, t):
        return f"{self.db}.{t.lower()}"

    def _table(self, t):
        return self.meta["tables"].get(self._key(t))

    def _load_external(self, t: str, m: dict):
        cols = m["columns"]
        files = [m["location"]] if Path(m["location"]).is_file() else sorted(
            p for p in Path(m["location"]).rglob("*") if p.is_file() and not p.name.startswith((".", "_")))
        frames = [pd.read_csv(f, names=[c for c, _ in cols], sep=m.get("delimiter", ","), header=None,
                              skipinitialspace=True) for f in files]
        df = pd.concat(frames, ignore_index=True) if frames else pd.DataFrame(columns=[c for c, _ in cols])
        for c, ty in cols:  # rows that do not parse as the declared type become NULL (as in Hive)
            if ty in ("INTEGER", "REAL"):
                df[c] = pd.to_numeric(df[c], errors="coerce")
        con = self._conn()
        con.execute(f'DROP TABLE IF EXISTS "{t}"')
        con.execute(f'CREATE TABLE "{t}" ({", ".join(f"{c} {ty}" for c, ty in cols)})')
        con.executemany(f'INSERT INTO "{t}" VALUES ({",".join("?" * len(cols))})',
                        [tuple(None if pd.isna(v) else v for v in r) for r in df.itertuples(index=False)])
        con.commit()
        m["loaded"] = True

    def _materialise(self, t: str, m: dict):
        fmt = m.get("format", "TEXTFILE")
        if fmt not in ("ORC", "PARQUET"):
            return
        import pyarrow as pa

        df = pd.read_sql_query(f'SELECT * FROM "{t}"', self._conn())
        base = self.root / "warehouse" / f"{self.db}.db" / t
        import shutil

        shutil.rmtree(base, ignore_errors=True)
        parts = [c for c, _ in m.get("partitions", [])]
        groups = df.groupby(parts, dropna=False) if parts else [((), df)]
        for key, g in groups:
            key = key if isinstance(key, tuple) else (key,)
            d = base.joinpath(*[f"{p}={v}" for p, v in zip(parts, key)])
            d.mkdir(parents=True, exist_ok=True)
            tbl = pa.Table.from_pandas(g.drop(columns=parts), preserve_index=False)
            if fmt == "ORC":
                import pyarrow.orc as orc

                orc.write_table(tbl, str(d / "part-00000.orc"))
            else:
                import pyarrow.parquet as pq

                pq.write_table(tbl, str(d / "part-00000.parquet"))

    # ------------------------------------------------------------------ statements
    def execute(self, sql: str):
        """Run one or more ';'-separated statements; returns the last result as a DataFrame
        (or None for DDL)."""
        res = None
        for stmt in [s.strip() for s in re.split(r";\s*(?=(?:[^']*'[^']*')*[^']*$)", sql) if s.strip()]:
            res = self._one(stmt)
        return res

    def _one(self, s: str):
        u = " ".join(s.split()).upper()
        if u.startswith("SET "):
            k, _, v = s[4:].partition("=")
            self.conf[k.strip()] = v.strip()
            return None
        if u.startswith("CREATE DATABASE"):
            name = re.findall(r"(\w+)\s*$", s)[0]
            if name not in self.meta["databases"]:
                self.meta["databases"].append(name)
                self._save()
            return None
        if u.startswith("USE "):
            self.db = s.split()[1]
            return None
        if u in ("SHOW DATABASES", "SHOW SCHEMAS"):
            return pd.DataFrame({"database_name": self.meta["databases"]})
        if u == "SHOW TABLES":
            names = sorted(k.split(".", 1)[1] for k in self.meta["tables"] if k.startswith(self.db + "."))
            return pd.DataFrame({"tab_name": names})
        if u.startswith("DESCRIBE ") or u.startswith("DESC "):
            t = s.split()[-1]
            m = self._table(t)
            cols = m["columns"] + m.get("partitions", [])
            return pd.DataFrame({"col_name": [c for c, _ in cols], "data_type": [ty for _, ty in cols]})
        if u.startswith("DROP TABLE"):
            t = s.split()[-1]
            self._conn().execute(f'DROP TABLE IF EXISTS "{t}"')
            self.meta["tables"].pop(self._key(t), None)
            self._save()
            return None
        if u.startswith("CREATE TABLE") or u.startswith("CREATE EXTERNAL TABLE"):
            return self._create(s, "EXTERNAL" in u.split("(")[0])
        if u.startswith("INSERT "):
            return self._insert(s)
        return self._select(s)

    def _create(self, s: str, external: bool):
        m = re.match(r"\s*CREATE\s+(?:EXTERNAL\s+)?TABLE\s+(?:IF\s+NOT\s+EXISTS\s+)?([`\w.]+)\s*\((.*?)\)\s*(.*)$", s,
                     re.I | re.S)
        if not m:
            raise ValueError(f"cannot parse CREATE TABLE: {s[:200]}")
        t, spec, rest = m.group(1).strip("`"), m.group(2), m.group(3)
        cols = _cols(spec)
        pm = re.search(r"PARTITIONED\s+BY\s*\((.*?)\)", rest, re.I | re.S)
        parts = _cols(pm.group(1)) if pm else []
        fm = re.search(r"STORED\s+AS\s+(\w+)", rest, re.I)
        dm = re.search(r"FIELDS\s+TERMINATED\s+BY\s+'(.*?)'", rest, re.I)
        lm = re.search(r"LOCATION\s+'(.*?)'", rest, re.I)
        meta = {"columns": cols, "partitions": parts, "format": (fm.group(1).upper() if fm else "TEXTFILE"),
                "external": external, "delimiter": dm.group(1) if dm else ",",
                "location": str(_path_of(lm.group(1))) if lm else None}
        con = self._conn()
        con.execute(f'CREATE TABLE IF NOT EXISTS "{t}" ({", ".join(f"{c} {ty}" for c, ty in cols + parts)})')
        con.commit()
        self.meta["tables"][self._key(t)] = meta
        self._save()
        if external and meta["location"]:
            self._load_external(t, meta)
        return None

    def _insert(self, s: str):
        m = re.match(r"\s*INSERT\s+(OVERWRITE|INTO)\s+(?:TABLE\s+)?([`\w.]+)\s*(?:PARTITION\s*\((.*?)\))?\s*(SELECT.*)$",
                     s, re.I | re.S)
        if not m:
            return self._select(s)
        mode, t, pspec, select = m.group(1).upper(), m.group(2).strip("`"), m.group(3), m.group(4)
        meta = self._table(t)
        self._ensure_loaded(select)
        df = pd.read_sql_query(select, self._conn())
        names = [c for c, _ in meta["columns"]] + [c for c, _ in meta.get("partitions", [])]
        static = {}
        if pspec:
            for p in pspec.split(","):
                if "=" in p:
                    k, v = p.split("=", 1)
                    static[k.strip()] = v.strip().strip("'\"")
        for k, v in static.items():
            df[k] = v
        df.columns = names[:len(df.columns)] if len(df.columns) == len(names) else df.columns
        con = self._conn()
        if mode == "OVERWRITE":
            parts = [c for c, _ in meta.get("partitions", [])]
            if parts:
                for key in df[parts].drop_duplicates().itertuples(index=False):
                    cond = " AND ".join(f'"{p}" = ?' for p in parts)
                    con.execute(f'DELETE FROM "{t}" WHERE {cond}', tuple(key))
            else:
                con.execute(f'DELETE FROM "{t}"')
        con.executemany(f'INSERT INTO "{t}" ({",".join(names)}) VALUES ({",".join("?" * len(names))})',
                        [tuple(None if pd.isna(v) else (v.item() if hasattr(v, "item") else v) for v in r)
                         for r in df[names].itertuples(index=False)])
        con.commit()
        self._materialise(t, meta)
        return None

    def _ensure_loaded(self, sql: str):
        for k, m in self.meta["tables"].items():
            db, t = k.split(".", 1)
            if db == self.db and m.get("external") and not m.get("loaded") and re.search(rf"\b{t}\b", sql, re.I):
                self._load_external(t, m)

    def _select(self, s: str):
        self._ensure_loaded(s)
        s = re.sub(r"\bLIMIT\s+(\d+)\s*$", r"LIMIT \1", s.strip(), flags=re.I)
        cur = self._conn().execute(s)
        if cur.description is None:
            self._conn().commit()
            return None
        return pd.DataFrame(cur.fetchall(), columns=[d[0] for d in cur.description])

    # DB-API flavour for %sql / pandas.read_sql users
    def cursor(self):
        return _Cursor(self)

    def register_temp_view(self, name: str, df: pd.DataFrame) -> None:
        """A session-scoped view over a DataFrame (Spark ``createOrReplaceTempView``): queryable by
        name, never written to the metastore or the warehouse."""
        df.to_sql(name, self._conn(), if_exists="replace", index=False)

    def close(self):
        for c in self._conns.values():
            c.close()
        self._conns.clear()


class _Cursor:
    def __init__(self, hc: HiveConnection):
        self.hc, self._rows, self.description = hc, [], None

    def execute(self, sql, params=None):
        df = self.hc.execute(sql)
        if df is None:
            self._rows, self.description = [], None
        else:
            self._rows = [tuple(r) for r in df.itertuples(index=False)]
            self.description = [(c, None, None, None, None, None, None) for c in df.columns]
        return self

    def fetchall(self):
        r, self._rows = self._rows, []
        return r

    def fetchone(self):
        return self._rows.pop(0) if self._rows else None


_default: HiveConnection | None = None


def setup_hive_connection(database: str = "default") -> HiveConnection:
    global _default
    _default = HiveConnection(database)
    return _default


def sql(query: str) -> pd.DataFrame | None:
    return (_default or setup_hive_connection()).execute(query)
