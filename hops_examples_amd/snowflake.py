"""Snowflake warehouse stand-in: the ``snowflake.connector`` DB-API surface the reference's Snowflake
notebooks use, over a local SQLite database per (account, database).

Reference: notebooks/featurestore/hsfs/snowflake/python.ipynb:51-488 and getting-started.ipynb:113-150
(``connector.snowflake_connector_options()`` -> ``snowflake.connector.connect(**opts)`` ->
``ctx.cursor().execute(sql).fetchall()`` -> pandas), pyspark.ipynb:92-192 and scala.ipynb:84-207
(``spark_options()`` + ``"query"`` -> ``spark.read.format("net.snowflake.spark.snowflake")``, an
on-demand feature group over the connector).  There is no Snowflake account here: the warehouse is
``<project>/Resources/snowflake/<account>/<database>.db`` (``HOPSX_SNOWFLAKE_ROOT`` overrides the
root), identifiers are case-insensitive as in Snowflake's unquoted form, and credentials are taken
from the connector options or ``SNOWFLAKE_PASSWORD`` — never from source.
"""
from __future__ import annotations

import os
import sqlite3
from pathlib import Path

import pandas as pd

paramstyle = "pyformat"


class Error(Exception):
    pass


class ProgrammingError(Error):
    pass


def _db_path(account: str | None, database: str | None) -> Path:
    root = os.environ.get("HOPSX_SNOWFLAKE_ROOT")
    if root:
        base = Path(root)
    else:
        from . import hdfs

        base = Path(hdfs.abs_path("Resources/snowflake"))
    p = base / (account or "local") / f"{(database or 'default').lower()}.db"
    p.parent.mkdir(parents=True, exist_ok=True)
    return p


class SnowflakeCursor:
    def __init__(self, conn: "SnowflakeConnection"):
        self._c = conn._db.cursor()
        self.description = None
        self.rowcount = -1
        self.sfqid = None

    def execute(self, command: str, params=None) -> "SnowflakeCursor":
        try:
            self._c.execute(command, params or ())
        except sqlite3.Error as e:
            raise ProgrammingError(f"SQL compilation error: {e}") from e
        self.description = self._c.description
        self.rowcount = self._c.rowcount
        return self

    def fetchone(self):
        return self._c.fetchone()

    def fetchmany(self, size: int = 1):
        return self._c.fetchmany(size)

    def fetchall(self):
        return self._c.fetchall()

    def fetch_pandas_all(self) -> pd.DataFrame:
        cols = [d[0].upper() for d in (self.description or [])]
        return pd.DataFrame(self._c.fetchall(), columns=cols)

    def __iter__(self):
        return iter(self._c)

    def close(self) -> None:
        self._c.close()


class SnowflakeConnection:
    def __init__(self, account=None, user=None, password=None, database=None, schema=None, warehouse=None,
                 role=None, url=None, **kw):
        if not user:
            raise ProgrammingError("user is required")
        password = password or os.environ.get("SNOWFLAKE_PASSWORD") or kw.get("token") or kw.get("authenticator")
        if not password:
            raise ProgrammingError("password (or token / authenticator) is required: pass it in the connector "
                                   "options or set SNOWFLAKE_PASSWORD")
        if url and not account:  # <account>.snowflakecomputing.com
            account = url.split("//")[-1].split(".")[0]
        self.account, self.user, self.database, self.schema = account, user, database, schema
        self.warehouse, self.role = warehouse, role
        self.path = _db_path(account, database)
        self._db = sqlite3.connect(str(self.path))

    def cursor(self) -> SnowflakeCursor:
        return SnowflakeCursor(self)

    def execute_string(self, sql: str) -> list[SnowflakeCursor]:
        return [self.cursor().execute(s) for s in sql.split(";") if s.strip()]

    def commit(self) -> None:
        self._db.commit()

    def close(self) -> None:
        self._db.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.commit()
        self.close()


def connect(**kw) -> SnowflakeConnection:
    """``snowflake.connector.connect(**connector.snowflake_connector_options())``."""
    return SnowflakeConnection(**kw)


def write_pandas(conn: SnowflakeConnection, df: pd.DataFrame, table_name: str, overwrite: bool = False,
                 quote_identifiers: bool = False, **kw):
    """``snowflake.connector.pandas_tools.write_pandas``: (success, nchunks, nrows, output)."""
    out = df if quote_identifiers else df.rename(columns=str.upper)
    out.to_sql(table_name.upper(), conn._db, index=False, if_exists="replace" if overwrite else "append")
    conn.commit()
    return True, 1, len(df), None
