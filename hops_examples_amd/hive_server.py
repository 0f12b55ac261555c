"""A HiveServer2-style SQL endpoint and a JDBC-flavoured client (HiveJDBCClient).

The reference's Java client (hive/src/main/java/io/hops/examples/hive/HiveJDBCClient.java:49-158)
reads ``hive_credentials.properties`` (hive_url, dbname, trust/key store paths and passwords),
opens ``<hive_url>/<db>;auth=noSasl;ssl=true;twoWay=true;sslTrustStore=..;trustStorePassword=..;
sslKeyStore=..;keyStorePassword=..`` through ``DriverManager.getConnection``, and runs ``SET``,
``CREATE EXTERNAL TABLE .. LOCATION``, ``CREATE TABLE .. STORED AS ORC``, ``INSERT OVERWRITE`` and a
``GROUP BY`` query whose ``ResultSet`` it walks with ``next()`` / ``getString(i)``.

Here:

* :class:`HiveServer2` — a threaded TCP server (newline-delimited JSON messages: open / execute /
  fetch / close) over the Hive-style warehouse (``hive.py``), optionally TLS with client
  certificates required (``two_way``: the reference's ``twoWay=true`` mutual TLS);
* :func:`connect` — parses the ``jdbc:hive2://`` URL (session variables after ``;``) and returns a
  :class:`Connection` with the JDBC surface (``createStatement``, ``Statement.execute`` /
  ``executeQuery`` / ``executeUpdate``, ``ResultSet.next`` / ``getString`` / ``getInt`` /
  ``getDouble`` / ``getMetaData``) and a DB-API cursor (``cursor().execute().fetchall()``);
* :func:`read_hive_credentials` / :func:`jdbc_url` — the properties file and the URL the
  reference builds from it.  Stores are PEM files here (``sslTrustStore``: CA bundle,
  ``sslKeyStore``: client certificate + key; the store passwords unlock an encrypted key).
"""
from __future__ import annotations

import json
import socket
import socketserver
import ssl
import threading
from urllib.parse import unquote

# ---------------------------------------------------------------------------------------- server


class _Handler(socketserver.StreamRequestHandler):
    def handle(self):
        from . import hive

        srv: HiveServer2 = self.server.owner  # type: ignore[attr-defined]
        conn = None
        rows, pos = [], 0
        for raw in self.rfile:
            try:
                req = json.loads(raw)
            except ValueError:
                self._send({"ok": False, "error": "malformed request", "sqlstate": "08S01"})
                return
            op = req.get("op")
            try:
                if op == "open":
                    db = req.get("db") or "default"
                    conn = hive.HiveConnection(db)
                    if db not in conn.meta["databases"]:
                        raise ValueError(f"Database '{db}' does not exist")
                    srv.sessions += 1
                    self._send({"ok": True, "session": srv.sessions, "server": "hopsx-hiveserver2"})
                elif op == "execute":
                    if conn is None:
                        raise ValueError("no open session")
                    df = conn.execute(req["sql"])
                    if df is None:
                        rows, pos = [], 0
                        self._send({"ok": True, "columns": None, "update_count": -1})
                    else:
                        rows = [[None if _isnull(v) else _py(v) for v in r] for r in df.itertuples(index=False)]
                        pos = 0
                        self._send({"ok": True, "columns": [str(c) for c in df.columns],
                                    "types": [_jdbc_type(t) for t in df.dtypes], "row_count": len(rows)})
                elif op == "fetch":
                    n = int(req.get("n", 1000))
                    chunk, pos = rows[pos:pos + n], min(len(rows), pos + n)
                    self._send({"ok": True, "rows": chunk, "done": pos >= len(rows)})
                elif op == "close":
                    self._send({"ok": True})
                    return
                else:
                    raise ValueError(f"unknown operation {op!r}")
            except Exception as e:  # noqa: BLE001 - reported to the client as an SQLException
                self._send({"ok": False, "error": f"{type(e).__name__}: {e}", "sqlstate": "42000"})

    def _send(self, obj):
        self.wfile.write((json.dumps(obj) + "\n").encode())
        self.wfile.flush()


def _isnull(v) -> bool:
    try:
        return v != v  # NaN
    except Exception:  # noqa: BLE001
        return v is None


def _py(v):
    if hasattr(v, "item"):
        return v.item()
    return v


def _jdbc_type(dt) -> str:
    k = getattr(dt, "kind", "O")
    return {"i": "BIGINT", "u": "BIGINT", "f": "DOUBLE", "b": "BOOLEAN"}.get(k, "STRING")


class _TCP(socketserver.ThreadingTCPServer):
    daemon_threads = True
    allow_reuse_address = True


class HiveServer2:
    """``host:port`` SQL endpoint over the project's Hive warehouse.  ``certfile`` / ``keyfile``:
    the server identity (TLS on); ``cafile`` + ``two_way``: client certificates signed by that CA
    are required (mutual TLS)."""

    def __init__(self, port: int = 0, certfile: str | None = None, keyfile: str | None = None,
                 cafile: str | None = None, two_way: bool = False):
        self.sessions = 0
        self._tcp = _TCP(("127.0.0.1", port), _Handler)
        self._tcp.owner = self  # type: ignore[attr-defined]
        self.ssl = certfile is not None
        if self.ssl:
            ctx = ssl.SSLContext(ssl.PROTOCOL_TLS_SERVER)
            ctx.load_cert_chain(certfile, keyfile)
            if two_way:
                if not cafile:
                    raise ValueError("two-way TLS needs the CA that signs the client certificates")
                ctx.verify_mode = ssl.CERT_REQUIRED
                ctx.load_verify_locations(cafile)
            self._tcp.socket = ctx.wrap_socket(self._tcp.socket, server_side=True)
        self.port = self._tcp.server_address[1]
        self.url = f"jdbc:hive2://127.0.0.1:{self.port}"
        self._thread = threading.Thread(target=self._tcp.serve_forever, daemon=True)
        self._thread.start()

    def close(self) -> None:
        self._tcp.shutdown()
        self._tcp.server_close()


# ---------------------------------------------------------------------------------------- client


class SQLException(RuntimeError):
    def __init__(self, msg: str, sqlstate: str = "HY000"):
        super().__init__(msg)
        self.sqlstate = sqlstate


def parse_url(url: str) -> dict:
    """``jdbc:hive2://host:port/db;k=v;...`` -> {host, port, db, vars}."""
    if not url.startswith("jdbc:hive2://"):
        raise SQLException(f"not a HiveServer2 JDBC URL: {url}", "08001")
    rest = url[len("jdbc:hive2://"):]
    main, _, sess = rest.partition(";")
    hostport, _, db = main.partition("/")
    host, _, port = hostport.partition(":")
    kv = {}
    for part in sess.split(";"):
        if part:
            k, _, v = part.partition("=")
            kv[k.strip()] = unquote(v.strip())
    return {"host": host or "127.0.0.1", "port": int(port or 10000), "db": db or "default", "vars": kv}


def read_hive_credentials(path: str) -> dict:
    """A Java ``.properties`` file (``key=value`` / ``key: value``, ``#`` / ``!`` comments)."""
    props = {}
    with open(path) as f:
        for line in f:
            s = line.strip()
            if not s or s[0] in "#!":
                continue
            sep = min((i for i in (s.find("="), s.find(":")) if i >= 0), default=-1)
            if sep < 0:
                props[s] = ""
            else:
                props[s[:sep].strip()] = s[sep + 1:].strip()
    return props


def jdbc_url(props: dict) -> str:
    """The URL HiveJDBCClient.getHiveJDBCConnection builds from the credentials properties."""
    return (f"{props['hive_url']}/{props['dbname']};auth=noSasl;ssl=true;twoWay=true"
            f";sslTrustStore={props['truststore_path']};trustStorePassword={props.get('truststore_pw', '')}"
            f";sslKeyStore={props['keystore_path']};keyStorePassword={props.get('keystore_pw', '')}")


class ResultSetMetaData:
    def __init__(self, cols, types):
        self._c, self._t = cols, types

    def getColumnCount(self) -> int:  # noqa: N802 (JDBC names)
        return len(self._c)

    def getColumnName(self, i: int) -> str:  # noqa: N802
        return self._c[i - 1]

    def getColumnTypeName(self, i: int) -> str:  # noqa: N802
        return self._t[i - 1]


class ResultSet:
    def __init__(self, conn: "Connection", cols, types):
        self._conn, self._cols, self._types = conn, cols, types
        self._buf, self._done, self._row = [], False, None

    def next(self) -> bool:
        if not self._buf and not self._done:
            r = self._conn._call({"op": "fetch", "n": 1000})
            self._buf, self._done = list(r["rows"]), r["done"]
        if not self._buf:
            self._row = None
            return False
        self._row = self._buf.pop(0)
        return True

    def _get(self, i):
        if self._row is None:
            raise SQLException("no current row (call next() first)", "24000")
        idx = self._cols.index(i) if isinstance(i, str) else i - 1  # JDBC columns are 1-based
        return self._row[idx]

    def getString(self, i):  # noqa: N802
        v = self._get(i)
        return None if v is None else str(v)

    def getInt(self, i) -> int:  # noqa: N802
        v = self._get(i)
        return 0 if v is None else int(v)

    def getDouble(self, i) -> float:  # noqa: N802
        v = self._get(i)
        return 0.0 if v is None else float(v)

    getFloat = getDouble
    getLong = getInt

    def getObject(self, i):  # noqa: N802
        return self._get(i)

    def getMetaData(self) -> ResultSetMetaData:  # noqa: N802
        return ResultSetMetaData(self._cols, self._types)

    def __iter__(self):
        while self.next():
            yield tuple(self._row)

    def close(self) -> None:
        self._buf, self._done = [], True

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


class Statement:
    def __init__(self, conn: "Connection"):
        self._conn = conn
        self._rs: ResultSet | None = None

    def execute(self, sql: str) -> bool:
        """True when the statement produced a result set (JDBC semantics)."""
        r = self._conn._call({"op": "execute", "sql": sql})
        self._rs = ResultSet(self._conn, r["columns"], r.get("types", [])) if r["columns"] is not None else None
        return self._rs is not None

    def executeQuery(self, sql: str) -> ResultSet:  # noqa: N802
        if not self.execute(sql):
            raise SQLException("the statement did not return a result set", "07005")
        return self._rs

    def executeUpdate(self, sql: str) -> int:  # noqa: N802
        self.execute(sql)
        return 0

    def getResultSet(self) -> ResultSet | None:  # noqa: N802
        return self._rs

    def close(self) -> None:
        self._rs = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


class Cursor:
    """DB-API 2.0 view of the same connection (PyHive-style)."""

    def __init__(self, conn: "Connection"):
        self._st = Statement(conn)
        self.description = None

    def execute(self, sql: str, params=None) -> "Cursor":
        if params:
            raise SQLException("parameter binding is not supported", "0A000")
        has = self._st.execute(sql)
        rs = self._st.getResultSet()
        self.description = [(c, t, None, None, None, None, True) for c, t in zip(rs._cols, rs._types)] if has else None
        return self

    def fetchall(self) -> list:
        rs = self._st.getResultSet()
        return list(rs) if rs is not None else []

    def fetchone(self):
        rs = self._st.getResultSet()
        return tuple(rs._row) if rs is not None and rs.next() else None

    def fetchmany(self, size: int = 1) -> list:
        out = []
        for _ in range(size):
            r = self.fetchone()
            if r is None:
                break
            out.append(r)
        return out

    def close(self) -> None:
        self._st.close()


class Connection:
    def __init__(self, url: str, timeout: float = 60.0):
        u = parse_url(url)
        v = u["vars"]
        raw = socket.create_connection((u["host"], u["port"]), timeout=timeout)
        if v.get("ssl", "false").lower() == "true":
            ctx = ssl.create_default_context(ssl.Purpose.SERVER_AUTH, cafile=v.get("sslTrustStore") or None)
            ctx.check_hostname = False  # local endpoint; the chain is still verified against the store
            if v.get("twoWay", "false").lower() == "true":
                if not v.get("sslKeyStore"):
                    raise SQLException("twoWay=true needs sslKeyStore (client certificate + key)", "08001")
                ctx.load_cert_chain(v["sslKeyStore"], password=v.get("keyStorePassword") or None)
            raw = ctx.wrap_socket(raw, server_hostname=u["host"])
        self._sock = raw
        self._r = raw.makefile("rb")
        self._lock = threading.Lock()
        self.closed = False
        r = self._call({"op": "open", "db": u["db"], "auth": v.get("auth", "noSasl")})
        self.session = r["session"]

    def _call(self, req: dict) -> dict:
        with self._lock:
            try:
                self._sock.sendall((json.dumps(req) + "\n").encode())
                line = self._r.readline()
            except OSError as e:
                raise SQLException(f"connection lost: {e}", "08S01") from e
        if not line:
            raise SQLException("connection closed by the server", "08S01")
        r = json.loads(line)
        if not r.get("ok"):
            raise SQLException(r.get("error", "error"), r.get("sqlstate", "HY000"))
        return r

    def createStatement(self) -> Statement:  # noqa: N802
        return Statement(self)

    def cursor(self) -> Cursor:
        return Cursor(self)

    def close(self) -> None:
        if self.closed:
            return
        try:
            self._call({"op": "close"})
        except SQLException:
            pass
        self._r.close()
        self._sock.close()
        self.closed = True

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def connect(url: str, timeout: float = 60.0) -> Connection:
    """``DriverManager.getConnection(url)``."""
    return Connection(url, timeout)
