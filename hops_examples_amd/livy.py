"""Livy-style interactive sessions + the sparkmagic cell magics.

The reference's notebooks talk to the cluster through a Livy server: sparkmagic starts a session
(``%%configure``, the session table of ``%%info``), ships each cell to it as a *statement*
(``%%spark``), runs SQL there (``%%sql -o df -q --maxrows N``), and moves data across the
notebook/cluster boundary (``-o``: a remote DataFrame becomes a local pandas one; ``%%send_to_spark``:
the other way); ``%%local`` cells run on the notebook host
(notebooks/ml/Plotting/matplotlib_sparkmagic.ipynb:81-176 (the ``%%help`` table), :301 (``%%sql -c sql
-o python_df --maxrows 10``), :318 (``%%spark -o df``); notebooks/spark/KafkaSparkPython.ipynb).

Here the "cluster" is this node, but the boundary is real:

* :class:`LivyServer` — the Livy REST API (``POST /sessions``, ``GET /sessions/{id}``,
  ``POST /sessions/{id}/statements``, ``GET /sessions/{id}/statements/{sid}``,
  ``DELETE /sessions/{id}``, ``GET /sessions/{id}/log``) on a ThreadingHTTPServer.  Each session is
  its own Python worker *process* (the remote driver): statements execute there, in order, in a
  persistent namespace with ``spark`` (a SparkSession stand-in over the Hive warehouse) bound, and
  their results come back as Livy statement outputs (``text/plain`` / ``application/json`` data,
  or ``error`` with ``ename`` / ``evalue`` / ``traceback``).
* :class:`SparkMagics` — the cell-magic front end: ``run_cell("%%sql -o df\\nSELECT ...")``
  parses the magic line like sparkmagic does and drives the server through its REST API.

Nothing here needs Spark, Livy or IPython installed.
"""
from __future__ import annotations

import argparse
import io
import json
import os
import shlex
import subprocess
import sys
import threading
import time
import traceback
import urllib.request
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

import pandas as pd

# --------------------------------------------------------------------------- remote side
_WORKER = r'''
import io, json, sys, traceback, contextlib
import pandas as pd
sys.path.insert(0, {root!r})
from hops_examples_amd.livy import SparkStandIn
ns = {{"spark": SparkStandIn(), "pd": pd}}
ns["sqlContext"] = ns["spark"]
out = sys.stdout
sys.stdout = sys.stderr  # statement prints are captured per statement; keep the pipe clean
for line in sys.stdin:
    req = json.loads(line)
    buf = io.StringIO()
    try:
        with contextlib.redirect_stdout(buf):
            kind, code = req["kind"], req["code"]
            data = {{}}
            if kind == "sql":
                df = ns["spark"].sql(code).toPandas()
                if req.get("maxrows") is not None and req["maxrows"] >= 0:
                    df = df.head(req["maxrows"])
                data["application/json"] = json.loads(df.to_json(orient="split", date_format="iso"))
            elif kind == "fetch":  # -o VAR: a remote DataFrame's rows to the notebook
                v = ns[code]
                df = v.toPandas() if hasattr(v, "toPandas") else pd.DataFrame(v)
                if req.get("maxrows") is not None and req["maxrows"] >= 0:
                    df = df.head(req["maxrows"])
                data["application/json"] = json.loads(df.to_json(orient="split", date_format="iso"))
            elif kind == "store":  # %%send_to_spark: a local pandas DataFrame / string into the session
                val = req["value"]
                ns[code] = (ns["spark"].createDataFrame(pd.read_json(io.StringIO(val), orient="split"))
                            if req.get("as") == "df" else val)
            else:
                tree = compile(code, "<statement>", "exec")
                exec(tree, ns)
        data["text/plain"] = buf.getvalue()
        res = {{"status": "ok", "data": data}}
    except BaseException as e:  # noqa: BLE001 - reported to the client like Livy does
        res = {{"status": "error", "ename": type(e).__name__, "evalue": str(e),
                "traceback": traceback.format_exception(type(e), e, e.__traceback__)}}
    out.write(json.dumps(res) + "\n")
    out.flush()
'''


class SparkDataFrame:
    """The slice of ``pyspark.sql.DataFrame`` the notebooks' remote cells use, over pandas."""

    def __init__(self, pdf: pd.DataFrame):
        self._pdf = pdf.reset_index(drop=True)

    def toPandas(self) -> pd.DataFrame:  # noqa: N802 (pyspark name)
        return self._pdf.copy()

    def count(self) -> int:
        return len(self._pdf)

    @property
    def columns(self) -> list:
        return list(self._pdf.columns)

    def select(self, *cols) -> "SparkDataFrame":
        return SparkDataFrame(self._pdf[list(cols)])

    def limit(self, n: int) -> "SparkDataFrame":
        return SparkDataFrame(self._pdf.head(n))

    def filter(self, expr: str) -> "SparkDataFrame":
        return SparkDataFrame(self._pdf.query(expr))

    where = filter

    def show(self, n: int = 20) -> None:
        print(self._pdf.head(n).to_string(index=False))

    def createOrReplaceTempView(self, name: str) -> None:  # noqa: N802
        from . import hive

        (hive._default or hive.setup_hive_connection()).register_temp_view(name, self._pdf)

    registerTempTable = createOrReplaceTempView


class _FormatReader:
    """``spark.read.format(fmt).options(**o).load([path])``: csv / parquet / json files, ``jdbc`` (url +
    dbtable or query over SQLite) and the Snowflake Spark connector ``net.snowflake.spark.snowflake``
    (``sf*`` options + dbtable or query; hsfs/snowflake/pyspark.ipynb:92-120)."""

    def __init__(self, fmt: str):
        self.fmt, self.opts = fmt.lower(), {}

    def option(self, key: str, value) -> "_FormatReader":
        self.opts[key] = value
        return self

    def options(self, **kw) -> "_FormatReader":
        self.opts.update(kw)
        return self

    def load(self, path: str | None = None) -> SparkDataFrame:
        o = self.opts
        if self.fmt in ("net.snowflake.spark.snowflake", "snowflake"):
            from . import snowflake

            q = o.get("query") or f"SELECT * FROM {o['dbtable']}"
            with snowflake.connect(url=o.get("sfURL"), user=o.get("sfUser"), password=o.get("sfPassword"),
                                   database=o.get("sfDatabase"), schema=o.get("sfSchema"),
                                   warehouse=o.get("sfWarehouse"), role=o.get("sfRole")) as ctx:
                return SparkDataFrame(ctx.cursor().execute(q).fetch_pandas_all())
        if self.fmt == "jdbc":
            import sqlite3

            db = o["url"]
            for pre in ("jdbc:sqlite:", "sqlite:///"):
                db = db[len(pre):] if db.startswith(pre) else db
            q = o.get("query") or f"SELECT * FROM {o['dbtable']}"
            with sqlite3.connect(db) as c:
                return SparkDataFrame(pd.read_sql_query(q, c))
        r = _Reader()
        if self.fmt == "csv":
            return r.csv(path, header=str(o.get("header", True)).lower() == "true")
        return getattr(r, self.fmt)(path)


class _Reader:
    def format(self, fmt: str) -> _FormatReader:
        return _FormatReader(fmt)

    def parquet(self, path: str) -> SparkDataFrame:
        from . import hdfs

        return SparkDataFrame(pd.read_parquet(str(hdfs._resolve(path))))

    def csv(self, path: str, header: bool = True, inferSchema: bool = True, sep: str = ",") -> SparkDataFrame:  # noqa: N803
        from . import hdfs

        return SparkDataFrame(pd.read_csv(str(hdfs._resolve(path)), header=0 if header else None, sep=sep))

    def json(self, path: str) -> SparkDataFrame:
        from . import hdfs

        return SparkDataFrame(pd.read_json(str(hdfs._resolve(path)), lines=True))


class SparkStandIn:
    """``spark`` inside a session: SQL runs on the Hive-style warehouse (hive.py)."""

    read = _Reader()

    def sql(self, query: str) -> SparkDataFrame:
        from . import hive

        df = hive.sql(query)
        return SparkDataFrame(df if df is not None else pd.DataFrame())

    def createDataFrame(self, data, schema=None) -> SparkDataFrame:  # noqa: N802
        pdf = data if isinstance(data, pd.DataFrame) else pd.DataFrame(data, columns=schema)
        return SparkDataFrame(pdf)

    def range(self, n: int) -> SparkDataFrame:
        return SparkDataFrame(pd.DataFrame({"id": range(n)}))


class _Session:
    def __init__(self, sid: int, kind: str, conf: dict):
        self.id, self.kind, self.conf = sid, kind, conf
        self.state = "starting"
        self.log: list[str] = []
        self.statements: list[dict] = []
        self._lock = threading.Lock()
        self._q: list[int] = []
        self._cv = threading.Condition()
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        env = dict(os.environ)
        env.update({f"SPARK_CONF_{k}": str(v) for k, v in conf.items()})
        self._p = subprocess.Popen([sys.executable, "-u", "-c", _WORKER.format(root=root)], stdin=subprocess.PIPE,
                                   stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env)
        threading.Thread(target=self._drain_stderr, daemon=True).start()
        self._runner = threading.Thread(target=self._run, daemon=True)
        self._runner.start()
        self.state = "idle"

    def _drain_stderr(self):
        for line in self._p.stderr:
            self.log.append(line.rstrip("\n"))

    def submit(self, code: str, kind: str, **extra) -> dict:
        with self._lock:
            st = {"id": len(self.statements), "code": code, "kind": kind, "state": "waiting", "output": None,
                  "progress": 0.0, "started": 0, "completed": 0, "_extra": extra}
            self.statements.append(st)
        with self._cv:
            self._q.append(st["id"])
            self._cv.notify()
        return st

    def _run(self):
        n = 0
        while True:
            with self._cv:
                while not self._q and self.state != "dead":
                    self._cv.wait()
                if self.state == "dead":
                    return
                sid = self._q.pop(0)
            st = self.statements[sid]
            st["state"], st["started"] = "running", int(time.time() * 1000)
            self.state = "busy"
            req = {"code": st["code"], "kind": st["kind"], **st["_extra"]}
            try:
                self._p.stdin.write(json.dumps(req) + "\n")
                self._p.stdin.flush()
                line = self._p.stdout.readline()
                res = json.loads(line) if line else {"status": "error", "ename": "SessionDied",
                                                     "evalue": "the session process exited", "traceback": []}
            except (BrokenPipeError, ValueError) as e:
                res = {"status": "error", "ename": type(e).__name__, "evalue": str(e), "traceback": []}
            res["execution_count"] = n
            n += 1
            st["output"] = res
            st["state"], st["progress"], st["completed"] = "available", 1.0, int(time.time() * 1000)
            if self._p.poll() is not None:
                self.state = "dead"
                return
            self.state = "idle"

    def kill(self):
        self.state = "dead"
        with self._cv:
            self._cv.notify_all()
        if self._p.poll() is None:
            self._p.stdin.close()
            try:
                self._p.wait(timeout=5)
            except subprocess.TimeoutExpired:
                self._p.kill()

    def public(self) -> dict:
        return {"id": self.id, "kind": self.kind, "state": self.state, "appId": f"application_local_{self.id:04d}",
                "appInfo": {"driverLogUrl": None, "sparkUiUrl": None}, "conf": self.conf, "log": self.log[-20:]}


def _stmt_public(st: dict) -> dict:
    return {k: v for k, v in st.items() if not k.startswith("_")}


class LivyServer:
    """Livy's session REST API on ``127.0.0.1:port`` (0: any free port)."""

    def __init__(self, port: int = 0):
        self.sessions: dict[int, _Session] = {}
        self._next = 0
        self._lock = threading.Lock()
        server = self

        class H(BaseHTTPRequestHandler):
            def log_message(self, *a):  # quiet
                pass

            def _send(self, code: int, obj):
                body = json.dumps(obj).encode()
                self.send_response(code)
                self.send_header("Content-Type", "application/json")
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)

            def _body(self) -> dict:
                n = int(self.headers.get("Content-Length") or 0)
                return json.loads(self.rfile.read(n) or b"{}") if n else {}

            def _parts(self):
                return [p for p in self.path.split("?")[0].split("/") if p]

            def do_GET(self):  # noqa: N802
                p = self._parts()
                if p == ["sessions"]:
                    return self._send(200, {"from": 0, "total": len(server.sessions),
                                            "sessions": [s.public() for s in server.sessions.values()]})
                s = server._get(p)
                if s is None:
                    return self._send(404, {"msg": "session not found"})
                if len(p) == 2:
                    return self._send(200, s.public())
                if len(p) == 3 and p[2] == "state":
                    return self._send(200, {"id": s.id, "state": s.state})
                if len(p) == 3 and p[2] == "log":
                    return self._send(200, {"id": s.id, "from": 0, "total": len(s.log), "log": s.log})
                if len(p) == 3 and p[2] == "statements":
                    return self._send(200, {"statements": [_stmt_public(t) for t in s.statements]})
                if len(p) == 4 and p[2] == "statements":
                    i = int(p[3])
                    if 0 <= i < len(s.statements):
                        return self._send(200, _stmt_public(s.statements[i]))
                return self._send(404, {"msg": "not found"})

            def do_POST(self):  # noqa: N802
                p, body = self._parts(), self._body()
                if p == ["sessions"]:
                    kind = body.get("kind", "pyspark")
                    if kind not in ("pyspark", "spark", "sql", "shared"):
                        return self._send(400, {"msg": f"unsupported session kind {kind!r}"})
                    with server._lock:
                        sid = server._next
                        server._next += 1
                        server.sessions[sid] = _Session(sid, kind, body.get("conf", {}) or {})
                    return self._send(201, server.sessions[sid].public())
                s = server._get(p)
                if s is None or s.state == "dead":
                    return self._send(404, {"msg": "session not found"})
                if len(p) == 3 and p[2] == "statements":
                    extra = {k: body[k] for k in ("maxrows", "value", "as") if k in body}
                    st = s.submit(body.get("code", ""), body.get("kind", s.kind if s.kind != "shared" else "pyspark"),
                                  **extra)
                    return self._send(201, _stmt_public(st))
                return self._send(404, {"msg": "not found"})

            def do_DELETE(self):  # noqa: N802
                p = self._parts()
                s = server._get(p)
                if s is None:
                    return self._send(404, {"msg": "session not found"})
                s.kill()
                server.sessions.pop(s.id, None)
                return self._send(200, {"msg": "deleted"})

        self.httpd = ThreadingHTTPServer(("127.0.0.1", port), H)
        self.port = self.httpd.server_address[1]
        self.url = f"http://127.0.0.1:{self.port}"
        threading.Thread(target=self.httpd.serve_forever, daemon=True).start()

    def _get(self, p) -> _Session | None:
        if len(p) >= 2 and p[0] == "sessions" and p[1].isdigit():
            return self.sessions.get(int(p[1]))
        return None

    def close(self) -> None:
        for s in list(self.sessions.values()):
            s.kill()
        self.sessions.clear()
        self.httpd.shutdown()
        self.httpd.server_close()


# --------------------------------------------------------------------------- client side
class LivyError(RuntimeError):
    pass


def _http(method: str, url: str, body: dict | None = None) -> dict:
    data = None if body is None else json.dumps(body).encode()
    req = urllib.request.Request(url, data=data, method=method, headers={"Content-Type": "application/json"})
    with urllib.request.urlopen(req, timeout=60) as r:
        return json.loads(r.read() or b"{}")


def _frame(js: dict) -> pd.DataFrame:
    return pd.DataFrame(js["data"], columns=js["columns"])


_HELP = pd.DataFrame([
    ("info", "%%info", "Outputs session information for the current Livy endpoint."),
    ("cleanup", "%%cleanup -f", "Deletes all sessions for the current Livy endpoint."),
    ("delete", "%%delete -f -s 0", "Deletes a session by number for the current Livy endpoint."),
    ("logs", "%%logs", "Outputs the current session's Livy logs."),
    ("configure", '%%configure -f\n{"executorMemory": "1000M", "executorCores": 4}',
     "Configure the session creation parameters (-f drops and recreates the current session)."),
    ("sql", "%%sql -o tables -q\nSHOW TABLES",
     "Executes a SQL query against the session. -o VAR binds the result as a local pandas DataFrame, "
     "-q suppresses the output, -n/--maxrows limits the rows returned."),
    ("spark", "%%spark -o df\ndf = spark.read.parquet('...')",
     "Executes code against the session. -o VAR: the remote DataFrame VAR as a local pandas DataFrame."),
    ("local", "%%local\na = 1", "Runs the cell on the notebook host (this process)."),
    ("send_to_spark", "%%send_to_spark -i df -t df -n remote_df",
     "Sends a local pandas DataFrame (-t df) or string (-t str) into the session as -n NAME."),
], columns=["Magic", "Example", "Explanation"])


class SparkMagics:
    """sparkmagic's cell magics over a Livy endpoint.  ``run_cell`` takes a whole cell (magic line +
    body) and returns what the cell displays; ``-o`` results are bound in ``local_ns``."""

    def __init__(self, url: str | None = None, local_ns: dict | None = None, kind: str = "pyspark"):
        self._own = None
        if url is None:
            self._own = LivyServer()
            url = self._own.url
        self.url = url.rstrip("/")
        self.local_ns = {} if local_ns is None else local_ns
        self.kind = kind
        self.conf: dict = {}
        self.session_id: int | None = None

    # ---- session lifecycle
    def _ensure(self) -> int:
        if self.session_id is None:
            s = _http("POST", f"{self.url}/sessions", {"kind": self.kind, "conf": self.conf})
            self.session_id = s["id"]
            deadline = time.time() + 60
            while _http("GET", f"{self.url}/sessions/{self.session_id}/state")["state"] == "starting":
                if time.time() > deadline:
                    raise LivyError("session did not start")
                time.sleep(0.05)
        return self.session_id

    def _statement(self, code: str, kind: str, **extra) -> dict:
        sid = self._ensure()
        st = _http("POST", f"{self.url}/sessions/{sid}/statements", {"code": code, "kind": kind, **extra})
        while st["state"] in ("waiting", "running"):
            time.sleep(0.01)
            st = _http("GET", f"{self.url}/sessions/{sid}/statements/{st['id']}")
        out = st["output"]
        if out["status"] != "ok":
            raise LivyError(f"{out.get('ename')}: {out.get('evalue')}\n" + "".join(out.get("traceback", [])))
        return out["data"]

    def close(self) -> None:
        if self.session_id is not None:
            try:
                _http("DELETE", f"{self.url}/sessions/{self.session_id}")
            except Exception:  # noqa: BLE001 - already gone
                pass
            self.session_id = None
        if self._own is not None:
            self._own.close()
            self._own = None

    # ---- cells
    def run_cell(self, cell: str):
        line, _, body = cell.partition("\n")
        line = line.strip()
        if not line.startswith("%%"):
            return self._spark([], cell)
        argv = shlex.split(line[2:])
        name, args = argv[0], argv[1:]
        fn = {"sql": self._sql, "spark": self._spark, "local": self._local, "help": self._help,
              "info": self._info, "configure": self._configure, "cleanup": self._cleanup, "delete": self._delete,
              "logs": self._logs, "send_to_spark": self._send}.get(name)
        if fn is None:
            raise LivyError(f"unknown magic %%{name}")
        return fn(args, body)

    def _sql(self, args, body):
        ap = argparse.ArgumentParser(prog="%%sql", add_help=False)
        ap.add_argument("-o", "--output")
        ap.add_argument("-q", "--quiet", action="store_true")
        ap.add_argument("-n", "--maxrows", type=int, default=2500)
        ap.add_argument("-c", "--context", default="sql")
        ap.add_argument("-m", "--samplemethod", default="take")
        ap.add_argument("-r", "--samplefraction", type=float)
        a = ap.parse_args(args)
        df = _frame(self._statement(body.strip(), "sql", maxrows=a.maxrows)["application/json"])
        if a.output:
            self.local_ns[a.output] = df
        return None if a.quiet else df

    def _spark(self, args, body):
        ap = argparse.ArgumentParser(prog="%%spark", add_help=False)
        ap.add_argument("-o", "--output")
        ap.add_argument("-n", "--maxrows", type=int, default=2500)
        ap.add_argument("-m", "--samplemethod", default="take")
        ap.add_argument("-r", "--samplefraction", type=float)
        a = ap.parse_args(args)
        text = self._statement(body, "pyspark").get("text/plain", "") if body.strip() else ""
        if a.output:
            self.local_ns[a.output] = _frame(self._statement(a.output, "fetch", maxrows=a.maxrows)["application/json"])
        return text

    def _local(self, args, body):
        buf = io.StringIO()
        import contextlib

        with contextlib.redirect_stdout(buf):
            exec(compile(body, "<local>", "exec"), self.local_ns)
        return buf.getvalue()

    def _help(self, args, body):
        return _HELP.copy()

    def _info(self, args, body):
        ses = _http("GET", f"{self.url}/sessions")["sessions"]
        return pd.DataFrame([{"ID": s["id"], "YARN Application ID": s["appId"], "Kind": s["kind"],
                              "State": s["state"], "Current session?": s["id"] == self.session_id} for s in ses],
                            columns=["ID", "YARN Application ID", "Kind", "State", "Current session?"])

    def _configure(self, args, body):
        force = "-f" in args
        conf = json.loads(body) if body.strip() else {}
        if self.session_id is not None and not force:
            raise LivyError("a session is already running: use %%configure -f to drop and recreate it")
        if self.session_id is not None:
            _http("DELETE", f"{self.url}/sessions/{self.session_id}")
            self.session_id = None
        self.conf = conf
        self._ensure()
        return self._info([], "")

    def _cleanup(self, args, body):
        if "-f" not in args:
            raise LivyError("%%cleanup needs -f")
        for s in _http("GET", f"{self.url}/sessions")["sessions"]:
            _http("DELETE", f"{self.url}/sessions/{s['id']}")
        self.session_id = None

    def _delete(self, args, body):
        ap = argparse.ArgumentParser(prog="%%delete", add_help=False)
        ap.add_argument("-f", action="store_true")
        ap.add_argument("-s", type=int, required=True)
        a = ap.parse_args(args)
        if not a.f:
            raise LivyError("%%delete needs -f")
        if a.s == self.session_id:
            raise LivyError("cannot delete this kernel's own session")
        _http("DELETE", f"{self.url}/sessions/{a.s}")

    def _logs(self, args, body):
        sid = self._ensure()
        return "\n".join(_http("GET", f"{self.url}/sessions/{sid}/log")["log"])

    def _send(self, args, body):
        ap = argparse.ArgumentParser(prog="%%send_to_spark", add_help=False)
        ap.add_argument("-i", "--input", required=True)
        ap.add_argument("-t", "--type", default="str", choices=["str", "df"])
        ap.add_argument("-n", "--name")
        a = ap.parse_args(args)
        v = self.local_ns[a.input]
        if a.type == "df":
            payload = v.to_json(orient="split", date_format="iso")
        else:
            payload = str(v)
        self._statement(a.name or a.input, "store", value=payload, **({"as": "df"} if a.type == "df" else {}))


def main(argv=None) -> int:
    """``python -m hops_examples_amd.livy --port 8998``: a standalone Livy endpoint."""
    ap = argparse.ArgumentParser()
    ap.add_argument("--port", type=int, default=8998)
    a = ap.parse_args(argv)
    srv = LivyServer(a.port)
    print(json.dumps({"livy": srv.url}), flush=True)
    try:
        while True:
            time.sleep(3600)
    except KeyboardInterrupt:
        srv.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
