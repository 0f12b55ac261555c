"""Livy sessions + sparkmagic cell magics (hops_examples_amd/livy.py): the
matplotlib_sparkmagic.ipynb flow (:176 %%help, :301 %%sql -c sql -o python_df --maxrows 10,
:318 %%spark -o df, %%local plotting cells) against a real REST endpoint and session process."""
import json
import urllib.request

import pandas as pd
import pytest

from hops_examples_amd import livy


def _req(method, url, body=None):
    data = None if body is None else json.dumps(body).encode()
    r = urllib.request.Request(url, data=data, method=method, headers={"Content-Type": "application/json"})
    with urllib.request.urlopen(r, timeout=60) as f:
        return f.status, json.loads(f.read())


def test_sparkmagic_cells_roundtrip(project_root):
    ns = {}
    m = livy.SparkMagics(local_ns=ns)
    try:
        help_df = m.run_cell("%%help")
        assert {"sql", "spark", "local", "configure", "info"} <= set(help_df["Magic"])
        # remote: build a table in the session's warehouse, print from the driver
        out = m.run_cell("%%spark\n"
                         "spark.sql(\"CREATE TABLE sales (city STRING, amount DOUBLE)\")\n"
                         "spark.sql(\"INSERT INTO TABLE sales SELECT 'a', 1.5 UNION ALL SELECT 'b', 2.0 "
                         "UNION ALL SELECT 'a', 4.0\")\n"
                         "print('rows', spark.sql('SELECT * FROM sales').count())")
        assert "rows 3" in out
        # %%sql -c sql -o python_df --maxrows 10 (matplotlib_sparkmagic.ipynb:301)
        df = m.run_cell("%%sql -c sql -o python_df --maxrows 10\n"
                        "SELECT city, SUM(amount) AS total FROM sales GROUP BY city ORDER BY city")
        assert list(ns["python_df"]["city"]) == ["a", "b"]
        assert ns["python_df"]["total"].tolist() == [5.5, 2.0]
        assert df.equals(ns["python_df"])
        assert m.run_cell("%%sql -q -o t2\nSELECT * FROM sales") is None and len(ns["t2"]) == 3
        # %%spark -o df: a remote DataFrame bound locally as pandas (:318)
        m.run_cell("%%spark -o df\ndf = spark.sql('SELECT * FROM sales WHERE amount > 1.6')")
        assert isinstance(ns["df"], pd.DataFrame) and len(ns["df"]) == 2
        # %%local runs on the notebook host, against the bound frames
        assert m.run_cell("%%local\nprint(round(df['amount'].sum(), 2))").strip() == "6.0"
        # %%send_to_spark: local pandas -> session DataFrame, then query it there
        ns["local_df"] = pd.DataFrame({"x": [1, 2, 3]})
        m.run_cell("%%send_to_spark -i local_df -t df -n remote_df")
        assert "6" in m.run_cell("%%spark\nprint(int(remote_df.toPandas()['x'].sum()))")
        m.run_cell("%%spark\nremote_df.createOrReplaceTempView('xs')")
        assert m.run_cell("%%sql\nSELECT SUM(x) AS s FROM xs")["s"].tolist() == [6]
        # state persists across statements; errors come back as Livy errors with the remote traceback
        m.run_cell("%%spark\nk = 41")
        assert m.run_cell("%%spark\nprint(k + 1)").strip() == "42"
        with pytest.raises(livy.LivyError, match="ZeroDivisionError"):
            m.run_cell("%%spark\n1 / 0")
        info = m.run_cell("%%info")
        assert info["Current session?"].tolist() == [True] and info["State"].iloc[0] == "idle"
        # %%configure -f drops and recreates the session (new namespace)
        m.run_cell('%%configure -f\n{"executorMemory": "1000M", "executorCores": 4}')
        with pytest.raises(livy.LivyError, match="NameError"):
            m.run_cell("%%spark\nprint(k)")
        with pytest.raises(livy.LivyError):
            m.run_cell('%%configure\n{"executorCores": 2}')  # without -f while a session runs
    finally:
        m.close()


def test_livy_rest_api(project_root):
    srv = livy.LivyServer()
    try:
        code, s = _req("POST", f"{srv.url}/sessions", {"kind": "pyspark"})
        assert code == 201 and s["state"] in ("starting", "idle")
        sid = s["id"]
        code, st = _req("POST", f"{srv.url}/sessions/{sid}/statements", {"code": "print(6 * 7)"})
        assert code == 201 and st["state"] in ("waiting", "running", "available")
        for _ in range(600):
            _, st = _req("GET", f"{srv.url}/sessions/{sid}/statements/{st['id']}")
            if st["state"] == "available":
                break
            import time

            time.sleep(0.05)
        assert st["output"]["status"] == "ok" and st["output"]["data"]["text/plain"].strip() == "42"
        _, lst = _req("GET", f"{srv.url}/sessions")
        assert lst["total"] == 1 and lst["sessions"][0]["kind"] == "pyspark"
        code, _ = _req("DELETE", f"{srv.url}/sessions/{sid}")
        assert code == 200
        with pytest.raises(urllib.error.HTTPError):
            _req("GET", f"{srv.url}/sessions/{sid}")
        with pytest.raises(urllib.error.HTTPError):
            _req("POST", f"{srv.url}/sessions", {"kind": "sparkr"})
    finally:
        srv.close()
