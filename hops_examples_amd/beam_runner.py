"""The job-manager process behind ``beam.create_runner`` / ``start_runner`` (a Flink-session-cluster
stand-in): a REST server that accepts uploaded programs and runs them in task slots.

Reference: jobs-client/flink/jobs_flink_client.py:45-121 — start a Flink cluster as a Hopsworks job,
poll up to 90 s for RUNNING, upload the job jar (``POST /jars/upload``), run it
(``POST /jars/<id>/run?entry-class=...&program-args=...``), parse REST errors.  There is no JVM /
Flink in this image: a "jar" is a Python program (a ``.py`` file, or a ``.zip`` whose
``entry-class`` names the module to run).  Started by ``jobs.start_job`` (state, logs and GPU
assignment come from the jobs service); the endpoint is published in ``runner.json`` in the
execution directory, which is what readiness means here.

REST surface (JSON; errors as ``{"errors": [msg]}`` with a 4xx code, Flink's shape):
  GET  /overview                       taskmanagers, slots-total, slots-available, jobs-running
  POST /jars/upload                    multipart form field ``jarfile`` (or raw body + X-Filename)
  GET  /jars                           uploaded programs
  POST /jars/<jar_id>/run?entry-class=&program-args=   -> {"jobid": id}  (409 when no slot is free)
  GET  /jobs                           {"jobs": [{"id", "status"}]}
  GET  /jobs/<id>                      {"jid", "state": RUNNING|FINISHED|FAILED|CANCELED, "exit-code"}
  PATCH /jobs/<id>                     cancel
"""
import argparse
import json
import os
import shlex
import signal
import subprocess
import sys
import threading
import time
import urllib.parse
import uuid
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from pathlib import Path


class Runner:
    def __init__(self, workdir: Path, slots: int, taskmanagers: int):
        self.dir = workdir
        (self.dir / "jars").mkdir(parents=True, exist_ok=True)
        self.slots = max(1, slots) * max(1, taskmanagers)
        self.taskmanagers = taskmanagers
        self.jobs: dict = {}
        self.lock = threading.Lock()

    def running(self) -> int:
        return sum(1 for j in self.jobs.values() if j["proc"].poll() is None)

    def job_state(self, j) -> dict:
        rc = j["proc"].poll()
        state = "RUNNING" if rc is None else ("CANCELED" if j.get("canceled") else ("FINISHED" if rc == 0 else "FAILED"))
        return {"jid": j["id"], "name": j["name"], "state": state, "exit-code": rc, "start-time": j["start"]}

    def run(self, jar_id: str, entry: str, args: str) -> str:
        jar = self.dir / "jars" / jar_id
        if not jar.exists():
            raise KeyError(f"jar {jar_id} not found")
        with self.lock:
            if self.running() >= self.slots:
                raise RuntimeError(f"no free task slot ({self.slots} total)")
            jid = uuid.uuid4().hex[:16]
            env = dict(os.environ)
            if jar.suffix == ".zip":
                env["PYTHONPATH"] = str(jar) + os.pathsep + env.get("PYTHONPATH", "")
                if not entry:
                    raise ValueError("a .zip program needs an entry-class (module to run)")
                cmd = [sys.executable, "-m", entry]
            else:
                cmd = [sys.executable, str(jar)]
            cmd += shlex.split(args or "")
            log = open(self.dir / f"job_{jid}.log", "wb")
            p = subprocess.Popen(cmd, stdout=log, stderr=subprocess.STDOUT, env=env, cwd=str(self.dir),
                                 start_new_session=True)
            self.jobs[jid] = {"id": jid, "name": jar_id, "proc": p, "start": time.time(), "log": log}
            return jid

    def cancel(self, jid: str) -> None:
        j = self.jobs[jid]
        if j["proc"].poll() is None:
            j["canceled"] = True
            try:
                os.killpg(j["proc"].pid, signal.SIGTERM)
            except ProcessLookupError:
                pass

    def shutdown(self) -> None:
        for jid in list(self.jobs):
            self.cancel(jid)


def _multipart_file(body: bytes, ctype: str):
    """(filename, bytes) of the first file part of a multipart/form-data body."""
    from email.parser import BytesParser
    from email.policy import HTTP

    msg = BytesParser(policy=HTTP).parsebytes(b"Content-Type: " + ctype.encode() + b"\r\n\r\n" + body)
    for part in msg.iter_parts():
        fn = part.get_filename()
        if fn:
            return os.path.basename(fn), part.get_payload(decode=True)
    raise ValueError("multipart body has no file part")


def make_handler(runner: Runner):
    class H(BaseHTTPRequestHandler):
        def log_message(self, *a):  # quiet: the job's stdout is the runner log
            pass

        def _send(self, code: int, obj) -> None:
            b = json.dumps(obj).encode()
            self.send_response(code)
            self.send_header("Content-Type", "application/json")
            self.send_header("Content-Length", str(len(b)))
            self.end_headers()
            self.wfile.write(b)

        def _err(self, code: int, msg: str) -> None:
            self._send(code, {"errors": [msg]})

        def do_GET(self):  # noqa: N802
            u = urllib.parse.urlparse(self.path)
            parts = [p for p in u.path.split("/") if p]
            if parts == ["overview"]:
                return self._send(200, {"taskmanagers": runner.taskmanagers, "slots-total": runner.slots,
                                        "slots-available": runner.slots - runner.running(),
                                        "jobs-running": runner.running()})
            if parts == ["jars"]:
                return self._send(200, {"files": [{"id": p.name} for p in sorted((runner.dir / "jars").iterdir())]})
            if parts == ["jobs"]:
                return self._send(200, {"jobs": [{"id": j["id"], "status": runner.job_state(j)["state"]}
                                                 for j in runner.jobs.values()]})
            if len(parts) == 2 and parts[0] == "jobs":
                j = runner.jobs.get(parts[1])
                return self._send(200, runner.job_state(j)) if j else self._err(404, f"job {parts[1]} not found")
            return self._err(404, f"no such resource {u.path}")

        def do_POST(self):  # noqa: N802
            u = urllib.parse.urlparse(self.path)
            parts = [p for p in u.path.split("/") if p]
            body = self.rfile.read(int(self.headers.get("Content-Length", "0") or 0))
            if parts == ["jars", "upload"]:
                try:
                    ctype = self.headers.get("Content-Type", "")
                    if ctype.startswith("multipart/form-data"):
                        name, data = _multipart_file(body, ctype)
                    else:
                        name, data = os.path.basename(self.headers.get("X-Filename", "program.py")), body
                except Exception as e:  # noqa: BLE001
                    return self._err(400, f"bad upload: {e}")
                jid = f"{uuid.uuid4().hex[:8]}_{name}"
                (runner.dir / "jars" / jid).write_bytes(data)
                return self._send(200, {"filename": str(runner.dir / "jars" / jid), "status": "success"})
            if len(parts) == 3 and parts[0] == "jars" and parts[2] == "run":
                q = urllib.parse.parse_qs(u.query)
                try:
                    jid = runner.run(parts[1], (q.get("entry-class") or [""])[0], (q.get("program-args") or [""])[0])
                except KeyError as e:
                    return self._err(404, str(e).strip("'"))
                except RuntimeError as e:
                    return self._err(409, str(e))
                except ValueError as e:
                    return self._err(400, str(e))
                return self._send(200, {"jobid": jid})
            return self._err(404, f"no such resource {u.path}")

        def do_PATCH(self):  # noqa: N802
            parts = [p for p in urllib.parse.urlparse(self.path).path.split("/") if p]
            if len(parts) == 2 and parts[0] == "jobs" and parts[1] in runner.jobs:
                runner.cancel(parts[1])
                return self._send(202, {})
            return self._err(404, "job not found")

    return H


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--slots", type=int, default=1)
    ap.add_argument("--taskmanagers", type=int, default=1)
    a = ap.parse_args(argv)
    workdir = Path.cwd()
    runner = Runner(workdir, a.slots, a.taskmanagers)
    srv = ThreadingHTTPServer(("127.0.0.1", 0), make_handler(runner))
    stop = threading.Event()

    def on_term(signum, frame):
        stop.set()

    signal.signal(signal.SIGTERM, on_term)
    signal.signal(signal.SIGINT, on_term)
    th = threading.Thread(target=srv.serve_forever, daemon=True)
    th.start()
    port = srv.server_address[1]
    info = {"endpoint": f"http://127.0.0.1:{port}", "appId": os.environ.get("HOPSX_EXECUTION_ID", ""),
            "pid": os.getpid(), "slots": runner.slots}
    tmp = workdir / "runner.json.tmp"
    tmp.write_text(json.dumps(info))
    os.replace(tmp, workdir / "runner.json")  # readiness: the endpoint is published
    print(f"runner up at {info['endpoint']} with {runner.slots} task slot(s)", flush=True)
    while not stop.wait(0.2):
        pass
    runner.shutdown()
    srv.shutdown()
    (workdir / "runner.json").unlink(missing_ok=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
