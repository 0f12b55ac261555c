"""Execution wrapper for :mod:`hops_examples_amd.jobs`: runs the program as a child,
streams its output into the execution directory and records the state transitions
(RUNNING -> FINISHED/FAILED/KILLED) in ``state.json``.

Usage: python -m hops_examples_amd._job_exec <exec_dir> -- <cmd...>
"""
from __future__ import annotations

import json
import os
import signal
import subprocess
import sys
import time
from pathlib import Path


def _update(ed: Path, **kw) -> None:
    p = ed / "state.json"
    s = json.loads(p.read_text()) if p.exists() else {}
    s.update(kw)
    tmp = ed / "state.json.tmp"
    tmp.write_text(json.dumps(s))
    os.replace(tmp, p)


def main() -> int:
    ed = Path(sys.argv[1])
    cmd = sys.argv[sys.argv.index("--") + 1:]
    with open(ed / "stdout.log", "ab") as out, open(ed / "stderr.log", "ab") as err:
        proc = subprocess.Popen(cmd, stdout=out, stderr=err, cwd=str(ed))
        killed = []

        def on_term(signum, frame):
            killed.append(True)
            proc.terminate()
            # a program that does not exit on SIGTERM within the grace period is killed
            import threading

            def _force():
                if proc.poll() is None:
                    proc.kill()

            t = threading.Timer(float(os.environ.get("HOPSX_JOB_KILL_GRACE", "10")), _force)
            t.daemon = True
            t.start()

        signal.signal(signal.SIGTERM, on_term)
        t0 = time.time()
        _update(ed, state="RUNNING", pid=proc.pid, pgid=os.getpgid(0), startTime=t0)
        rc = proc.wait()
    if killed:
        state, final = "KILLED", "KILLED"
    else:
        state, final = ("FINISHED", "SUCCEEDED") if rc == 0 else ("FAILED", "FAILED")
    _update(ed, state=state, finalStatus=final, exitCode=rc, duration=time.time() - t0)
    return 0


if __name__ == "__main__":
    sys.exit(main())
