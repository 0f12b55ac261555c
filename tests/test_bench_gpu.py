"""bench.py on one GPU: the persistent engine's run, and the fallback when a persistent run reports a hand-off
error (HOPSX_BENCH_FAKE_PERSIST_ERR sets the error word after the timed run): the bench then times the
multi-kernel engine and says so, instead of dying without a JSON line."""
import json
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(env_extra):
    env = dict(os.environ, **env_extra)
    r = subprocess.run([sys.executable, "bench.py", "--steps", "20", "--warmup", "3", "--no-taxi"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_bench_persistent_and_fallback():
    ok = _bench({})
    assert ok["config"]["engine"] == "PersistentMnistStep" and ok["value"] > 0
    fb = _bench({"HOPSX_BENCH_FAKE_PERSIST_ERR": str((3 << 24) | 5)})
    assert fb["config"]["engine"] == "TrainStep", fb["config"]
    assert "timed on TrainStep instead" in (fb["config"]["persistent_note"] or "")
    assert fb["value"] > 0 and fb["final_loss"] == fb["final_loss"]
