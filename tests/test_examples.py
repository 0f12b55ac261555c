"""Run the example scripts (the notebook sources) end to end on CPU with HOPSX_FAST=1, each in
its own interpreter and project directory."""
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
EXAMPLES = sorted(p for p in (ROOT / "examples").rglob("*.py"))
SLOW = {"resnet50_benchmark.py", "inference_hello_world.py"}  # ResNet-50 on CPU: minutes


@pytest.mark.parametrize("path", [p for p in EXAMPLES if p.name not in SLOW], ids=lambda p: str(p.relative_to(ROOT)))
def test_example_runs(path, tmp_path):
    env = dict(os.environ, HOPSX_FAST="1", HOPSX_PROJECT_ROOT=str(tmp_path / "project"), HOPSX_PROJECT_NAME="demo",
               HOPSX_NUM_GPUS="0", PYTHONPATH=str(ROOT), HOPSX_REPO=str(ROOT))
    r = subprocess.run([sys.executable, str(path)], cwd=tmp_path, env=env, capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
