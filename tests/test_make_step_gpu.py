"""runtime.step.make_step: the framework's step factory picks the persistent whole-step kernel for the
reference's MirroredStrategy MNIST CNN (mirroredstrategy_mnist_example.ipynb:189-231) — through the
API, not only in bench.py — and falls back to TrainStep where the kernel cannot be resident."""
import os
import re
import subprocess
import sys
from pathlib import Path

import pytest
import torch

pytestmark = pytest.mark.gpu
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from hops_examples_amd import optim  # noqa: E402
from hops_examples_amd.models.mnist import MirroredMnistCNN  # noqa: E402
from hops_examples_amd.runtime import persist  # noqa: E402
from hops_examples_amd.runtime.arena import ParamArena  # noqa: E402
from hops_examples_amd.runtime.step import make_step  # noqa: E402

dev = torch.device("cuda", 0)
ROOT = Path(__file__).resolve().parents[1]


def _model():
    torch.manual_seed(0)
    m = MirroredMnistCNN().to(dev)
    ParamArena.from_module(m, dev)
    return m, optim.Adadelta(m, lr=1.0)


def test_make_step_picks_the_persistent_engine_and_trains():
    m, opt = _model()
    st = make_step(m, opt, "sparse_ce", batch=32)
    assert st.kind == "persistent" and isinstance(st, persist.PersistentMnistStep)
    assert persist.launchable(dev)[0] and persist._occupancy(False) >= 1
    xs = torch.randint(0, 256, (8, 32, 28, 28, 1), dtype=torch.uint8, device=dev)
    ys = torch.randint(0, 10, (8, 32), device=dev)
    l0 = float(st.run_resident(xs, ys, 1)["loss"])
    for _ in range(6):
        r = st.run_resident(xs, ys, 40)
    st.check()
    assert float(r["loss"]) < l0  # the 8 random batches are memorised
    r = st(xs[0], ys[0])  # the TrainStep call form: one step on an explicit batch
    assert torch.isfinite(r["loss"]).item()


def test_make_step_falls_back_when_the_grid_cannot_be_resident(monkeypatch):
    monkeypatch.setattr(persist, "_device_cus", lambda d: 128)  # a partitioned GPU
    m, opt = _model()
    st = make_step(m, opt, "sparse_ce", batch=32)
    assert st.kind == "trainstep" and "128 CUs" in st.note
    xs = torch.randint(0, 256, (4, 32, 28, 28, 1), dtype=torch.uint8, device=dev)
    ys = torch.randint(0, 10, (4, 32), device=dev)
    r = st.run_resident(xs, ys, 8)
    assert torch.isfinite(r["loss"]).all().item()


def test_mirrored_example_runs_the_persistent_engine(tmp_path):
    """examples/ml/Distributed_Training/mirrored_mnist.py through experiment.mirrored on one GPU."""
    env = dict(os.environ, HOPSX_NUM_GPUS="1", PYTHONPATH=str(ROOT), HOPSX_REPO=str(ROOT),
               HOPSX_PROJECT_ROOT=str(tmp_path / "project"), HOPSX_PROJECT_NAME="demo")
    env.pop("HOPSX_FAST", None)
    r = subprocess.run([sys.executable, str(ROOT / "examples/ml/Distributed_Training/mirrored_mnist.py")],
                       env=env, cwd=tmp_path, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if "images_per_sec" in ln][-1]
    print(line)
    eng = re.search(r"'engine': '(\w+)'", line).group(1)
    ips = float(re.search(r"'images_per_sec': ([0-9.e+]+)", line).group(1))
    assert eng == "persistent"
    assert ips > 5e5
