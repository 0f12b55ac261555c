import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture
def project_root(tmp_path, monkeypatch):
    """An isolated hopsx project (replaces a Hopsworks project on HopsFS)."""
    root = tmp_path / "project"
    monkeypatch.setenv("HOPSX_PROJECT_ROOT", str(root))
    monkeypatch.setenv("HOPSX_PROJECT_NAME", "demo")
    from hops_examples_amd import config as _cfg

    _cfg.reset()
    yield root
    _cfg.reset()


@pytest.fixture(autouse=True)
def _hopsx_device_checks(request):
    """HOPSX_DEBUG=1 (the _hopsx_ops_dbg build): every GPU test ends with no device-side check record
    (common.h hx_check); without it this fixture does nothing."""
    yield
    if os.environ.get("HOPSX_DEBUG", "0") != "1" or request.node.get_closest_marker("gpu") is None:
        return
    from hops_examples_amd.ops import _C

    errs = _C.debug_errors()
    assert not errs, f"device-side bound checks failed: {errs}"
