"""Ordered native teardown at rank exit (parallel/dist.py register / shutdown): comm handles first, then
the staging pools, then the process group — on an explicit shutdown() and, without one, at interpreter
exit (atexit, no collectives).  Two gloo ranks on the CPU, each exiting with everything still alive."""
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
SCRIPT = r'''
import os, sys
sys.path.insert(0, os.environ["HOPSX_REPO"])
import torch
from hops_examples_amd.parallel import dist as hdist
from hops_examples_amd.parallel.dp import DataParallel
from hops_examples_amd.runtime.arena import ParamArena
from hops_examples_amd.io import parquet  # (its staging registry is torn down after the comm handles)

log = open(os.environ["TD_LOG"] + f".{os.environ['RANK']}", "w")
class Handle:  # a stand-in for an IPC-mapped comm handle: records which teardown path ran
    def __init__(self, name): self.name = name
    def close(self): log.write(f"close {self.name}\n"); log.flush()
    def release_local(self): log.write(f"release {self.name}\n"); log.flush()

rank, _, world = hdist.init()
m = torch.nn.Linear(4, 2)
ParamArena.from_module(m, "cpu")
dp = DataParallel(m)  # a live gloo engine with its hooks subscribed
h1, h2 = Handle("a"), Handle("b")
hdist.register(h1); hdist.register(h2)
parquet._STAGING["fake"] = type("S", (), {"slots": [], "pool": None})()  # a live staging entry
if os.environ.get("TD_MODE") == "shutdown":
    hdist.shutdown()
    log.write(f"pg {int(torch.distributed.is_initialized())}\n")
log.write(f"staging {len(parquet._STAGING)}\n"); log.flush()
# (mode "exit": returns with the group, the engine, the handles and the staging entry alive)
'''


@pytest.mark.parametrize("mode", ["exit", "shutdown"])
def test_rank_exit_tears_down_in_order(tmp_path, mode):
    script = tmp_path / "rank.py"
    script.write_text(SCRIPT)
    log = tmp_path / "td"
    env = dict(os.environ, HOPSX_REPO=str(ROOT), TD_LOG=str(log), TD_MODE=mode, HOPSX_DIST_BACKEND="gloo",
               CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    sys.path.insert(0, str(ROOT))
    from hops_examples_amd.parallel import launch

    rc = launch.launch(2, [str(script)], rehearse=True, timeout_s=120, extra_env={k: env[k] for k in (
        "HOPSX_REPO", "TD_LOG", "TD_MODE", "HOPSX_DIST_BACKEND")})
    assert rc == 0
    for r in (0, 1):
        lines = (tmp_path / f"td.{r}").read_text().split("\n")
        if mode == "shutdown":
            # reverse registration order, collective close, then the staging registry, then the group
            assert lines[:4] == ["close b", "close a", "pg 0", "staging 0"], lines
        else:
            # the script ends with everything alive; atexit released the handles locally, in order
            assert lines[0] == "staging 1" and lines[1:3] == ["release b", "release a"], lines
