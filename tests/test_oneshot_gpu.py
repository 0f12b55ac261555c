"""One-shot xGMI all-reduce (csrc/comm/oneshot.hip): 2 ranks sharing the GPU, bitwise equal to the
rank-ordered fp32 sum, epoch reuse and hipGraph replay (tools/oneshot_check.py)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_oneshot_allreduce_two_ranks():
    env = dict(os.environ, HOPSX_DIST_BACKEND="gloo", HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29633", os.path.join(ROOT, "tools", "oneshot_check.py")]
    r = subprocess.run(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                       timeout=110)
    assert r.returncode == 0 and "ONESHOT" in r.stdout, r.stdout[-3000:]


def test_oneshot_module_imports_without_gpu():
    from hops_examples_amd.parallel import oneshot

    assert oneshot.enabled() in (True, False)
