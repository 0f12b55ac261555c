"""ResNet-20 through DataParallel on two gloo ranks (CPU): bucketed all-reduces launched from
hooks.grad_ready during the backward keep the replicas bit-identical (tools/dp_resnet_check.py; the
GPU variants with the padded stem and the zero-copy P2P step are in tests/test_p2p_gpu.py)."""
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def test_dp_resnet_overlap_two_gloo_ranks(capfd):
    sys.path.insert(0, str(ROOT))
    from hops_examples_amd.parallel import launch

    env = {"HOPSX_DIST_BACKEND": "gloo", "HOPSX_DPR_MODE": "pg", "CUDA_VISIBLE_DEVICES": "", "HIP_VISIBLE_DEVICES": "",
           "PYTHONPATH": str(ROOT)}
    rc = launch.launch(2, [str(ROOT / "tools" / "dp_resnet_check.py")], rehearse=True, timeout_s=240, extra_env=env)
    out = capfd.readouterr().out
    assert rc == 0, out[-3000:]
    assert "DPRESNET" in out and '"replicas_identical": true' in out, out[-3000:]
