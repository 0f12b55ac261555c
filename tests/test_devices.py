"""hops.devices (notebooks/ml/Benchmarks/benchmark.ipynb:111-112): GPU count and architecture."""
import pytest
import torch

from hops_examples_amd import devices


def test_kfd_target_version_decoding():
    assert devices._gfx_name(90500) == "gfx950"
    assert devices._gfx_name(90402) == "gfx942"
    assert devices._gfx_name(90010) == "gfx90a"
    assert devices._gfx_name(110001) == "gfx1101"


def test_arch_list_is_consistent_with_count():
    archs = devices.list_gpu_archs()
    assert all(a.startswith("gfx") for a in archs)
    if not archs:
        assert devices.get_gpu_arch(0) in ("",) or torch.cuda.is_available()


@pytest.mark.gpu
@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a GPU")
def test_gpu_arch_is_gfx950():
    assert devices.get_num_gpus() >= 1
    assert devices.get_gpu_arch(0) == "gfx950"
    assert torch.cuda.get_device_properties(0).gcnArchName.startswith(devices.get_gpu_arch(0))
