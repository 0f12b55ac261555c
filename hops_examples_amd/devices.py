"""``hops.devices``: accelerators visible to this worker (imported by the reference
notebooks, e.g. notebooks/ml/Benchmarks/benchmark.ipynb:111-112).  Counting does
not initialise the GPU runtime on ROCm."""
from __future__ import annotations

import os


def get_num_gpus() -> int:
    env = os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("CUDA_VISIBLE_DEVICES")
    try:
        import torch

        return torch.cuda.device_count()
    except Exception:  # pragma: no cover
        return len(env.split(",")) if env else 0


def get_gpu_arch() -> str:
    return "gfx950"
