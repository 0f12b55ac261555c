"""``hops.devices``: accelerators visible to this worker (imported by the reference
notebooks, e.g. notebooks/ml/Benchmarks/benchmark.ipynb:111-112).  Counting does
not initialise the GPU runtime on ROCm; the architecture query reads the KFD
topology (sysfs) first and only falls back to the HIP runtime when that is absent."""
from __future__ import annotations

import glob
import os

_KFD_NODES = "/sys/class/kfd/kfd/topology/nodes"


def get_num_gpus() -> int:
    env = os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("CUDA_VISIBLE_DEVICES")
    try:
        import torch

        return torch.cuda.device_count()
    except Exception:  # pragma: no cover
        return len(env.split(",")) if env else 0


def _gfx_name(target_version: int) -> str:
    """KFD ``gfx_target_version`` (major*10000 + minor*100 + stepping, minor/stepping in hex digits)
    -> LLVM target name, e.g. 90500 -> gfx950, 90402 -> gfx942."""
    major, minor, step = target_version // 10000, (target_version // 100) % 100, target_version % 100
    return f"gfx{major}{minor:x}{step:x}"


def list_gpu_archs() -> list:
    """Architectures of the GPU agents in the KFD topology (CPU nodes report version 0), in node order."""
    archs = []
    for node in sorted(glob.glob(os.path.join(_KFD_NODES, "*")), key=lambda p: int(os.path.basename(p))):
        try:
            with open(os.path.join(node, "properties")) as f:
                props = dict(line.split(None, 1) for line in f if " " in line.strip())
        except (OSError, ValueError):
            continue
        tv = int(props.get("gfx_target_version", "0").strip() or 0)
        if tv:
            archs.append(_gfx_name(tv))
    return archs


def get_gpu_arch(device: int = 0) -> str:
    """The ``gfxNNN`` target of visible GPU ``device`` ('' when there is none)."""
    archs = list_gpu_archs()
    vis = os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("ROCR_VISIBLE_DEVICES")
    if archs and vis:
        try:
            archs = [archs[int(i)] for i in vis.split(",") if i.strip()]
        except (ValueError, IndexError):
            pass
    if device < len(archs):
        return archs[device]
    try:
        import torch

        if torch.cuda.is_available() and device < torch.cuda.device_count():
            return torch.cuda.get_device_properties(device).gcnArchName.split(":")[0]
    except Exception:  # pragma: no cover
        pass
    return ""
