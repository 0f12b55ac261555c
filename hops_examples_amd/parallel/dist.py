"""Process-group bootstrap: one process per GPU, RCCL over xGMI on MI355X
(``backend="nccl"`` is RCCL on ROCm), gloo on CPU.

Reads the torchrun contract (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR /
MASTER_PORT).  This replaces TF's TF_CONFIG cluster spec that
``experiment.mirrored`` builds for MultiWorkerMirroredStrategy in the reference
(notebooks/ml/Distributed_Training/multiworker_mirrored_strategy/multiworkermirroredstrategy_mnist_example.ipynb:137).
"""
from __future__ import annotations

import datetime
import os

import torch
import torch.distributed as dist


def env_world() -> tuple[int, int, int]:
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0")),
            int(os.environ.get("WORLD_SIZE", "1")))


def init(backend: str | None = None, timeout_s: float = 600.0) -> tuple[int, int, int]:
    """Initialise the default process group if WORLD_SIZE > 1 (idempotent).

    Returns (rank, local_rank, world_size) and pins this process to cuda:local_rank.
    """
    rank, local_rank, world = env_world()
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    if torch.cuda.is_available():
        torch.cuda.set_device(local_rank % max(1, torch.cuda.device_count()))
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29500")
        if backend is None:
            # HOPSX_DIST_BACKEND=gloo rehearses the multi-rank GPU path with several ranks on one
            # GPU (RCCL refuses two ranks per device); production is RCCL ("nccl")
            backend = os.environ.get("HOPSX_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
        kw = {}
        if backend == "nccl":
            kw["device_id"] = torch.device("cuda", torch.cuda.current_device())
        dist.init_process_group(backend=backend, rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=timeout_s), **kw)
        # every rank all-reduces a known vector at startup, so a broken fabric / wrong
        # rendezvous fails here, loudly, instead of as silently diverging replicas later
        if os.environ.get("HOPSX_DIST_SELFTEST", "1") == "1" and not self_test():
            raise RuntimeError(f"collective self-test failed on rank {rank}: an all-reduce of rank+1 over "
                               f"{world} ranks did not sum to {world * (world + 1) // 2} (backend {backend})")
    return rank, local_rank, world


def is_dist() -> bool:
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


def rank() -> int:
    return dist.get_rank() if is_dist() else 0


def world_size() -> int:
    return dist.get_world_size() if is_dist() else 1


def barrier() -> None:
    if is_dist():
        if dist.get_backend() == "nccl":
            dist.barrier(device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier()


def device() -> torch.device:
    if torch.cuda.is_available():
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def all_reduce_(t: torch.Tensor, op: str = "sum") -> torch.Tensor:
    if is_dist():
        dist.all_reduce(t, op={"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN}[op])
    return t


def all_reduce_scalar(v: float, op: str = "sum") -> float:
    if not is_dist():
        return float(v)
    t = torch.tensor([float(v)], dtype=torch.float64, device=device())
    return float(all_reduce_(t, op).item())


def broadcast_(t: torch.Tensor, src: int = 0) -> torch.Tensor:
    if is_dist():
        dist.broadcast(t, src)
    return t


def self_test() -> bool:
    """All-reduce checksum self-test: every rank contributes rank+1."""
    n = world_size()
    dev = device() if (not is_dist() or dist.get_backend() == "nccl") else torch.device("cpu")
    t = torch.full((1024,), float(rank() + 1), device=dev)
    all_reduce_(t)
    ok = bool(torch.all(t == n * (n + 1) / 2).item())
    return ok


# Native resources a rank holds, torn down by ``shutdown`` in a fixed order: first the P2P comm handles
# (IPC-mapped peer buffers: unmapped while every peer and the process group still exist), then the
# Parquet staging pools (decode threads joined, pinned memory freed while the HIP runtime is alive),
# last the process group.  Interpreter exit runs the same order locally (atexit: no collectives), so no
# destructor of a mapped buffer or a pool thread runs after the runtime or the group it needs is gone.
ORDER_COMM, ORDER_STAGING = 0, 1
_RESOURCES: list = []


def register(obj, order: int = ORDER_COMM) -> None:
    """Track ``obj`` (weakly) for ordered teardown: ``close()`` (collective) from ``shutdown()``,
    ``release_local()`` (else ``close()``) at interpreter exit."""
    import weakref

    _RESOURCES.append((order, weakref.ref(obj)))


def _teardown(collective: bool) -> list:
    errors = []
    for order in (ORDER_COMM, ORDER_STAGING):
        for o, ref in reversed(list(_RESOURCES)):
            obj = ref()
            if o != order or obj is None:
                continue
            fn = obj.close if collective or not hasattr(obj, "release_local") else obj.release_local
            try:
                fn()
            except Exception as e:  # noqa: BLE001 - keep tearing the rest down
                errors.append(repr(e))
    _RESOURCES.clear()
    import sys

    pq = sys.modules.get("hops_examples_amd.io.parquet")
    if pq is not None:
        pq.close_staging()
    return errors


def shutdown(collective: bool = True) -> None:
    """Ordered teardown (see ``register``) and the process group.  ``collective``: every rank calls it
    (the comm handles' close synchronises the ranks); atexit runs it with ``collective=False``."""
    _teardown(collective)
    if dist.is_available() and dist.is_initialized():
        if collective:
            dist.destroy_process_group()


def _at_exit() -> None:
    try:
        _teardown(False)
    except Exception:  # noqa: BLE001
        pass


import atexit  # noqa: E402

atexit.register(_at_exit)
