"""Checkpoint / resume for hopsx training.

The reference checkpoints through Keras ``ModelCheckpoint(filepath=log_dir)`` once per epoch
(notebooks/ml/Distributed_Training/mirrored_strategy/mirroredstrategy_mnist_example.ipynb:210-213)
and ``torch.save(state_dict)`` (notebooks/ml/Experiment/PyTorch/mnist.ipynb:215); it has no resume
API.  Here a checkpoint captures everything a hipGraph-replayed step depends on:

* the flat fp32 master arena (every parameter is a view of it) and every optimizer state
  buffer of that arena, so a resumed run continues bit-for-bit from the same floats;
* each optimizer's device step counter (bias correction) and the dropout RNG (seed, counter);
* any non-arena module buffers (BatchNorm running stats) via ``module.state_dict()``;
* user extras (epoch, data-loader cursor, best metric ...).

Writes are rank-0 only, atomic (temp file + ``os.replace``) and followed by a barrier so all
ranks see the file; loads read on every rank (``weights_only=True``: nothing executes).
Files are ``<dir>/ckpt-<step>.pt`` and ``latest()`` resolves the newest one, which is what
``experiment.mirrored(..., max_restarts=N)`` relies on to restart a failed job.
"""
from __future__ import annotations

import os
import re
from pathlib import Path

import torch

from .parallel import dist as hdist

_NAME = re.compile(r"^ckpt-(\d+)\.pt$")


def _arena(model):
    return getattr(model, "_hx_arena", None)


def _rng_tensor(device):
    from .ops.functional import rng_state

    return rng_state(device)


def gather_sharded(model) -> None:
    """Collective (every rank): a sharded data-parallel engine keeps parts of the fp32 master and
    of the optimizer moments current only on their owner rank (ShardedPS on GPU all-gathers only
    the bf16 shadow; the fused P2P step keeps moments owner-only).  Reassemble them so the
    checkpoint written by rank 0 holds every shard's real values, not its stale local copy."""
    arena = _arena(model)
    eng = getattr(arena, "_hx_engine", None) if arena is not None else None
    if eng is not None and hasattr(eng, "gather_state"):
        eng.gather_state()


def state(model, optimizer=None, step: int = 0, **extra) -> dict:
    """Collect a CPU-resident checkpoint dict (no file I/O)."""
    sd: dict = {"step": int(step), "extra": extra}
    arena = _arena(model)
    if arena is not None:
        sd["arena"] = arena.state_dict()
        sd["arena_numel"] = int(arena.numel)
        dev = arena.device
    else:
        dev = next(model.parameters()).device
    # non-arena tensors (BN running stats, buffers); arena params are restored from the arena
    sd["module"] = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    opts = optimizer if isinstance(optimizer, (list, tuple)) else ([optimizer] if optimizer is not None else [])
    sd["optim"] = []
    for o in opts:
        od = {"lr": float(getattr(o, "lr", 0.0))}
        sc = getattr(o, "step_count", None)
        if isinstance(sc, torch.Tensor):
            od["step_count"] = sc.detach().cpu()
        if hasattr(o, "_sl"):
            od["slice"] = [o._sl.start, o._sl.stop]
        sd["optim"].append(od)
    sd["rng"] = _rng_tensor(dev).detach().cpu()
    sd["torch_rng"] = torch.get_rng_state()
    return sd


def restore(sd: dict, model, optimizer=None) -> dict:
    """Apply a checkpoint dict to ``model`` / ``optimizer``; returns ``{"step", **extra}``."""
    arena = _arena(model)
    with torch.no_grad():
        model_sd = model.state_dict()
        for k, v in sd.get("module", {}).items():
            if k in model_sd and model_sd[k].shape == v.shape:
                model_sd[k].copy_(v.to(model_sd[k].device))
    if arena is not None and "arena" in sd:
        if int(sd.get("arena_numel", arena.numel)) != arena.numel:
            raise ValueError(f"checkpoint arena has {sd['arena_numel']} elements, model arena {arena.numel}")
        arena.load_state_dict(sd["arena"])
        arena.zero_grad()
        dev = arena.device
    else:
        dev = next(model.parameters()).device
    opts = optimizer if isinstance(optimizer, (list, tuple)) else ([optimizer] if optimizer is not None else [])
    for o, od in zip(opts, sd.get("optim", [])):
        if "lr" in od and hasattr(o, "lr"):
            o.lr = od["lr"]
            if getattr(o, "param_groups", None):
                o.param_groups[0]["lr"] = od["lr"]
        if "step_count" in od and isinstance(getattr(o, "step_count", None), torch.Tensor):
            o.step_count.copy_(od["step_count"].to(o.step_count.device))
    if "rng" in sd:
        _rng_tensor(dev).copy_(sd["rng"].to(dev))
    if "torch_rng" in sd:
        torch.set_rng_state(sd["torch_rng"])
    return {"step": int(sd.get("step", 0)), **sd.get("extra", {})}


def save(directory, model, optimizer=None, step: int = 0, keep: int = 3, **extra) -> Path | None:
    """Write ``<directory>/ckpt-<step>.pt`` on rank 0 (atomic), keep the newest ``keep``, barrier.
    Returns the path on rank 0, None elsewhere."""
    d = Path(directory)
    path = d / f"ckpt-{int(step)}.pt"
    out = None
    gather_sharded(model)  # collective: owner-only shards (parameter server / fused P2P step) -> rank 0
    sd = state(model, optimizer, step, **extra) if hdist.rank() == 0 else None
    if hdist.rank() == 0:
        d.mkdir(parents=True, exist_ok=True)
        tmp = d / f".ckpt-{int(step)}.pt.tmp"
        torch.save(sd, tmp)
        os.replace(tmp, path)
        if keep and keep > 0:
            for old in list_checkpoints(d)[:-keep]:
                try:
                    old.unlink()
                except OSError:
                    pass
        out = path
    hdist.barrier()
    return out


def list_checkpoints(directory) -> list[Path]:
    d = Path(directory)
    if not d.is_dir():
        return []
    found = [(int(m.group(1)), d / n) for n in os.listdir(d) if (m := _NAME.match(n))]
    return [p for _, p in sorted(found)]


def latest(directory) -> Path | None:
    c = list_checkpoints(directory)
    return c[-1] if c else None


def load(path_or_dir, model, optimizer=None) -> dict | None:
    """Restore from a file, or from the newest checkpoint of a directory (None if there is none,
    e.g. the first attempt of a job whose checkpoint directory does not exist yet)."""
    p = Path(path_or_dir)
    if not p.exists():
        return None
    if p.is_dir():
        p = latest(p)
        if p is None:
            return None
    sd = torch.load(p, map_location="cpu", weights_only=True)
    return restore(sd, model, optimizer)


class CheckpointHook:
    """Periodic checkpointing for hand-written loops: ``hook(step)`` saves every ``every`` steps."""

    def __init__(self, directory, model, optimizer=None, every: int = 100, keep: int = 3):
        self.directory, self.model, self.optimizer, self.every, self.keep = directory, model, optimizer, every, keep

    def resume(self) -> int:
        r = load(self.directory, self.model, self.optimizer)
        return 0 if r is None else r["step"]

    def __call__(self, step: int, **extra) -> None:
        if self.every > 0 and step > 0 and step % self.every == 0:
            save(self.directory, self.model, self.optimizer, step=step, keep=self.keep, **extra)
