"""One-shot / two-shot all-reduce for small and mid-size messages over IPC-mapped peer buffers (``_hopsx_comm``).

SURVEY §5.8 item 3 / §2.4: a ring all-reduce needs 2(N-1) latency-bound hops, but MI355X wires
every GPU to its 7 peers directly over xGMI, so below ~1 MB one hop is cheaper: each rank stages
its data in an IPC-shared buffer, flags every peer, and sums all N staging buffers itself
(csrc/comm/oneshot.hip).  Small models (the taxi wide&deep net's 75 KB of gradients, metric
scalars C7) and small buckets use it; larger buckets stay on RCCL rings.

Setup exchanges ``hipIpcMemHandle`` bytes through the default process group (any backend), so
it works for RCCL and gloo groups alike.  The launch is hipGraph-capturable (device-resident
epochs).  A peer that never arrives sets an error flag instead of hanging; ``check()`` raises.

Reference parity: the implicit TF collectives of MirroredStrategy.
"""
from __future__ import annotations

import importlib
import os

import torch
import torch.distributed as dist

from . import dist as hdist

_ext = None


def ext():
    global _ext
    if _ext is None:
        try:
            _ext = importlib.import_module("hops_examples_amd._hopsx_comm")
        except ImportError as e:
            raise RuntimeError("hopsx comm library _hopsx_comm is not built: run "
                               "`python -m hops_examples_amd._build`") from e
    return _ext


def enabled() -> bool:
    """Opt-in via HOPSX_ONESHOT_AR=1 (RCCL rings remain the default for every bucket)."""
    return os.environ.get("HOPSX_ONESHOT_AR", "0") == "1"


class OneShotAllReduce:
    """Sum-all-reduce of fp32 device tensors of up to ``cap_bytes`` across the default group."""

    def __init__(self, cap_bytes: int = 8 << 20, blocks: int = 64, device=None):
        C = ext()
        self.rank, self.world = hdist.rank(), hdist.world_size()
        if self.world > C.MAX_RANKS:
            raise ValueError(f"one-shot all-reduce supports <= {C.MAX_RANKS} ranks (one node)")
        self.device = device or hdist.device()
        self.cap = (int(cap_bytes) // 4 + 3) & ~3
        self.blocks = max(1, min(int(blocks), C.MAX_BLOCKS))
        self._buf, hb = C.alloc(4 * self.cap * 4, False)
        self._flag, hf = C.alloc(C.FLAG_ROWS * C.MAX_RANKS * C.MAX_BLOCKS * 4, True)
        # two-shot (reduce-scatter + all-gather) above this size when N > 2: 2(N-1)/N * n of xGMI
        # reads per GPU instead of (N-1) * n
        self.two_shot_min = int(os.environ.get("HOPSX_TWOSHOT_MIN_KB", "256")) * 1024 // 4
        self._opened: list[int] = []
        if self.world > 1:
            objs = [None] * self.world
            dist.all_gather_object(objs, (self.rank, bytes(hb), bytes(hf)))
            bufs, flags = [0] * self.world, [0] * self.world
            for r, b, f in objs:
                if r == self.rank:
                    bufs[r], flags[r] = self._buf, self._flag
                else:
                    bufs[r], flags[r] = C.open(b), C.open(f)
                    self._opened += [bufs[r], flags[r]]
        else:
            bufs, flags = [self._buf], [self._flag]
        self.bufs, self.flags = bufs, flags
        self.epochs = torch.zeros(C.MAX_BLOCKS, dtype=torch.int32, device=self.device)
        self.err = torch.zeros(1, dtype=torch.int32, device=self.device)
        hdist.barrier()

    def fits(self, t: torch.Tensor) -> bool:
        return (t.dtype == torch.float32 and t.is_contiguous() and t.numel() <= self.cap
                and t.data_ptr() % 16 == 0)

    def mode(self, n: int) -> str:
        return "two_shot" if self.world > 2 and n >= self.two_shot_min else "one_shot"

    def __call__(self, t: torch.Tensor, out: torch.Tensor | None = None, mode: str | None = None) -> torch.Tensor:
        """In place by default; identical (rank-ordered) sums on every rank."""
        if not self.fits(t):
            raise ValueError("tensor must be contiguous fp32, 16-B aligned and within the staging capacity")
        out = t if out is None else out
        if not self.fits(out) or out.numel() != t.numel():
            raise ValueError("bad output tensor")
        st = torch.cuda.current_stream(self.device).cuda_stream
        ext().allreduce_f32(t.data_ptr(), out.data_ptr(), t.numel(), self.cap, self.rank, self.world,
                            self.bufs, self.flags, self.epochs.data_ptr(), self.err.data_ptr(), self.blocks, st,
                            (mode or self.mode(t.numel())) == "two_shot")
        return out

    def check(self) -> None:
        """Raise if a peer failed to arrive within the spin bound (synchronises the device)."""
        e = int(self.err.item())
        if e:
            raise RuntimeError(f"one-shot all-reduce: rank {e - 1} never raised its flag (peer lost?)")

    def close(self) -> None:
        if self._buf is None:
            return
        torch.cuda.synchronize(self.device)
        hdist.barrier()  # no peer may still read our staging buffer
        C = ext()
        for p in self._opened:
            C.close(p)
        C.free(self._buf)
        C.free(self._flag)
        self._buf = self._flag = None
        self._opened = []
