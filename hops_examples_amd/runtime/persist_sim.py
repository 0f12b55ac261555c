"""ExchangeSim: one process plays every rank of the persistent flagship's data-parallel step, each rank
on its OWN batch, through the real (non-loopback) exchange code of csrc/ops/mnist_persist.hip.

Why.  Two ranks of the persistent kernel cannot share one GPU (2 x 201 one-per-CU workgroups), and the
loopback mode (one kernel, every "peer" slot holding this rank's own payload) only proves
x/W + ... + x/W = x.  The MirroredStrategy step the headline runs at 2/4/8 GPUs sums DIFFERENT
gradients (mirroredstrategy_mnist_example.ipynb:125-131).  What makes a faithful single-GPU rehearsal
possible: a replica's exchange payloads for one step — its pooled-activation and dh^T fragments, head
gradients and conv slice sums — depend only on the step's (replica-identical) weights and its own batch,
never on a peer's payload.  So one step of W ranks is:

  1. harvest: for each rank r, from the step's start state, launch the real DP kernel as rank r of W on
     batch r.  Its pushes land in a SINK buffer standing in for every peer (slot r of parity 0), its own
     flag page is pre-raised so its waits pass; the update it computes is discarded.
  2. inject: for each rank q, from the same start state, copy every other rank's harvested payload into
     q's own exchange buffer at that rank's slot, pre-raise q's flag page, launch as rank q.  q's kernel
     sums the W contributions in rank order exactly as on W GPUs.
  3. the W updated states must be bit-identical (the replicas' invariant), and equal to the fp64
     reference of the global batch (tests/test_persist_dp_sim_gpu.py).

Everything the launch touches besides the exchange (arena, optimizer state, RNG counter, cursor) is
saved and restored around the harvest / inject launches; the local flag epochs and the cross-rank step
counter keep growing (a restored epoch would match stale flags).  ``drop`` (a rank whose injected
payload is zeroed) is the deliberately broken exchange the numeric self-test must catch.
"""
from __future__ import annotations

import torch

from .persist import PersistentMnistStep, geometry

REGIONS = ("pool", "dht", "fc2", "conv")


def _comm():
    from ..parallel import oneshot

    return oneshot.ext()


class ExchangeSim:
    def __init__(self, world: int):
        g = geometry()
        if not 2 <= world <= g["max_ranks"]:
            raise ValueError(f"world must be 2..{g['max_ranks']}")
        self.world = int(world)
        self.g = g
        C = _comm()
        self._bufs = []
        self.own, self.own_h = C.alloc(int(g["x_bytes"]), True)
        self.own_flags, self.own_flags_h = C.alloc(int(g["xflag_words"]) * 4, True)
        self.sink, _ = C.alloc(int(g["x_bytes"]), True)
        self.sink_flags, _ = C.alloc(int(g["xflag_words"]) * 4, True)
        self._bufs = [self.own, self.own_flags, self.sink, self.sink_flags]
        # where pushes to every peer land: the sink, or (cross-process test) a peer process's mapped buffer
        self.peer_buf, self.peer_flags = self.sink, self.sink_flags
        self.eng: PersistentMnistStep | None = None
        self.drop: int | None = None
        self.last_payload: list | None = None

    # ------------------------------------------------------------------ plumbing
    def attach(self, eng: PersistentMnistStep) -> None:
        self.eng = eng
        self._point(0)

    def _point(self, rank: int) -> None:
        """Make the engine rank ``rank`` of W: its own buffer / page at [rank], the sink at every peer."""
        e = self.eng
        e.rank = rank
        bufs = [self.own if r == rank else self.peer_buf for r in range(self.world)]
        flags = [self.own_flags if r == rank else self.peer_flags for r in range(self.world)]
        e._xptrs = [e.xstep.data_ptr()] + bufs + flags

    def _region(self, base: int, name: str, slot: int, par: int = 0) -> tuple[int, int]:
        g = self.g
        xo, xs = int(g["xo_" + name]), int(g["xs_" + name])
        return base + xo + (par * g["max_ranks"] + slot) * xs, xs

    def _raise_own_flags(self) -> None:
        """Every word of the own flag page at the coming launch's cross-rank epoch (xstep + 1)."""
        C = _comm()
        ep = (int(self.eng.xstep.item()) + 1) & 0xFFFFFFFF
        page = torch.full((int(self.g["xflag_words"]),), ep, dtype=torch.int64).to(torch.int32).to(self.eng.device)
        C.copy(self.own_flags, page.data_ptr(), page.numel() * 4)

    def harvest(self, rank: int) -> dict:
        """Copy the payload rank ``rank`` pushed to its peers (the sink, slot ``rank``, parity 0)."""
        C = _comm()
        out = {}
        for n in REGIONS:
            ptr, nb = self._region(self.sink, n, rank)
            t = torch.empty(nb, dtype=torch.uint8, device=self.eng.device)
            C.copy(t.data_ptr(), ptr, nb)
            out[n] = t
        return out

    def inject(self, rank: int, payload: dict, zero: bool = False) -> None:
        C = _comm()
        for n in REGIONS:
            ptr, nb = self._region(self.own, n, rank)
            src = torch.zeros_like(payload[n]) if zero else payload[n]
            C.copy(ptr, src.data_ptr(), nb)

    # ------------------------------------------------------------------ one data-parallel step
    def step(self, xs_list, ys_list) -> list[dict]:
        """One training step of all W replicas, replica r on its resident epoch ``xs_list[r]`` /
        ``ys_list[r]`` (the same cursor).  Leaves the engine in replica 0's post-step state and returns,
        per replica, {"master", "s1", "s2", "loss", "correct"} after the step (device tensors)."""
        e = self.eng
        W = self.world
        if len(xs_list) != W or len(ys_list) != W:
            raise ValueError("one resident epoch per replica")
        nbs = [e._check_data(x, y) for x, y in zip(xs_list, ys_list)]
        if len(set(nbs)) != 1:
            raise ValueError("every replica's epoch must hold the same number of batches")
        nb = nbs[0]
        start = [t.clone() for t in e._state()]

        def restore():
            for t, s in zip(e._state(), start):
                t.copy_(s)

        pay = []
        for r in range(W):
            restore()
            self._point(r)
            self._raise_own_flags()
            e._launch(xs_list[r], ys_list[r], nb, 1)
            torch.cuda.synchronize(e.device)
            e.check()
            pay.append(self.harvest(r))
        self.last_payload = pay
        res = []
        for q in range(W):
            restore()
            self._point(q)
            for r in range(W):
                if r != q:
                    self.inject(r, pay[r], zero=(self.drop == r))
            self._raise_own_flags()
            e._launch(xs_list[q], ys_list[q], nb, 1)
            torch.cuda.synchronize(e.device)
            e.check()
            a = e.arena
            res.append({"master": a.master.clone(), "shadow": a.shadow.clone(), "s1": e.s1.clone(),
                        "s2": e.s2.clone(), "loss": float(e.out[0].item()), "correct": float(e.out[1].item()),
                        "state": [t.clone() for t in e._state()]})
        # leave the engine in replica 0's state
        for t, s in zip(e._state(), res[0]["state"]):
            t.copy_(s)
        self._point(0)
        torch.cuda.synchronize(e.device)
        for r in res:
            r.pop("state")
        return res

    def close(self) -> None:
        if self._bufs:
            torch.cuda.synchronize()
            C = _comm()
            for p in self._bufs:
                C.free(p)
            self._bufs = []
