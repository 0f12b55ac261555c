"""Data-parallel engine: bucketed gradient all-reduce over RCCL, overlapped with backward.

The gradients of a model live in ONE flat fp32 buffer (ParamArena), laid out in
forward order.  Backward produces them roughly in reverse, so buckets are cut
walking the parameters backwards: each bucket is a CONTIGUOUS slice of the
grad buffer — no pack/unpack copies, and the all-reduce is issued the moment
the bucket's last gradient kernel has been enqueued (hopsx kernels notify via
runtime.hooks.grad_ready).  RCCL runs on its own stream, so the collective of
bucket i overlaps the backward kernels of buckets i+1..

Bucket sizing for MI355X xGMI: a ring all-reduce is bound per
link (~153 GB/s x 7 links per GPU); below ~10 MB the per-collective latency
dominates, so models under ~10 M params (every reference CNN) get ONE bucket
and ResNet50-class models 4-8 buckets of >= 16 MB.

On one node the engine prefers the P2P path (parallel/oneshot.py, ``HOPSX_P2P=auto``): the
peers' IPC-mapped staging buffers are read directly over the 7 xGMI links, and when the
optimizer is one fused optimizer over the whole arena the ENTIRE step tail — gradient
reduce-scatter, the optimizer on this rank's 1/N slice, all-gather of the new weights — is one
kernel (``fused_update``) that lives inside the step's hipGraph (so multi-rank steps also replay
``steps_per_execution`` at a time).  Setup is collective and fail-safe: unless every rank maps
its peers and passes the self-test, everyone stays on RCCL.

Modes (the three strategies the reference names):
  * ``mirrored`` / ``collective_allreduce`` — synchronous all-reduce (this class);
  * ``parameter_server`` — see parallel/ps.py (reduce-scatter to shard owners +
    all-gather, i.e. a sharded PS over the same RCCL communicator).
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

from ..runtime import hooks
from ..runtime.arena import ParamArena
from . import dist as hdist
from . import oneshot

MB = 1 << 20


def plan_buckets(arena: ParamArena, bucket_mb: float, first_bucket_mb: float | None = None,
                 min_split_mb: float = 10.0):
    """Contiguous [start, end) slices of the flat grad buffer, in backward order; one bucket for
    arenas of <= ``min_split_mb``."""
    ranges = arena.ranges()
    total_bytes = arena.numel * 4
    if total_bytes <= min_split_mb * MB or bucket_mb <= 0:
        return [(0, arena.numel, [id(p) for p, _, _ in ranges])]
    cap = int(bucket_mb * MB / 4)
    first_cap = int((first_bucket_mb or bucket_mb) * MB / 4)
    buckets = []
    end = arena.numel
    cur_ids, cur_start = [], arena.numel
    limit = first_cap
    for p, off, n in reversed(ranges):
        cur_ids.append(id(p))
        cur_start = off
        if end - cur_start >= limit:
            buckets.append((cur_start, end, cur_ids))
            end, cur_ids, limit = cur_start, [], cap
    if cur_ids:
        buckets.append((0, end, cur_ids))
    elif buckets and buckets[-1][0] != 0:
        s, e, ids = buckets[-1]
        buckets[-1] = (0, e, ids)
    return buckets


class DataParallel:
    def __init__(self, model_or_arena, bucket_mb: float = 25.0, overlap: bool = True, broadcast: bool = True,
                 grad_dtype: torch.dtype = torch.float32, p2p: bool | None = None):
        """``p2p``: None follows ``HOPSX_P2P`` (auto), False forces RCCL / the process group."""
        if isinstance(model_or_arena, ParamArena):
            self.arena = model_or_arena
        else:
            self.arena = getattr(model_or_arena, "_hx_arena", None) or ParamArena.from_module(model_or_arena)
        self.world = hdist.world_size()
        self.overlap = overlap and self.world > 1
        # HOPSX_DP_BUCKET_MB / HOPSX_DP_MIN_SPLIT_MB override the bucket plan (tests split small models)
        bucket_mb = float(os.environ.get("HOPSX_DP_BUCKET_MB", bucket_mb))
        self.buckets = plan_buckets(self.arena, bucket_mb,
                                    min_split_mb=float(os.environ.get("HOPSX_DP_MIN_SPLIT_MB", "10")))
        self._owner = {}
        for bi, (_, _, ids) in enumerate(self.buckets):
            for i in ids:
                self._owner[i] = bi
        self._pending = [len(ids) for _, _, ids in self.buckets]
        self._handles: list = []
        self._launched = [False] * len(self.buckets)
        self.grad_dtype = grad_dtype
        # P2P xGMI collectives (parallel/oneshot.py): staging sized for the whole arena, so every
        # bucket (and the fused step tail) fits
        self._oneshot = None
        if self.world > 1 and (oneshot.enabled() if p2p is None else p2p) and self.arena.grad.is_cuda:
            self._oneshot = oneshot.P2PComm.create(cap_bytes=self.arena.numel * 4, device=self.arena.grad.device)
        self.zero_copy = False
        if self._oneshot is not None:
            self._setup_zero_copy()
        self._rs_stream = None
        self._rs_mode = False
        self._rs_next = 0
        self._fused_opt = None
        self._wmask = None
        self._polls = 0
        self.poll_every = int(os.environ.get("HOPSX_P2P_POLL_EVERY", "64"))
        if broadcast and self.world > 1:
            self.broadcast_params()
        self.arena._hx_engine = self  # checkpoint.save gathers the owner-only optimizer slices
        if self.overlap:
            hooks.subscribe(self._on_ready)
        # ZeRO-1 wire: between sync points the fp32 master is current only on each slice's owner, so a
        # host read of the module's state (export, keras save, a TFX model.pt) would see stale weights.
        # sync_master is collective, so it cannot run from a state_dict() that one rank calls: refuse
        # instead of writing stale weights.
        self._stale = False
        if isinstance(model_or_arena, torch.nn.Module) and hasattr(model_or_arena, "register_state_dict_pre_hook"):
            model_or_arena.register_state_dict_pre_hook(self._state_dict_guard)

    # -------------------------------------------------------------- zero-copy gradients
    def _setup_zero_copy(self) -> None:
        """Collective: put the arena gradient in IPC-shared memory that every peer maps
        (``OneShotAllReduce.make_grad_buffer``), so the fused step's owners read the peers' gradients
        in place — the staging copy + zeroing pass of the copy path disappears (HBM bytes per parameter
        per step: ``grad_hbm_bytes_per_param``).  fp32 gradient wire only (a bf16 wire converts, so it
        stages); ``HOPSX_P2P_ZEROCOPY=0`` keeps the staged copy.  The zero-copy kernels are self-tested
        on the live buffer first; any rank failing keeps every rank on the copy path."""
        comm = self._oneshot
        if os.environ.get("HOPSX_P2P_ZEROCOPY", "1") != "1" or comm.grad_bf16:
            return
        buf = comm.make_grad_buffer(self.arena.numel)
        if buf is None:
            return
        ok = False
        try:
            ok = oneshot.dp_self_test(comm, rounds=3)
        except Exception:  # noqa: BLE001 - a failing self-test keeps the copy path
            ok = False
        if not oneshot._agree(ok):
            comm.gpeers = []
            return
        self.arena.rebind_grad(buf)
        self.zero_copy = True

    @property
    def grad_hbm_bytes_per_param(self) -> float | None:
        """Local HBM bytes per parameter per step that the fused step tail moves for the GRADIENT (the
        optimizer state and weights aside): staged copy = read the gradient + write the staging copy +
        zero the gradient + the owner reading N staged copies of its 1/N slice = 4+4+4+4 = 16 (fp32 wire),
        4+2+4+2 = 12 (bf16 wire); zero-copy = the owner's N in-place reads of its 1/N slice + the zeroing
        = 8 (per-bucket reduce-scatter: + its 4 B in-place write and the tail's 4 B local read = 16, moved
        into the backward's shadow)."""
        if self._fused_opt is None:
            return None
        if self.zero_copy:
            return 16.0 if self._rs_mode else 8.0
        return 12.0 if self._oneshot.grad_bf16 else 16.0

    # -------------------------------------------------------------- per-bucket reduce-scatter
    def _rs_blocks(self) -> int:
        return max(1, min(self._oneshot.blocks, int(os.environ.get("HOPSX_P2P_RS_BLOCKS", "64"))))

    def _on_ready_rs(self, p) -> None:
        """hooks.grad_ready subscriber of the overlapped zero-copy step: when a bucket's last gradient
        kernel is enqueued, reduce-scatter it on the side stream while the backward goes on.  Buckets
        are issued strictly in plan order (a bucket that completes early waits for its predecessors),
        so every rank issues the same sequence."""
        bi = self._owner.get(id(p))
        if bi is None:
            return
        self._pending[bi] -= 1
        while self._rs_next < len(self.buckets) and self._pending[self._rs_next] <= 0:
            self._launch_rs(self._rs_next)
            self._rs_next += 1

    def _launch_rs(self, bi: int) -> None:
        s, e, _ = self.buckets[bi]
        cur = torch.cuda.current_stream(self.arena.device)
        if self._rs_stream is None:
            self._rs_stream = torch.cuda.Stream(self.arena.device)
        self._rs_stream.wait_stream(cur)  # after the bucket's gradient kernels (a fork when capturing)
        self._oneshot.dp_rs(self.arena.grad, s, e, self._rs_blocks(), self._rs_stream)

    def _finish_rs(self) -> None:
        """Issue the buckets the hooks did not (parameters without a grad_ready notification), join the
        side stream, reset the counters for the next step."""
        while self._rs_next < len(self.buckets):
            self._launch_rs(self._rs_next)
            self._rs_next += 1
        if self._rs_stream is not None:
            torch.cuda.current_stream(self.arena.device).wait_stream(self._rs_stream)
        self._rs_next = 0
        self._pending = [len(ids) for _, _, ids in self.buckets]

    # -------------------------------------------------------------- fused P2P step tail
    def bind_optimizer(self, opt) -> None:
        """Called by TrainStep: use the fused reduce-scatter / sharded update / all-gather kernel when
        the P2P path is up and ``opt`` is ONE fused optimizer over the whole arena."""
        from ..optim import FusedOptimizer

        ok = (self._oneshot is not None and os.environ.get("HOPSX_P2P_FUSED", "1") == "1"
              and isinstance(opt, FusedOptimizer) and opt.arena is self.arena
              and opt._sl == slice(0, self.arena.numel) and self.arena.shadow is not None)
        self._fused_opt = opt if ok else None
        self._wmask = self.arena.wire_mask() if ok and self._oneshot.weight_bf16 else None
        if ok and self.overlap:
            hooks.unsubscribe(self._on_ready)  # no per-bucket all-reduce: the step tail does it all
            self.overlap = False
            # zero-copy gradients and more than one bucket: per-bucket reduce-scatter during the backward,
            # the tail then only updates + all-gathers (HOPSX_P2P_OVERLAP=0 keeps one tail kernel)
            if (self.zero_copy and len(self.buckets) > 1 and not self._rs_mode
                    and os.environ.get("HOPSX_P2P_OVERLAP", "1") == "1"):
                self._rs_mode = True
                self._rs_next = 0
                self._pending = [len(ids) for _, _, ids in self.buckets]
                hooks.subscribe(self._on_ready_rs)

    def fuses_optimizer(self, opt) -> bool:
        return self._fused_opt is not None and opt is self._fused_opt

    def fused_update(self, opt) -> None:
        if self._rs_mode:
            self._finish_rs()
            self._oneshot.dp_step(opt, self._wmask, pre_reduced=True, cuts=self._cuts())
        else:
            self._oneshot.dp_step(opt, self._wmask)
        self._stale = self.master_sharded

    def _state_dict_guard(self, module, prefix, keep_vars) -> None:
        if self._stale and self.master_sharded:
            raise RuntimeError("DataParallel: the fp32 master is sharded across ranks (bf16 weight wire, "
                               "HOPSX_P2P_WEIGHT_WIRE=bf16); call dp.sync_master() on EVERY rank (collective) "
                               "before state_dict() / export / save, or dp.close() at the end of training")

    def _cuts(self) -> list[int] | None:
        """Owner-piece boundaries of the fused step: the buckets when their reduce-scatters overlap the
        backward (rank r owns slice r of EVERY bucket, so every rank reduces a share of every bucket and
        the post-backward tail is 1/N of the last bucket), else None (one piece: slice r of the arena)."""
        if not getattr(self, "_rs_mode", False):
            return None
        return sorted({0, self.arena.numel} | {int(s) for s, _, _ in self.buckets} | {int(e) for _, e, _ in self.buckets})

    def owner_slices(self) -> list[list[slice]] | None:
        """Per rank, the slices whose optimizer state only that rank keeps current (fused mode: slice r of
        every owner piece, parallel.oneshot.owner_pieces), else None."""
        if self._fused_opt is None:
            return None
        from .oneshot import owner_pieces

        return owner_pieces(self.arena.numel, self.world, self._cuts())

    @property
    def master_sharded(self) -> bool:
        """ZeRO-1 wire (bf16 weight all-gather): the fp32 master is current only on each slice's
        owner between sync points; the bf16 compute weights are complete on every rank."""
        return self._fused_opt is not None and self._wmask is not None

    def sync_master(self) -> None:
        """Collective: make every rank's fp32 master complete (each slice from its owner).  Call on
        every rank before reading parameters on the host (export, evaluation on the CPU);
        checkpoint.save, verify_replicas and close do it themselves."""
        sl = self.owner_slices()
        if sl is None or not self.master_sharded:
            return
        _gather_slices(self.arena.master, sl, self._oneshot.rank)
        self._stale = False

    def gather_state(self) -> None:
        """Collective: make every rank's optimizer-state buffers (and, on the ZeRO-1 wire, the fp32
        master) complete, each slice from its owner; checkpoint.save calls this on every rank before
        rank 0 serialises."""
        sl = self.owner_slices()
        if sl is None:
            return
        self.sync_master()
        for t in self.arena.states.values():
            _gather_slices(t, sl, self._oneshot.rank)

    @property
    def p2p_world(self) -> int:
        """Ranks the P2P communicator spans (0: RCCL / process-group path)."""
        if getattr(self, "_closed", None) is not None:
            return self._closed[2]
        return 0 if self._oneshot is None else self._oneshot.world

    @property
    def wire_bytes_per_param(self) -> int | None:
        """Bytes per parameter per step in the exchange's wire format: fused step = gradient +
        weight formats (each GPU reads (N-1)/N of them over xGMI); all-reduce = 2 x the gradient
        format (reduce-scatter + all-gather halves of a ring / two-shot)."""
        if getattr(self, "_closed", None) is not None:
            return self._closed[1]
        if self.world <= 1:
            return None
        if self._fused_opt is not None:
            f = 0.0
            if self._wmask is not None:
                f = min(1.0, float(self._wmask.sum().item()) * 64 / max(1, self.arena.numel))
            return self._oneshot.wire_bytes_per_param(f)
        return 4 if self.grad_dtype == torch.bfloat16 and self._oneshot is None else 8

    # -------------------------------------------------------------- health
    def poll(self) -> None:
        """Every ``poll_every`` calls: asynchronous check of the P2P error flag (raises when a peer
        never arrived; the kernels skipped that reduction instead of summing stale buffers)."""
        if self._oneshot is None:
            return
        self._polls += 1
        if self._polls % max(1, self.poll_every) == 0:
            self._oneshot.poll()

    def verify_replicas(self) -> dict:
        """Collective consistency check (after the same steps on every rank): the fp32 master and the
        bf16 compute weights must be bit-identical on every rank, and the compute weights must be
        the bf16 rounding of the master (a torn or stale all-gather fails this even on the ZeRO-1
        wire, where the master is first reassembled from its owners).
        Returns {'identical': bool, 'max_abs_diff': float}."""
        self.sync_master()
        m = self.arena.master
        ref = m.clone()
        hdist.broadcast_(ref, 0)
        d = float((m - ref).abs().max().item()) if m.numel() else 0.0
        sh = self.arena.shadow
        if sh is not None and sh.numel():
            bits = sh.view(torch.int16).to(torch.int32)  # int32: every backend can broadcast it
            ref_bits = bits.clone()
            hdist.broadcast_(ref_bits, 0)
            if not torch.equal(bits, ref_bits):
                d = max(d, float((bits - ref_bits).abs().max().item()))
            mb = m.to(torch.bfloat16)
            if not torch.equal(sh, mb):
                d = max(d, float((sh.float() - mb.float()).abs().max().item()) or 1e-30)
        d = hdist.all_reduce_scalar(d, "max")
        return {"identical": d == 0.0, "max_abs_diff": d}

    @property
    def path(self) -> str:
        if getattr(self, "_closed", None) is not None:
            return self._closed[0]
        if self.world <= 1:
            return "none"
        if self._fused_opt is not None:
            return "p2p-xgmi-fused-step" + ("-zerocopy" if self.zero_copy else "") + ("-overlap" if self._rs_mode else "")
        if self._oneshot is not None:
            return "p2p-xgmi-allreduce"
        be = "rccl" if dist.get_backend() == "nccl" else dist.get_backend()
        return be + ("-bf16" if self.grad_dtype == torch.bfloat16 else "")

    def broadcast_params(self) -> None:
        hdist.broadcast_(self.arena.master, 0)
        self.arena.refresh_shadow()

    # -------------------------------------------------------------- backward
    def _launch(self, bi: int) -> None:
        if self._launched[bi]:
            return
        s, e, _ = self._launched_bucket(bi)
        view = self.arena.grad[s:e]
        if self._oneshot is not None and self._oneshot.fits(view):
            self._oneshot(view)  # stream-ordered: later kernels see the reduced bucket
        elif self.grad_dtype == torch.bfloat16:
            # compressed all-reduce: bf16 on the wire, fp32 master accumulate
            tmp = view.to(torch.bfloat16)
            h = dist.all_reduce(tmp, async_op=True)
            self._handles.append((h, view, tmp))
        else:
            self._handles.append((dist.all_reduce(view, async_op=True), None, None))
        self._launched[bi] = True

    def _launched_bucket(self, bi):
        return self.buckets[bi]

    def _on_ready(self, p) -> None:
        bi = self._owner.get(id(p))
        if bi is None:
            return
        self._pending[bi] -= 1
        if self._pending[bi] == 0:
            self._launch(bi)

    def finish(self) -> None:
        """Complete the gradient all-reduce (called after loss.backward())."""
        if self.world <= 1:
            return
        for bi in range(len(self.buckets)):
            if not self._launched[bi]:
                self._launch(bi)
        for h, view, tmp in self._handles:
            h.wait()
            if tmp is not None:
                view.copy_(tmp)
        self._handles.clear()
        self._pending = [len(ids) for _, _, ids in self.buckets]
        self._launched = [False] * len(self.buckets)

    def allreduce_all(self) -> None:
        """Non-overlapped path (used between captured graph segments)."""
        if self.world <= 1:
            return
        for s, e, _ in self.buckets:
            view = self.arena.grad[s:e]
            if self._oneshot is not None and self._oneshot.fits(view):
                self._oneshot(view)
            elif self.grad_dtype == torch.bfloat16:
                # bf16 on the wire (half the ring bytes), fp32 arena kept as the accumulator
                tmp = view.to(torch.bfloat16)
                dist.all_reduce(tmp)
                view.copy_(tmp)
            else:
                dist.all_reduce(view)

    def capturable(self) -> bool:
        """Every bucket goes through the one-shot kernel (no RCCL call), so the whole step,
        all-reduce included, can live in one hipGraph (runtime/step.py)."""
        return self._oneshot is not None and all(self._oneshot.fits(self.arena.grad[s:e]) for s, e, _ in self.buckets)

    def grad_scale(self) -> float:
        return 1.0 / self.world

    def close(self) -> None:
        """Collective.  Leaves the fp32 master complete on every rank; raises if a P2P collective
        failed since the last poll."""
        hooks.unsubscribe(self._on_ready)
        hooks.unsubscribe(self._on_ready_rs)  # (a zero-copy gradient stays where it is: this rank's own memory)
        if getattr(self, "_closed", None) is None:
            self._closed = (self.path, self.wire_bytes_per_param, self.p2p_world)  # reported after teardown
        if self._oneshot is not None:
            try:
                # a failed P2P collective (dead peer, sticky error) raises here, BEFORE the collective
                # master gather, which would otherwise block until the process-group timeout and copy
                # slices the failed kernels never wrote
                self._oneshot.check()
                self.sync_master()
            finally:
                self._oneshot.close()
                self._oneshot = None


def _gather_slices(t: torch.Tensor, slices: list, rank: int) -> None:
    """All-gather each rank's owner slices (a slice or a list of slices per rank) of a flat tensor in
    place (any backend)."""
    if not hdist.is_dist():
        return
    per = [s if isinstance(s, list) else [s] for s in slices]
    sizes = [sum(x.stop - x.start for x in ss) for ss in per]
    mx = max(sizes)
    buf = torch.zeros(mx, dtype=t.dtype, device=t.device)
    if sizes[rank]:
        buf[:sizes[rank]].copy_(torch.cat([t[x] for x in per[rank]]))
    parts = [torch.empty_like(buf) for _ in per]
    dist.all_gather(parts, buf)
    for ss, p in zip(per, parts):
        o = 0
        for x in ss:
            m = x.stop - x.start
            t[x].copy_(p[o:o + m])
            o += m
