"""P2P collectives over IPC-mapped peer buffers (``_hopsx_comm``, csrc/comm/oneshot.hip).

SURVEY §5.8 item 3 / §2.4: a ring all-reduce needs 2(N-1) latency-bound hops, but MI355X wires
every GPU to its 7 peers directly over xGMI.  Each rank stages its data in an IPC-shared buffer,
flags every peer, and reads the peers' buffers itself:

* one-shot all-reduce (small messages): every rank sums all N staging buffers;
* two-shot all-reduce (mid-size): reduce-scatter + all-gather, 2(N-1)/N of the bytes;
* ``dp_step``: the data-parallel step tail in ONE launch — reduce-scatter of the gradient, the
  fused optimizer on this rank's slice only, all-gather of the new weights, grad zeroing,
  step/RNG bookkeeping and the next-batch prefetch.  Wire formats (``HOPSX_P2P_GRAD_WIRE`` /
  ``HOPSX_P2P_WEIGHT_WIRE``): fp32 gradients + bf16 weights by default — ZeRO-1, 6 B per parameter
  per step instead of 8: the fp32 master and the optimizer moments of a slice are current only on
  its owner, the replicas share the bf16 compute weights bit-for-bit, and the engine gathers the
  owners' fp32 slices at sync points (``DataParallel.sync_master``; checkpoints, close).  bf16
  gradients (fp32 accumulation) bring it to 4 B.

Setup exchanges ``hipIpcMemHandle`` bytes through the default process group (any backend), so it
works for RCCL and gloo groups alike, then runs a self-test on every rank: known all-reduces in
both modes AND the fused dp_step of every optimizer kind the benches use, several rounds each (both
staging parities written, read and reused), checked against the single-rank optimizer kernel on
the summed gradient.  ``HOPSX_P2P_SELFTEST_FAIL=<rank>`` forces that rank's verdict to "fail"
(fault injection: every rank must then fall back to RCCL).  ``P2PComm.create`` returns None when any rank fails to map a peer or the self-test
disagrees — the caller then stays on RCCL.  Launches are hipGraph-capturable (device-resident
epochs).  A peer that never arrives makes the kernels set a sticky error flag and write nothing;
``poll()`` (cheap, asynchronous) and ``check()`` (synchronous) raise on it.

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


def mode() -> str:
    """``HOPSX_P2P``: ``auto`` (default: used when every rank shares one node and the self-test
    passes), ``1`` (required: setup failures raise), ``0`` (RCCL only).  ``HOPSX_ONESHOT_AR`` is the
    round-1 spelling of the same switch."""
    m = os.environ.get("HOPSX_P2P")
    if m is None:
        legacy = os.environ.get("HOPSX_ONESHOT_AR")
        m = {"1": "1", "0": "0"}.get(legacy or "", "auto")
    return m if m in ("auto", "1", "0") else "auto"


def enabled() -> bool:
    return mode() != "0"


def _timeout() -> float:
    """Seconds a P2P workgroup waits for a peer before it declares it lost (sticky error, every rank
    raises).  300 s by default: a rank-local phase (rank-0 evaluation, logging, a checkpoint write)
    must not read as a dead peer; RCCL's own watchdog is 30 min.  A job with longer rank-local
    phases raises ``HOPSX_P2P_TIMEOUT_S`` or puts a barrier before its next step."""
    return float(os.environ.get("HOPSX_P2P_TIMEOUT_S", "300"))


def _wire() -> tuple[bool, bool]:
    """(bf16 gradients, bf16 weights) on the fused step's wire."""
    g = os.environ.get("HOPSX_P2P_GRAD_WIRE", "fp32").lower() in ("bf16", "bfloat16")
    w = os.environ.get("HOPSX_P2P_WEIGHT_WIRE", "bf16").lower() in ("bf16", "bfloat16")
    return g, w


def _default_blocks(ranks_per_device: int) -> int:
    """One workgroup per CU at most (the flag protocol needs every block of every rank resident):
    256 on a GPU of its own.  Ranks that share one physical GPU (multi-rank rehearsal on a one-GPU
    box) split its 256 CUs.  ``ranks_per_device`` comes from the ranks' PCI ids (``_colocation``),
    not from the visible device count: the experiment launcher pins every worker to one device with
    HIP_VISIBLE_DEVICES, so each process sees one GPU even when the 8 workers drive 8 GPUs."""
    env = os.environ.get("HOPSX_P2P_BLOCKS")
    if env:
        return int(env)
    if ranks_per_device > 1:
        return max(8, min(64, 256 // (2 * ranks_per_device)))
    return 256


def device_id(dev) -> str:
    """Physical identity of a device: PCI domain:bus:device (+ uuid when the runtime reports one)."""
    p = torch.cuda.get_device_properties(dev)
    uid = str(getattr(p, "uuid", "") or "")
    return f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}/{uid}"


def _colocation(dev) -> int:
    """Collective: the largest number of ranks that drive the same physical GPU."""
    me = device_id(dev)
    if hdist.world_size() <= 1:
        return 1
    ids = [None] * hdist.world_size()
    dist.all_gather_object(ids, me)
    return max(ids.count(i) for i in ids)


class OneShotAllReduce:
    """Sum-all-reduce (and the fused DP step) of fp32 device tensors of up to ``cap_bytes`` across the
    default group.  The constructor raises on any setup failure (see ``P2PComm.create`` for the
    collective, fail-safe variant)."""

    def __init__(self, cap_bytes: int = 8 << 20, blocks: int | None = None, device=None, timeout: float | None = None):
        C = ext()
        self.rank, self.world = hdist.rank(), hdist.world_size()
        if self.world > C.MAX_RANKS:
            raise ValueError(f"P2P collectives support <= {C.MAX_RANKS} ranks (one node)")
        self.device = device or hdist.device()
        self.cap = (int(cap_bytes) // 4 + 3) & ~3
        self.ranks_per_device = _colocation(self.device) if self.device.type == "cuda" else 1
        self.blocks = max(1, min(int(blocks or _default_blocks(self.ranks_per_device)), C.MAX_BLOCKS))
        self.timeout = float(timeout or _timeout())
        self.grad_bf16, self.weight_bf16 = _wire()
        self._buf = self._flag = None
        self._opened: list[int] = []
        self._buf, hb = C.alloc(C.STAGING_FLOATS_PER_CAP * self.cap * 4, False)
        self._flag, hf = C.alloc(C.FLAG_ROWS * C.MAX_RANKS * C.MAX_BLOCKS * 4, True)
        hdist.register(self, hdist.ORDER_COMM)  # ordered teardown at shutdown / interpreter exit
        # two-shot (reduce-scatter + all-gather) above this size when N > 2: 2(N-1)/N * n of xGMI
        # reads per GPU instead of (N-1) * n
        self.two_shot_min = int(os.environ.get("HOPSX_TWOSHOT_MIN_KB", "256")) * 1024 // 4
        if self.world > 1:
            objs = [None] * self.world
            dist.all_gather_object(objs, (self.rank, bytes(hb), bytes(hf)))
            self._map(objs)
        else:
            self.bufs, self.flags = [self._buf], [self._flag]
        self.epochs = torch.zeros(C.MAX_BLOCKS, dtype=torch.int32, device=self.device)
        self.err = torch.zeros(1, dtype=torch.int32, device=self.device)
        self._err_host = torch.zeros(1, dtype=torch.int32).pin_memory() if self.device.type == "cuda" else None
        self._err_event = None
        hdist.barrier()

    def _map(self, objs) -> None:
        C = ext()
        bufs, flags = [0] * self.world, [0] * self.world
        for r, b, f in objs:
            if r == self.rank:
                bufs[r], flags[r] = self._buf, self._flag
            else:
                if b is None or f is None:
                    raise RuntimeError(f"rank {r} has no P2P staging buffer")
                bufs[r] = C.open(b)
                self._opened.append(bufs[r])
                flags[r] = C.open(f)
                self._opened.append(flags[r])
        self.bufs, self.flags = bufs, flags

    # ------------------------------------------------------------ collectives
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
                            (mode or self.mode(t.numel())) == "two_shot", self.timeout)
        return out

    # ------------------------------------------------------------ zero-copy gradients
    def make_grad_buffer(self, n: int) -> "torch.Tensor | None":
        """Collective, fail-safe: an fp32 [n] device tensor in IPC-shared memory, mapped by every peer,
        to be the arena gradient (``ParamArena.rebind_grad``).  The fused step then reads the peers'
        gradients in place instead of staging a copy (``zero_copy``).  None on every rank unless every
        rank allocated and mapped (each rank keeps its own memory either way)."""
        C = ext()
        t = h = None
        try:
            cap, ptr, h = C.alloc_tensor(int(n), self.device.index or 0)
            t = torch.from_dlpack(cap)
            h = bytes(h)
        except Exception:  # noqa: BLE001 - every failure falls back to the staged copy
            t = h = None
        objs = [(self.rank, h)]
        if self.world > 1:
            objs = [None] * self.world
            dist.all_gather_object(objs, (self.rank, h))
        gp, opened = [0] * self.world, []
        ok = t is not None and all(o[1] is not None for o in objs)
        if ok:
            try:
                for r, hb in objs:
                    if r == self.rank:
                        gp[r] = t.data_ptr()
                    else:
                        gp[r] = C.open(hb)
                        opened.append(gp[r])
            except Exception:  # noqa: BLE001
                ok = False
        if not _agree(ok):
            for q in opened:
                C.close(q)
            return None
        self._opened += opened
        self.gpeers = gp
        self.zc_grad = t
        return t

    @property
    def zero_copy(self) -> bool:
        return bool(getattr(self, "gpeers", None)) and not self.grad_bf16

    def dp_rs(self, grad: torch.Tensor, lo: int, hi: int, blocks: int, stream) -> None:
        """Per-bucket reduce-scatter (zero-copy fp32 gradients): sum every rank's gradient over
        [lo, hi) ∩ this rank's owner slice into ``grad`` in place, on ``stream``.  Every rank must issue
        the same sequence of buckets with the same ``blocks``."""
        ext().dp_rs(grad.data_ptr(), grad.numel(), int(lo), int(hi), self.cap, self.rank, self.world, self.bufs,
                    self.flags, self.gpeers, self.epochs.data_ptr(), self.err.data_ptr(), int(blocks),
                    stream.cuda_stream, self.timeout)

    def dp_step(self, opt, wmask: torch.Tensor | None = None, pre_reduced: bool = False,
                cuts: list[int] | None = None) -> None:
        """Reduce-scatter the arena gradient, run ``opt``'s update on this rank's slice, all-gather the
        new weights; one launch (see the module docstring).  ``opt`` must own the whole arena.
        ``wmask`` (arena.wire_mask()): chunks whose weights travel in bf16 (ZeRO-1).  When the arena
        gradient is this comm's zero-copy buffer the peers' gradients are read in place (no staging
        copy); ``pre_reduced``: dp_rs already summed this rank's slice (per-bucket overlap).  ``cuts``: the
        owner pieces' boundaries 0 = c_0 < ... < c_K = numel (the per-bucket reduce-scatter's buckets: rank r
        owns slice r of every piece, see ``owner_pieces``); None: one piece."""
        from ..ops._C import OPTIM

        a = opt.arena
        if a.numel > self.cap:
            raise ValueError(f"arena of {a.numel} elements exceeds the P2P staging capacity {self.cap}")
        opt.sync_hp()
        st = [t.data_ptr() for t in opt._states] + [0] * (3 - len(opt._states))
        srcs, dsts, nbytes, cur, nb = [], [], [], 0, 0
        if opt.prefetch is not None:
            pairs, cursor = opt.prefetch
            for src, dst in pairs:
                srcs.append(src.data_ptr())
                dsts.append(dst.data_ptr())
                nbytes.append(dst.numel() * dst.element_size())
                nb = src.shape[0]
            cur = cursor.data_ptr()
        ext().dp_step(OPTIM[opt.kind], a.master.data_ptr(), a.grad.data_ptr(), st[0], st[1], st[2],
                      a.shadow.data_ptr(), a.numel, [float(v) for v in opt._hp()], opt._hp_dev.data_ptr(),
                      opt.step_count.data_ptr(), opt._arrive.data_ptr(),
                      opt.rng.data_ptr() if opt.rng is not None else 0, srcs, dsts, nbytes, cur, nb, self.cap,
                      self.rank, self.world, self.bufs, self.flags, self.epochs.data_ptr(), self.err.data_ptr(),
                      self.blocks, torch.cuda.current_stream(self.device).cuda_stream, self.timeout,
                      self.grad_bf16, wmask.data_ptr() if (wmask is not None and self.weight_bf16) else 0,
                      self._zc_peers(a.grad), bool(pre_reduced), [int(c) for c in (cuts or [])])

    def _zc_peers(self, grad: torch.Tensor) -> list:
        zg = getattr(self, "zc_grad", None)
        if self.zero_copy and zg is not None and grad.data_ptr() == zg.data_ptr():
            return list(self.gpeers)
        return []

    def wire_bytes_per_param(self, bf16_fraction: float = 1.0) -> float:
        """Bytes per parameter per step of the fused step's wire (each GPU reads (N-1)/N of them);
        ``bf16_fraction``: share of the parameters on the bf16 weight wire."""
        f = bf16_fraction if self.weight_bf16 else 0.0
        return round((2 if self.grad_bf16 else 4) + 2 * f + 4 * (1 - f), 2)

    # ------------------------------------------------------------ failure detection
    def check(self) -> None:
        """Raise if a peer failed to arrive within the spin bound (synchronises the device)."""
        e = int(self.err.item())
        if e:
            raise RuntimeError(f"P2P collective: rank {e - 1} never raised its flag within {self.timeout:g} s "
                               "(peer lost or stalled); the reduction was skipped, not applied")

    def poll(self) -> None:
        """Asynchronous check: read the result of the previous poll's device->host copy (if it has
        landed) and enqueue a new one.  Costs one 4-byte copy on the stream; raises like check()."""
        if self._err_host is None:
            return self.check()
        ev = self._err_event
        if ev is not None and ev.query():
            e = int(self._err_host[0])
            if e:
                raise RuntimeError(f"P2P collective: rank {e - 1} never raised its flag within {self.timeout:g} s "
                                   "(peer lost or stalled); the reduction was skipped, not applied")
            ev = None
        if ev is None:
            self._err_host.copy_(self.err, non_blocking=True)
            self._err_event = torch.cuda.Event()
            self._err_event.record(torch.cuda.current_stream(self.device))

    def close(self) -> None:
        """Collective: every rank must call it (no peer may still read our staging buffer)."""
        if self._buf is None:
            return
        torch.cuda.synchronize(self.device)
        hdist.barrier()
        self._release()

    def release_local(self) -> None:
        """Interpreter-exit teardown (no collectives): unmap the peers' buffers, free ours."""
        self._release()

    def _release(self) -> None:
        """Local teardown (the caller has synchronised the ranks)."""
        C = ext()
        for p in self._opened:
            C.close(p)
        if self._buf is not None:
            C.free(self._buf)
        if self._flag is not None:
            C.free(self._flag)
        self._buf = self._flag = None
        self._opened = []


def _agree(ok: bool) -> bool:
    """Every rank's verdict, combined (min) over the default group."""
    if hdist.world_size() <= 1:
        return ok
    return hdist.all_reduce_scalar(1.0 if ok else 0.0, "min") > 0.5


# optimizer kinds the dp_step self-test covers (everything the benches and examples train with)
SELFTEST_KINDS = ("sgd", "adam", "adadelta", "rmsprop")


def owner_pieces(n: int, world: int, cuts: list[int] | None = None) -> list[list[slice]]:
    """Per rank, the slices of a length-``n`` arena whose update that rank owns in the fused step
    (csrc/comm/oneshot.hip PieceSlices): the arena is cut at ``cuts`` (0 .. n; None: one piece) and rank r
    owns slice r — ceil(len / world) rounded up to 4 — of every piece."""
    cuts = list(cuts) if cuts else [0, n]
    out: list[list[slice]] = [[] for _ in range(world)]
    for p0, p1 in zip(cuts[:-1], cuts[1:]):
        L = ((p1 - p0 + world - 1) // world + 3) & ~3
        for r in range(world):
            lo, hi = min(p1, p0 + r * L), min(p1, p0 + (r + 1) * L)
            if hi > lo:
                out[r].append(slice(lo, hi))
    return out


def _dp_selftest_hp(kind: str, world: int) -> list[float]:
    return {"sgd": [0.5, 1.0 / world, 0.0, 0.9, 0.0, 0.0], "adam": [1e-2, 1.0 / world, 0.0, 0.9, 0.999, 1e-8],
            "adadelta": [1.0, 1.0 / world, 0.0, 0.95, 1e-7], "rmsprop": [1e-2, 1.0 / world, 0.0, 0.9, 1e-7, 0.0, 0.0]}[kind]


def dp_self_test(comm: "OneShotAllReduce", kinds=SELFTEST_KINDS, rounds: int = 3) -> bool:
    """The fused dp_step on a synthetic arena, every optimizer kind, ``rounds`` steps each (both
    staging parities, reused): this rank's owner slice of the fp32 master and the whole bf16
    shadow must match the single-rank optimizer kernel run on the exactly-summed gradient, and
    the shadows must agree across ranks bit-for-bit.  Gradients are small integers, exact in fp32
    and bf16 in any summation order, so only stale or torn peer data can fail the test."""
    from ..ops import kernels as K
    from ..ops._C import OPTIM

    C = ext()
    dev, W, r = comm.device, comm.world, comm.rank
    n = min(comm.cap, 8192 * W + 20)
    n -= n % 4
    idx = torch.arange(n, device=dev, dtype=torch.float32)
    # two owner pieces (every rank owns a slice of each: the per-bucket layout), the same in every round —
    # on the bf16 weight wire only the owner's fp32 master and optimizer state are current, so ownership
    # must not move between steps; the per-bucket rounds reduce-scatter exactly these two buckets
    half = (n // 2) & ~63
    cuts = [0, half, n]
    own = torch.zeros(n, dtype=torch.bool, device=dev)
    for s in owner_pieces(n, W, cuts)[r]:
        own[s] = True
    st = torch.cuda.current_stream(dev).cuda_stream
    # weight wire: every other 64-element chunk in bf16 (both formats cross every slice boundary)
    chunks = -(-n // C.WIRE_CHUNK)
    wmask = (torch.arange(chunks, device=dev) % 2).to(torch.uint8) if comm.weight_bf16 else None
    f32 = torch.ones(n, dtype=torch.bool, device=dev)
    if wmask is not None:
        f32 = (wmask == 0).repeat_interleave(C.WIRE_CHUNK)[:n]
    # the zero-copy gradient buffer of the comm (make_grad_buffer), when it has one
    zg = comm.zc_grad if comm.zero_copy and getattr(comm, "zc_grad", None) is not None else None
    if zg is not None and zg.numel() < n:
        zg = None
    if zg is not None:
        saved = zg[:n].clone()
    for kind in kinds:
        k = OPTIM[kind]
        hp = _dp_selftest_hp(kind, W)
        hp_dev = torch.tensor((hp + [0.0] * 8)[:8], device=dev)
        master = (idx % 13) * 0.25 - 1.5
        ref_m = master.clone()
        states = [torch.zeros(n, device=dev) for _ in range(3)]
        ref_s = [torch.zeros(n, device=dev) for _ in range(3)]
        shadow = torch.zeros(n, dtype=torch.bfloat16, device=dev)
        ref_sh = torch.zeros(n, dtype=torch.bfloat16, device=dev)
        step, ref_step = torch.zeros(1, device=dev), torch.zeros(1, device=dev)
        arrive = torch.zeros(9 * 32, dtype=torch.int32, device=dev)
        ref_arrive = torch.zeros(9 * 32, dtype=torch.int32, device=dev)
        for it in range(rounds):
            grad = ((idx * (it + 3)) % 23) - 11.0 + r
            gsum = sum(((idx * (it + 3)) % 23) - 11.0 + q for q in range(W))
            # rounds alternate the gradient paths: staged copy, zero-copy (peers read in place), and
            # zero-copy with two per-bucket reduce-scatters ahead of a pre-reduced tail
            zmode = it % 3 if zg is not None else 0
            if zmode:
                zg[:n].copy_(grad)
                grad = zg[:n]
            if zmode == 2:
                for lo, hi in ((half, n), (0, half)):
                    C.dp_rs(grad.data_ptr(), n, lo, hi, comm.cap, r, W, comm.bufs, comm.flags, comm.gpeers,
                            comm.epochs.data_ptr(), comm.err.data_ptr(), min(comm.blocks, 16), st, comm.timeout)
            C.dp_step(k, master.data_ptr(), grad.data_ptr(), states[0].data_ptr(), states[1].data_ptr(),
                      states[2].data_ptr(), shadow.data_ptr(), n, hp, hp_dev.data_ptr(), step.data_ptr(),
                      arrive.data_ptr(), 0, [], [], [], 0, 0, comm.cap, r, W, comm.bufs, comm.flags,
                      comm.epochs.data_ptr(), comm.err.data_ptr(), comm.blocks, st, comm.timeout,
                      comm.grad_bf16, 0 if wmask is None else wmask.data_ptr(),
                      list(comm.gpeers) if zmode else [], zmode == 2, cuts)
            K.optim_step(k, ref_m, gsum, ref_s[0], ref_s[1], ref_s[2], ref_sh, hp, ref_step, zero_grad=True,
                         arrive=ref_arrive, hp_dev=hp_dev)
            torch.cuda.synchronize(dev)
            if int(comm.err.item()) != 0 or bool(grad.abs().max().item() != 0.0):
                return False
            tol = 1e-5 * (1.0 + ref_m.abs())
            if not bool(((master[own] - ref_m[own]).abs() <= tol[own]).all().item()):
                return False
            if not bool(((master - ref_m).abs() <= tol)[f32].all().item()):
                return False  # fp32-wire chunks: every rank holds the owners' fp32 master
            # the gathered bf16 weights: each owner's rounding of its fp32 result (1 bf16 ulp slack
            # against the reference kernel's own rounding)
            d = (shadow.float() - ref_sh.float()).abs()
            if not bool((d <= ref_sh.float().abs() * 2.0 ** -7 + 1e-6).all().item()):
                return False
            if float(step.item()) != float(it + 1):
                return False
        if W > 1:
            sh = shadow.view(torch.int32).clone()  # n % 4 == 0: bf16 pairs as int32 (any backend)
            ref = sh.clone()
            hdist.broadcast_(ref, 0)
            if not torch.equal(sh, ref):
                return False
    if zg is not None:
        zg[:n].copy_(saved)  # the live arena gradient (zero at rest) as it was
        torch.cuda.synchronize(dev)
    return True


def self_test(comm: OneShotAllReduce, rounds: int = 3) -> bool:
    """Known all-reduces in both modes, checked exactly on this rank (integer-valued floats: every
    summation order gives the same result).  Several rounds with changing values, so both staging
    parities are written, read, and REUSED — a peer that saw a stale cached copy of an earlier
    epoch (a missing write-back or invalidate over xGMI) fails the test."""
    dev = comm.device
    n = min(comm.cap, 4096 * comm.world + 12)
    idx = torch.arange(n, device=dev, dtype=torch.float32)
    for it in range(rounds):
        want = sum(((idx * (it + 1)) % 97) + r + 1 for r in range(comm.world))
        for mode in ("one_shot", "two_shot"):
            x = ((idx * (it + 1)) % 97) + comm.rank + 1
            comm(x, mode=mode)
            torch.cuda.synchronize(dev)
            if int(comm.err.item()) != 0 or not torch.equal(x, want):
                return False
    if os.environ.get("HOPSX_P2P_SELFTEST_DP", "1") == "1" and not dp_self_test(comm, rounds=rounds):
        return False
    forced = os.environ.get("HOPSX_P2P_SELFTEST_FAIL")
    if forced is not None and forced.strip() in (str(comm.rank), "all"):
        return False  # fault injection: this rank reports a failed self-test
    return True


class P2PComm:
    @staticmethod
    def create(cap_bytes: int, device=None, required: bool | None = None) -> OneShotAllReduce | None:
        """Collective, fail-safe setup: every rank allocates, exchanges handles, maps its peers and runs
        the self-test; unless ALL ranks succeed everyone gets None (or RuntimeError if required)."""
        required = mode() == "1" if required is None else required
        world = hdist.world_size()
        if world <= 1 or world > ext().MAX_RANKS:
            if required and world > 1:
                raise RuntimeError(f"P2P collectives need 2..{ext().MAX_RANKS} ranks on one node")
            return None
        lw = int(os.environ.get("LOCAL_WORLD_SIZE", world))
        if lw != world:  # ranks on other nodes are not IPC-reachable
            if required:
                raise RuntimeError("P2P collectives need every rank on one node")
            return None
        comm = _create_local(cap_bytes, device)  # never raises after joining the handle exchange
        why = repr(comm._setup_err) if comm._setup_err is not None else ""
        ok = _agree(comm._setup_err is None)
        if ok:
            try:
                ok = self_test(comm)
            except Exception as e:  # noqa: BLE001 - every failure falls back to RCCL
                ok, why = False, repr(e)
            ok = _agree(ok)
        if not ok:
            # every rank reaches this point: drain, meet, then tear down locally
            try:
                torch.cuda.synchronize(comm.device)
            except Exception:  # noqa: BLE001
                pass
            hdist.barrier()
            try:
                comm._release()
            except Exception:  # noqa: BLE001
                pass
            if required:
                raise RuntimeError(f"P2P collectives unavailable on rank {hdist.rank()}: {why or 'self-test failed'}")
            return None
        return comm


def _create_local(cap_bytes: int, device) -> OneShotAllReduce:
    """OneShotAllReduce whose setup tolerates a failing rank: it sends None handles, every rank still
    joins the exchange, and the failure is recorded in ``_setup_err`` instead of raised."""
    C = ext()
    comm = OneShotAllReduce.__new__(OneShotAllReduce)
    comm.rank, comm.world = hdist.rank(), hdist.world_size()
    comm.device = device or hdist.device()
    comm.cap = (int(cap_bytes) // 4 + 3) & ~3
    comm.ranks_per_device = _colocation(comm.device)
    comm.blocks = max(1, min(_default_blocks(comm.ranks_per_device), C.MAX_BLOCKS))
    comm.timeout = _timeout()
    comm.grad_bf16, comm.weight_bf16 = _wire()
    comm.two_shot_min = int(os.environ.get("HOPSX_TWOSHOT_MIN_KB", "256")) * 1024 // 4
    comm._buf = comm._flag = None
    comm._opened = []
    err = None
    hb = hf = None
    try:
        comm._buf, hb = C.alloc(C.STAGING_FLOATS_PER_CAP * comm.cap * 4, False)
        comm._flag, hf = C.alloc(C.FLAG_ROWS * C.MAX_RANKS * C.MAX_BLOCKS * 4, True)
        hb, hf = bytes(hb), bytes(hf)
    except Exception as e:  # noqa: BLE001
        err, hb, hf = e, None, None
    objs = [None] * comm.world
    dist.all_gather_object(objs, (comm.rank, hb, hf))
    comm._setup_err = err
    if err is None:
        try:
            comm._map(objs)
            comm.epochs = torch.zeros(C.MAX_BLOCKS, dtype=torch.int32, device=comm.device)
            comm.err = torch.zeros(1, dtype=torch.int32, device=comm.device)
            comm._err_host = torch.zeros(1, dtype=torch.int32).pin_memory()
            comm._err_event = None
        except Exception as e:  # noqa: BLE001
            comm._setup_err = e
    return comm
