"""Chicago-taxi wide & deep classifier ("big tipper": tips > 20% of the fare).

The reference README names a TFX Chicago-taxi pipeline (README.md:99-112) whose
notebooks are absent from the repo, so the model follows the public
TFX taxi trainer it points to:

* dense (DNN) inputs: trip_miles, fare, trip_seconds — z-scored by the Transform stage;
* wide (linear) inputs: 13 identity-categorical columns —
  4 bucketized lat/long columns (10 buckets each), 2 vocabulary columns
  (payment_type, company: 1000 vocab + 10 OOV buckets) and 7 categorical columns
  (trip_start_hour 24, trip_start_day 31, trip_start_month 12, pickup/dropoff census
  tract 2000, pickup/dropoff community area 80) — 6,287 one-hot slots in total;
* DNN hidden units [100, 70, 48, 34] (first_dnn_layer_size=100, num_dnn_layers=4,
  dnn_decay_factor=0.7), logits = wide + deep, sigmoid cross-entropy;
* optimizers as tf.estimator.DNNLinearCombinedClassifier: FTRL (lr 0.2) on the wide
  part, Adagrad (lr 0.05, accumulator 0.1) on the deep part; train batch 40.

MI355X mapping: the wide part is a fixed-length embedding-bag (13 rows of a
[6287, 1] table per example, thread-per-bag gather / atomic scatter-add kernel);
the deep part runs on the MFMA linear kernels with fused bias+ReLU epilogues; the
two optimizers are single fused kernels over two slices of ONE parameter arena
(so data parallelism all-reduces one flat buffer); the whole step is one hipGraph.
"""
from __future__ import annotations

import math
import os

import numpy as np
import torch

from ..runtime.capture import graph as _capture_graph
from torch import nn

from .. import nn as hnn
from ..ops import functional as HF

DENSE_FLOAT_FEATURE_KEYS = ["trip_miles", "fare", "trip_seconds"]
BUCKET_FEATURE_KEYS = ["pickup_latitude", "pickup_longitude", "dropoff_latitude", "dropoff_longitude"]
FEATURE_BUCKET_COUNT = 10
VOCAB_FEATURE_KEYS = ["payment_type", "company"]
VOCAB_SIZE, OOV_SIZE = 1000, 10
CATEGORICAL_FEATURE_KEYS = ["trip_start_hour", "trip_start_day", "trip_start_month", "pickup_census_tract",
                            "dropoff_census_tract", "pickup_community_area", "dropoff_community_area"]
MAX_CATEGORICAL_FEATURE_VALUES = [24, 31, 12, 2000, 2000, 80, 80]
LABEL_KEY = "tips"
TRAIN_BATCH_SIZE = 40


def hidden_units(first: int = 100, num_layers: int = 4, decay: float = 0.7) -> list[int]:
    return [max(2, int(first * decay ** i)) for i in range(num_layers)]


def wide_cardinalities() -> list[int]:
    return ([FEATURE_BUCKET_COUNT] * len(BUCKET_FEATURE_KEYS) + [VOCAB_SIZE + OOV_SIZE] * len(VOCAB_FEATURE_KEYS)
            + list(MAX_CATEGORICAL_FEATURE_VALUES))


def wide_offsets() -> np.ndarray:
    c = wide_cardinalities()
    return np.concatenate([[0], np.cumsum(c)[:-1]]).astype(np.int64)


WIDE_ROWS = int(sum(wide_cardinalities()))  # 6287
N_WIDE = len(wide_cardinalities())  # 13


class TaxiWideDeep(nn.Module):
    def __init__(self, hidden=None):
        super().__init__()
        hidden = hidden or hidden_units()
        # wide part first, deep part second: each is one contiguous slice of the arena
        self.wide = nn.Module()
        self.wide.weight = nn.Parameter(torch.zeros(WIDE_ROWS, 1))  # linear model init = 0 (tf.estimator)
        layers, d = [], len(DENSE_FLOAT_FEATURE_KEYS)
        for h in hidden:
            layers.append(hnn.Linear(d, h, activation="relu"))
            d = h
        layers.append(hnn.Linear(d, 1, out_f32=True))
        self.deep = nn.Sequential(*layers)

    def forward(self, dense, cat):
        """dense: [B, 3] z-scored floats; cat: [B, 13] int64 ids, already offset into the
        concatenated one-hot space (see ``wide_offsets``). Returns fp32 logits [B, 1]."""
        deep = self.deep(dense if not dense.is_cuda else HF.to_compute(dense))
        wide = HF.embedding_bag(cat, self.wide.weight)
        return deep.float() + wide


def make_optimizer(model: TaxiWideDeep, ftrl_lr: float = 0.2, adagrad_lr: float = 0.05):
    from .. import optim

    return optim.Chain(optim.Ftrl(model.wide, lr=min(ftrl_lr, 1.0 / math.sqrt(N_WIDE))),
                       optim.Adagrad(model.deep, lr=adagrad_lr, initial_accumulator_value=0.1))


class TaxiExchange:
    """The cross-rank exchange of the data-parallel v2 taxi step (csrc/ops/taxi_step.hip, DP
    instantiation): this rank's uncached exchange buffer and flag page, every peer's mapped through IPC
    handles exchanged over the default process group (ranks on one node; they may share a GPU — the step
    is one workgroup), the global step counter (exchange epoch base) and a sticky error word.

    Each rank's kernel pushes its dW accumulators and wide-row gradients into every rank's buffer, raises
    its flag word in every peer's page and sums the W ranks' gradients in rank order before the update:
    one cross-rank hop per step and bit-identical replicas, the MirroredStrategy global-batch step of the
    reference's TFX trainer (README.md:99-112) at 2..8 GPUs.  ``loopback=W``: ONE process plays W ranks
    (the peers' buffers are its own), for tests."""

    def __init__(self, device, world: int | None = None, loopback: int = 0, timeout_s: float | None = None):
        import torch.distributed as dist

        from ..ops import _C
        from ..parallel import dist as hdist
        from ..parallel import oneshot

        self.device = torch.device(device)
        xb, xf, xmax, self.pay = _C.ext().taxi_step2_xgeom()
        self.loopback = int(loopback)
        if self.loopback > 1:
            self.world, self.rank = self.loopback, 0
        else:
            self.world = int(world) if world is not None else hdist.world_size()
            self.rank = hdist.rank() if self.world > 1 else 0
        if not 2 <= self.world <= xmax:
            raise ValueError(f"the data-parallel taxi step takes 2..{xmax} ranks")
        self.timeout_ms = int(1000 * float(timeout_s or os.environ.get("HOPSX_TAXI_DP_TIMEOUT_S", "60")))
        C = oneshot.ext()
        self._owned, self._opened = [], []
        err = None
        try:
            buf, hb = C.alloc(int(xb), True)
            self._owned.append(buf)
            flg, hf = C.alloc(int(xf) * 4, True)
            self._owned.append(flg)
        except Exception as e:  # every rank must learn of it before the handle exchange
            err, hb, hf = repr(e), None, None
        self.xstep = torch.zeros(1, device=self.device, dtype=torch.int64)
        self.err = torch.zeros(4, device=self.device, dtype=torch.int32)
        if self.loopback > 1:
            if err:
                raise RuntimeError(f"taxi DP exchange setup failed: {err}")
            self.bufs, self.flags = [buf] * self.world, [flg] * self.world
            return
        objs = [None] * self.world
        dist.all_gather_object(objs, (self.rank, None if err else bytes(hb), None if err else bytes(hf), err))
        bad = [(o[0], o[3]) for o in objs if o[3]]
        if bad:
            self.close()
            raise RuntimeError(f"taxi DP exchange setup failed on ranks {bad}")
        self.bufs, self.flags = [0] * self.world, [0] * self.world
        try:
            for r, b, f, _ in objs:
                if r == self.rank:
                    self.bufs[r], self.flags[r] = buf, flg
                else:
                    self.bufs[r] = C.open(b)
                    self._opened.append(self.bufs[r])
                    self.flags[r] = C.open(f)
                    self._opened.append(self.flags[r])
        except Exception as e:
            err = repr(e)
        oks = [None] * self.world
        dist.all_gather_object(oks, err)
        if any(oks):
            self.close()
            raise RuntimeError(f"taxi DP: mapping a peer's exchange buffer failed: {oks}")

    def ptrs(self) -> list[int]:
        """The kernel's data-parallel pointer tail (taxi_step.hip hopsx_taxi_step2)."""
        mode = self.world | (self.rank << 8) | ((1 if self.loopback > 1 else 0) << 16)
        return [mode, self.timeout_ms, self.err.data_ptr(), self.xstep.data_ptr()] + list(self.bufs) + list(self.flags)

    def sync_replicas(self, arena) -> None:
        """Collective: every replica starts from rank 0's parameters and optimizer state."""
        import torch.distributed as dist

        if self.loopback > 1:
            return
        gloo = dist.get_backend() == "gloo"  # (rehearsals: ranks sharing a GPU; gloo broadcasts host copies)
        for t in [arena.master] + [arena.state(k) for k in ("adagrad_s0", "ftrl_s0", "ftrl_s1")]:
            if gloo:
                h = t.cpu()
                dist.broadcast(h, 0)
                t.copy_(h)
            else:
                dist.broadcast(t, 0)
        if arena.shadow is not None:
            arena.shadow.copy_(arena.master.to(arena.shadow.dtype))
        torch.cuda.synchronize(self.device)
        dist.barrier()

    def check(self) -> None:
        e = int(self.err[0].item()) & 0xFFFFFFFF
        if e:
            raise RuntimeError(f"taxi DP: a peer's gradients did not arrive within {self.timeout_ms} ms "
                               f"(step {e & 0xFFFFFF} of its launch); the replicas' state is partial")

    def close(self) -> None:
        if not self._owned:
            return
        from ..parallel import oneshot

        C = oneshot.ext()
        torch.cuda.synchronize(self.device)
        for q in self._opened:
            C.close(q)
        for q in self._owned:
            C.free(q)
        self._opened, self._owned = [], []


class FusedWideDeepStep:
    """The whole taxi training step as ONE kernel launch (csrc/ops/widedeep_step.hip): forward,
    sigmoid cross-entropy, backward, FTRL (wide) + Adagrad (deep) updates, step counters and the
    batch cursor of an HBM-resident epoch — one workgroup holding the model and the batch in LDS.

    Same model, optimizers and results as ``TrainStep(model, make_optimizer(model), "bce_logits")``
    (fp32 GEMMs instead of bf16).  Data-parallel, two forms: ``xdp`` (a :class:`TaxiExchange`) runs the
    v2 kernel's data-parallel instantiation — the replicas exchange gradients inside the launch and
    update in registers, "fused-v2-dp"; ``dp`` (a DataParallel engine): the v1 kernel stops at the
    gradients, which are all-reduced and applied by the regular optimizer kernels.  ``ok()`` says whether
    the model/batch fit one workgroup's LDS; otherwise use TrainStep."""

    def __init__(self, model: TaxiWideDeep, optimizer, dp=None, xdp: "TaxiExchange | None" = None):
        from ..runtime.arena import ParamArena  # noqa: F401 (the model must live in an arena)

        self.model, self.opt, self.dp, self.xdp = model, optimizer, dp, xdp
        if dp is not None and xdp is not None:
            raise ValueError("dp (v1 + all-reduce) and xdp (in-kernel exchange) are exclusive")
        self.arena = model.wide.weight._hx_arena
        self.ftrl, self.ada = optimizer.opts
        lins = [m for m in model.deep if isinstance(m, hnn.Linear)]
        self.lins = lins
        self.dims = [lins[0].weight.shape[1]] + [m.weight.shape[0] for m in lins]
        self.acts_ok = (all(m.activation == "relu" for m in lins[:-1]) and lins[-1].activation is None
                        and all(m.bias is not None for m in lins))
        if dp is not None:
            optimizer.grad_scale = dp.grad_scale()
        self._graph = None
        self._key = None
        self._graphU = None
        self._keyU = None
        self._graphR: dict = {}  # remainder graphs (Keras steps_per_execution tail): U -> graph
        # steps per replayed graph; on one GPU they run inside ONE launch (widedeep_step.hip nsteps)
        self.steps_per_execution = max(1, int(os.environ.get("HOPSX_TAXI_STEPS_PER_EXEC",
                                                             os.environ.get("HOPSX_STEPS_PER_EXEC", "32"))))
        self._slot_cache = {}
        self._n = 0
        self._B = None
        self._v2: dict = {}
        self._zn = None
        self._v2slots = {}  # cached v2 launch arguments: key -> C++ slot (_v2_slot)
        dev = self.arena.device
        self.loss = torch.zeros(1, device=dev)
        self.correct = torch.zeros(1, device=dev, dtype=torch.int32)
        self.cursor = torch.zeros(1, device=dev, dtype=torch.int64)
        # HOPSX_PHASE_DBG=1: the kernel stamps its phase boundaries here (tools/taxi_phases.py)
        self.dbg = (torch.zeros(32, device=dev, dtype=torch.int64)
                    if os.environ.get("HOPSX_PHASE_DBG") == "1" else None)

    def _ints(self, B: int, nbatch: int, nsteps: int = 1) -> list[int]:
        L = len(self.lins)
        iv = ([L, B, nbatch, N_WIDE, int(self.model.wide.weight._hx_off), int(self.dp is None), 2] + self.dims
              + [int(m.weight._hx_off) for m in self.lins] + [int(m.bias._hx_off) for m in self.lins])
        return iv + [int(nsteps)] if nsteps > 1 else iv

    def ok(self, B: int) -> bool:
        from ..ops import _C

        dev = self.arena.device
        if self.xdp is not None:  # the in-kernel exchange exists in the v2 kernel only
            return dev.type == "cuda" and self.v2(B)
        return (dev.type == "cuda" and self.acts_ok and self.dims[-1] == 1
                and (self.v2(B) or _C.ext().widedeep_step_lds(self._ints(B, 1)) > 0))

    def check(self) -> None:
        """Raise if the data-parallel exchange of any launch failed (sticky device error word)."""
        if self.xdp is not None:
            self.xdp.check()

    def digest(self) -> tuple[float, int]:
        """(sum, integer bit-sum) of the fp32 arena: equal on every replica iff the replicas agree."""
        m = self.arena.master
        return float(m.double().sum()), int(m.view(torch.int32).long().sum())

    def v2(self, B: int) -> bool:
        """The v2 kernel (csrc/ops/taxi_step.hip: bf16 MFMA, wide table + optimizer state on chip) takes
        the default taxi shape on one GPU; HOPSX_TAXI_KERNEL=v1 forces the fp32 v1 kernel."""
        from ..ops import _C

        key = (B, self.dp is None, os.environ.get("HOPSX_TAXI_KERNEL", "v2"), self.xdp is not None)
        r = self._v2.get(key)
        if r is None:
            r = (self.dp is None and key[2] != "v1" and self.acts_ok and self.arena.device.type == "cuda"
                 and _C.ext().taxi_step2_ok(self._ints(B, 1), int(self.model.wide.weight.shape[0])) > 0)
            self._v2[key] = r
        return r

    @property
    def kernel(self) -> str:
        k = "v2" if self.v2(self._B or TRAIN_BATCH_SIZE) else "v1"
        return k + "-dp" if self.xdp is not None and k == "v2" else k

    def _slots(self, B: int):
        """Host-built table: LDS slot of every deep arena element for batch size B (cached)."""
        from ..ops import _C
        from ..ops.kernels import check

        t = self._slot_cache.get(B)
        if t is None:
            lo = int(self.lins[0].weight._hx_off)
            hi = int(self.lins[-1].bias._hx_off) + self.dims[-1]
            host = torch.empty(hi - lo, dtype=torch.int32)
            check(_C.ext().widedeep_slots(self._ints(B, 1), host.data_ptr(), hi - lo), "widedeep_slots")
            t = host.to(self.arena.device)
            self._slot_cache[B] = t
        return t

    def _floats(self) -> list[float]:
        def pad8(v):
            return [float(x) for x in v] + [0.0] * (8 - len(v))

        self.ada.lr = self.ada.param_groups[0]["lr"]
        self.ftrl.lr = self.ftrl.param_groups[0]["lr"]
        return pad8(self.ada._hp()) + pad8(self.ftrl._hp())

    def _v2_slot(self, dense, cat, label, nbatch: int, cursor, nsteps: int) -> int:
        """The C++-side argument slot of this v2 launch shape, built once per key (the data, the step count,
        the hyper-parameters): a run's few launch shapes (warm-up, steps_per_execution, the remainder) each
        get their own, so no argument vector is rebuilt inside a timed loop."""
        from ..ops import _C
        from ..ops.functional import rng_state

        a = self.arena
        B = dense.shape[-2]
        fl = self._floats()
        key = (dense.data_ptr(), cat.data_ptr(), label.data_ptr(), nbatch, cursor.data_ptr(), nsteps, B,
               tuple(fl), id(a.master), self.dbg is not None, id(self.xdp))
        slots = self.__dict__.setdefault("_v2slots", {})
        sid = slots.get(key)
        if sid is not None:
            return sid
        ptr = lambda t: 0 if t is None else int(t.data_ptr())  # noqa: E731
        rows = int(self.model.wide.weight.shape[0])
        if self._zn is None:
            self._zn = torch.empty(rows, 2, device=a.device)  # the kernel's (z, n) scratch
        # Adagrad as w -= lr g rsq(s) (one transcendental): exact to fp32 when wd == 0 and eps is
        # below the resolution of sqrt(s), whose floor is the initial accumulator
        floor = float(getattr(self.ada, "initial_accumulator_value", 0.0))
        rsq = int(self.ada.weight_decay == 0 and floor > 0 and self.ada.hp["eps"] < 1e-7 * math.sqrt(floor))
        ptrs = [ptr(a.master), ptr(a.grad), ptr(a.shadow), ptr(a.state("adagrad_s0")),
                ptr(a.state("ftrl_s0")), ptr(a.state("ftrl_s1")), ptr(dense), ptr(cat), ptr(label),
                ptr(cursor), ptr(self.loss), ptr(self.correct), ptr(self.ada.step_count),
                ptr(self.ftrl.step_count), ptr(rng_state(a.device)), ptr(self.dbg), ptr(self._zn), rsq]
        if self.xdp is not None:
            ptrs += self.xdp.ptrs()
        free = slots.pop(next(iter(slots))) if len(slots) >= 8 else -1  # reuse the oldest slot id
        sid = _C.ext().taxi_step2_store(free, ptrs, self._ints(B, nbatch, nsteps), fl, rows)
        slots[key] = sid
        return sid

    def _launch(self, dense, cat, label, nbatch: int, cursor, nsteps: int = 1):
        from ..ops import _C
        from ..ops.functional import rng_state
        from ..ops.kernels import check, stream

        a = self.arena
        B = dense.shape[-2]
        self._B = B
        if self.v2(B):
            check(_C.ext().taxi_step2_slot(self._v2_slot(dense, cat, label, nbatch, cursor, nsteps), stream()),
                  "taxi_step2")
            return
        ptr = lambda t: 0 if t is None else int(t.data_ptr())  # noqa: E731
        ptrs = [ptr(a.master), ptr(a.grad), ptr(a.shadow), ptr(a.state("adagrad_s0")), ptr(a.state("ftrl_s0")),
                ptr(a.state("ftrl_s1")), ptr(dense), ptr(cat), ptr(label), ptr(cursor), ptr(self.loss),
                ptr(self.correct), ptr(self.ada.step_count), ptr(self.ftrl.step_count), ptr(rng_state(a.device)),
                ptr(self.dbg)]
        ptrs.append(ptr(self._slots(B)))
        check(_C.ext().widedeep_step(ptrs, self._ints(B, nbatch, nsteps), self._floats(), stream()),
              "widedeep_step")

    def _finish(self):
        if self.dp is not None:
            self.dp.allreduce_all()
            self.opt.step()
            if hasattr(self.dp, "post_step"):
                self.dp.post_step()

    def __call__(self, x, y):
        """One step on an explicit batch: x = (dense [B, 3], cat [B, 13] int64), y [B, 1]."""
        from ..runtime import health

        self._n += 1
        health.beat(self._n)
        dense, cat = x
        self._launch(dense.float().contiguous(), cat.contiguous(), y.float().contiguous(), 1, None)
        self._finish()
        return {"loss": self.loss, "correct": self.correct, "count": dense.shape[0]}

    def step_resident(self, xs, ys, graph: bool = True):
        """One step on batch ``cursor`` of a resident epoch xs = (dense [nb, B, 3] fp32, cat [nb, B, 13]),
        ys [nb, B, 1]; the kernel advances the cursor.  Single-GPU steps replay a captured graph."""
        from ..runtime import health

        self._n += 1
        health.beat(self._n)
        dense, cat = xs
        key = (dense.data_ptr(), cat.data_ptr(), ys.data_ptr(), tuple(self._floats()))
        if not graph or not self._graphable():
            self._launch(dense, cat, ys, dense.shape[0], self.cursor)
            self._finish()
        else:
            if self._key != key:  # new data or hyper-parameters (e.g. an lr schedule): recapture
                if not self.v2(dense.shape[-2]):
                    self._slots(dense.shape[-2])  # host->device copy of the slot table must precede capture
                self._sync_hp()
                torch.cuda.synchronize()
                g = torch.cuda.CUDAGraph()
                with _capture_graph(g):
                    self._launch(dense, cat, ys, dense.shape[0], self.cursor)
                    self._finish()  # multi-rank: the P2P all-reduce + optimizers are graph nodes too
                self._graph, self._key = g, key
                # capture does not execute: run this step through the graph
            self._graph.replay()
            if self.dp is not None:
                self.dp.poll()
        return {"loss": self.loss, "correct": self.correct, "count": dense.shape[1]}

    def _direct(self, dense) -> bool:
        """Single-GPU v2 step with its in-kernel step loop: launched directly (``HOPSX_TAXI_DIRECT=0``
        keeps the graph replays)."""
        return (self.dp is None and self.arena.device.type == "cuda" and self.v2(dense.shape[-2])
                and os.environ.get("HOPSX_TAXI_INKERNEL_LOOP", "1") == "1"
                and os.environ.get("HOPSX_TAXI_DIRECT", "1") == "1")

    def _graphable(self) -> bool:
        """One GPU, or a data-parallel engine whose collectives are graph-capturable (P2P kernels)."""
        return self.arena.device.type == "cuda" and (
            self.dp is None or getattr(self.dp, "capturable", lambda: False)())

    def _sync_hp(self):
        if self.dp is not None and hasattr(self.opt, "sync_hp"):
            self.opt.sync_hp()

    def _capture_u(self, dense, cat, ys, U: int):
        """U consecutive steps in one graph: ONE launch running U steps in-kernel on one GPU (the
        weights stay on chip between them); U launches + gradient exchanges when data-parallel."""
        if not self.v2(dense.shape[-2]):
            self._slots(dense.shape[-2])
        self._sync_hp()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with _capture_graph(g):
            if self.dp is None and os.environ.get("HOPSX_TAXI_INKERNEL_LOOP", "1") == "1":
                self._launch(dense, cat, ys, dense.shape[0], self.cursor, nsteps=U)
            else:
                for _ in range(U):
                    self._launch(dense, cat, ys, dense.shape[0], self.cursor)
                    self._finish()
        return g

    def prepare_resident(self, xs, ys, n: int | None = None) -> None:
        """Capture (not run) the U-step graph for this resident epoch, so it is built before a timed
        loop; with ``n`` also the graph of the remainder n % U (Keras steps_per_execution tail)."""
        dense, cat = xs
        U = self.steps_per_execution
        if n and self._direct(dense) and self.v2(dense.shape[-2]):
            # direct launches (run_resident): their argument slots for the launch shapes of n steps
            for k in {min(int(n), U), int(n) % U} - {0}:
                self._v2_slot(dense, cat, ys, dense.shape[0], self.cursor, k)
            return
        if U <= 1 or not self._graphable() or self._graph is None:
            return
        key = (dense.data_ptr(), cat.data_ptr(), ys.data_ptr(), tuple(self._floats()), U)
        if self._keyU != key:
            self._graphU, self._keyU = self._capture_u(dense, cat, ys, U), key
            self._graphR = {}
        rem = (n or 0) % U
        if rem > 1 and rem not in self._graphR:
            self._graphR[rem] = self._capture_u(dense, cat, ys, rem)

    def run_resident(self, xs, ys, n: int, graph: bool = True):
        """``n`` consecutive resident steps; single-GPU graph steps are replayed ``steps_per_execution``
        launches per graph (Keras steps_per_execution; each launch is a whole step on the next batch,
        the kernel advances the device cursor), so the per-replay gap is paid once per U steps."""
        from ..runtime import health

        U = self.steps_per_execution
        dense, cat = xs
        r = None
        if graph and self._direct(dense):
            # one GPU, whole steps in one kernel: each launch runs up to U steps in-kernel, launched
            # directly (a one-node graph replay costs more host time than the launch it replaces) with
            # the argument vectors kept in a C++ slot
            while n > 0:
                k = min(n, U)
                health.beat_range(self._n + 1, k)
                self._n += k
                self._launch(dense, cat, ys, dense.shape[0], self.cursor, nsteps=k)
                n -= k
            return {"loss": self.loss, "correct": self.correct, "count": dense.shape[1]}
        while n > 0:
            usable = U > 1 and graph and self._graphable() and self._graph is not None
            if usable and n < U and n in self._graphR:
                self.prepare_resident(xs, ys)  # (re-keys on new data / hyper-parameters)
                g = self._graphR.get(n)
                if g is not None:
                    health.beat_range(self._n + 1, n)
                    self._n += n
                    g.replay()
                    if self.dp is not None:
                        self.dp.poll()
                    n = 0
                    r = {"loss": self.loss, "correct": self.correct, "count": dense.shape[1]}
                    continue
            if n < U or not usable:
                r = self.step_resident(xs, ys, graph=graph)
                n -= 1
                continue
            self.prepare_resident(xs, ys)
            health.beat_range(self._n + 1, U)
            self._n += U
            self._graphU.replay()
            if self.dp is not None:
                self.dp.poll()
            n -= U
            r = {"loss": self.loss, "correct": self.correct, "count": dense.shape[1]}
        return r


def reference_steps(W, b, w4, b4, wide, ada_s, ftrl_z, ftrl_n, hp_ada, hp_ftrl, dense, cat, label, steps):
    """fp64 replay of ``steps`` v2 taxi steps that rounds to bf16 exactly where the kernel
    (csrc/ops/taxi_step.hip) holds bf16 images: inputs, hidden activations, W images and the backward
    gradients G.  W/b: the 4 hidden layers ([out, in] / [out]); w4, b4: logits; wide: [rows];
    ada_s: name -> Adagrad accumulator ("W0".."W3", "b0".."b3", "w4", "b4"); ftrl_z/n: [rows];
    hp_ada / hp_ftrl: the kernel's 8-float hyper-parameter vectors; dense/cat/label: [nb, B, ...].
    Everything is updated in place; returns the per-step mean losses.  A data-parallel step of W
    replicas is this with their batches concatenated along the batch axis (global-batch mean, one FTRL
    update per touched row with the summed gradient)."""
    def bf(x):
        return x.to(torch.bfloat16).to(torch.float64)

    lr, gscale, wd, eps = hp_ada[:4]
    flr, fgs, _, l1, l2, beta = hp_ftrl[:6]

    def adagrad(p, g, s):
        g = g * gscale + wd * p
        s += g * g
        return p - lr * g / (s.sqrt() + eps)

    losses = []
    for i in range(steps):
        j = i % dense.shape[0]
        x, c, y = dense[j], cat[j], label[j].reshape(-1)
        B = x.shape[0]
        acts = [bf(x)]
        a = acts[0]
        for l in range(4):
            a = bf(torch.relu(a @ bf(W[l]).T + b[l]))
            acts.append(a)
        z = a @ w4 + b4 + wide[c].sum(1)
        p = torch.sigmoid(z)
        losses.append(float(torch.nn.functional.binary_cross_entropy_with_logits(z, y)))
        g = (p - y) / B
        grads = {"w4": g @ a, "b4": g.sum()}  # the logits layer: fp32 g times the bf16 activations
        G = bf(g[:, None] * w4[None, :] * (a > 0))
        for l in (3, 2, 1, 0):
            grads[f"W{l}"] = G.T @ acts[l]
            grads[f"b{l}"] = G.sum(0)
            if l > 0:
                G = bf((G @ bf(W[l])) * (acts[l] > 0))
        # wide: summed example gradients per touched row, FTRL
        gw = torch.zeros_like(wide)
        gw.index_add_(0, c.reshape(-1), g[:, None].expand(-1, c.shape[1]).reshape(-1))
        rows = torch.unique(c.reshape(-1))
        gr = gw[rows] * fgs
        n_old = ftrl_n[rows]
        nn_ = n_old + gr * gr
        sigma = (nn_.sqrt() - n_old.sqrt()) / flr
        ftrl_z[rows] += gr - sigma * wide[rows]
        ftrl_n[rows] = nn_
        zz = ftrl_z[rows]
        wide[rows] = torch.where(zz.abs() <= l1, torch.zeros_like(zz),
                                 -(zz - torch.sign(zz) * l1) / ((beta + nn_.sqrt()) / flr + 2 * l2))
        for l in range(4):
            W[l] = adagrad(W[l], grads[f"W{l}"], ada_s[f"W{l}"])
            b[l] = adagrad(b[l], grads[f"b{l}"], ada_s[f"b{l}"])
        w4[:] = adagrad(w4, grads["w4"], ada_s["w4"])
        b4[:] = adagrad(b4, grads["b4"].reshape(1), ada_s["b4"])
    return losses


def reference_state(model, fused):
    """The fp64 host copies ``reference_steps`` takes, from a model's arena: (W, b, w4, b4, wide, ada_s,
    ftrl_z, ftrl_n, hp_ada, hp_ftrl)."""
    a = model.wide.weight._hx_arena
    lins = fused.lins
    f64 = lambda t: t.detach().double().cpu().clone()  # noqa: E731
    W = [f64(m.weight).reshape(m.weight.shape) for m in lins[:4]]
    b = [f64(m.bias) for m in lins[:4]]
    w4 = f64(lins[4].weight).reshape(-1)
    b4 = f64(lins[4].bias).reshape(1)
    s = a.state("adagrad_s0").double().cpu()
    ada = {}
    for l in range(5):
        m = lins[l]
        ws = s[m.weight._hx_off:m.weight._hx_off + m.weight.numel()].clone()
        bs = s[m.bias._hx_off:m.bias._hx_off + m.bias.numel()].clone()
        ada[f"W{l}" if l < 4 else "w4"] = ws.reshape(m.weight.shape) if l < 4 else ws
        ada[f"b{l}" if l < 4 else "b4"] = bs
    wo, rows = int(model.wide.weight._hx_off), model.wide.weight.shape[0]
    wide = a.master[wo:wo + rows].double().cpu().clone()
    z = a.state("ftrl_s0")[wo:wo + rows].double().cpu().clone()
    n = a.state("ftrl_s1")[wo:wo + rows].double().cpu().clone()
    fl = fused._floats()
    return W, b, w4, b4, wide, ada, z, n, fl[:8], fl[8:]


def synth_taxi(n: int, seed: int = 0, device="cpu"):
    """Transformed-feature synthetic taxi trips with a learnable tip rule.
    Returns dense [n, 3] f32, cat [n, 13] int64 (global one-hot ids), label [n, 1] f32."""
    g = torch.Generator().manual_seed(seed)
    dense = torch.randn(n, len(DENSE_FLOAT_FEATURE_KEYS), generator=g)
    card = wide_cardinalities()
    cols = []
    for c in card:
        if c == VOCAB_SIZE + OOV_SIZE:  # vocabulary columns are heavy-tailed
            r = torch.rand(n, generator=g)
            cols.append(torch.clamp((c * r ** 3).long(), max=c - 1))
        else:
            cols.append(torch.randint(0, c, (n,), generator=g))
    cat = torch.stack(cols, 1) + torch.from_numpy(wide_offsets())
    w_true = torch.randn(WIDE_ROWS, generator=g) * 0.5
    logit = dense @ torch.tensor([0.8, -0.6, 0.3]) + w_true[cat].sum(1) * 0.5
    label = (torch.rand(n, generator=g) < torch.sigmoid(logit)).float().unsqueeze(1)
    dev = torch.device(device)
    return dense.to(dev), cat.to(dev), label.to(dev)


def bench_taxi(dev, batch: int, steps: int, warmup: int, timed, world: int = 1, graph: bool = True,
               pool_examples: int = 200_000, from_transform: bool = False) -> dict:
    """Steps/sec of the taxi trainer (per-GPU batch ``batch``; DP all-reduce when world > 1).
    ``from_transform``: the training examples come from the TFX Transform stage (tfx.transform:
    raw synthetic trips analyzed + transformed on the device) instead of pre-transformed features;
    the analyze/apply time is reported, not timed with the steps."""
    from ..parallel.dp import DataParallel
    from ..runtime.arena import ParamArena
    from ..runtime.step import TrainStep

    model = TaxiWideDeep().to(dev)
    ParamArena.from_module(model, dev)
    opt = make_optimizer(model)
    xdp = None
    if (world > 1 and dev.type == "cuda" and os.environ.get("HOPSX_TAXI_FUSED", "1") == "1"
            and os.environ.get("HOPSX_TAXI_DP_FUSED", "1") == "1" and FusedWideDeepStep(model, opt).v2(batch)):
        # every rank decides alike (same model, batch and environment): the in-kernel exchange (collective setup)
        xdp = TaxiExchange(dev, world)
    dp = DataParallel(model) if world > 1 and xdp is None else None
    nb = max(8, -(-pool_examples // batch))
    transform_s = None
    if from_transform:
        import time as _time

        from ..tfx import analyze, synth_raw_trips

        raw = synth_raw_trips(nb * batch, seed=7)
        t0 = _time.perf_counter()
        tf = analyze(raw, device=dev)
        dense, cat, label = tf.apply(raw, device=dev)
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        transform_s = round(_time.perf_counter() - t0, 3)
    else:
        from ..parallel import dist as hdist

        # every replica trains on its own examples (data parallel): the seed carries the rank
        dense, cat, label = synth_taxi(nb * batch, seed=7 + 1009 * hdist.rank(), device=dev)
    cat = cat.view(nb, batch, -1)
    label = label.view(nb, batch, 1)
    out = {}
    fused = FusedWideDeepStep(model, opt, dp=dp, xdp=xdp) if os.environ.get("HOPSX_TAXI_FUSED", "1") == "1" else None
    if xdp is not None:
        xdp.sync_replicas(model.wide.weight._hx_arena)
    if fused is not None and fused.ok(batch):
        dense = dense.view(nb, batch, -1)
        path = f"fused-{fused.kernel}"

        def run(i):
            # one launch: the kernel reads batch `cursor` of the resident epoch and advances it
            out["r"] = fused.step_resident((dense, cat), label, graph=graph)

        def run_n(n):
            out["r"] = fused.run_resident((dense, cat), label, n, graph=graph)

        run.run_n = run_n
        run.prepare = lambda: fused.prepare_resident((dense, cat), label, n=steps)
    else:
        step = TrainStep(model, opt, "bce_logits", dp=dp, graph=graph, forward_fn=lambda m, x: m(*x))
        dense = dense.to(torch.bfloat16).view(nb, batch, -1)
        path = "layerwise"

        def run(i):
            j = i % nb
            out["r"] = step((dense[j], cat[j]), label[j])

    for i in range(warmup):
        run(i)
    if hasattr(run, "prepare"):
        run.prepare()  # build the multi-step graph outside the timed region
    el = timed(run, steps, dev)
    loss = float(out["r"]["loss"].reshape(-1)[0])
    replicas = None
    if xdp is not None:
        import torch.distributed as dist

        fused.check()  # the exchange's sticky error word (outside the timed region)
        digs = [None] * world
        dist.all_gather_object(digs, fused.digest())
        replicas = all(d == digs[0] for d in digs)
        xdp.close()
    return {"steps_per_sec": round(steps / el, 1), "examples_per_sec": round(batch * world * steps / el, 1),
            "ms_per_step": round(el / steps * 1e3, 4), "batch_per_gpu": batch, "loss": round(loss, 4),
            "params": sum(p.numel() for p in model.parameters()), "hidden_units": hidden_units(), "step": path,
            "data": "tfx-transform" if from_transform else "synthetic-transformed",
            **({"replicas_identical": replicas} if replicas is not None else {}),
            **({"transform_s": transform_s} if transform_s is not None else {})}
