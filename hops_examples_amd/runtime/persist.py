"""PersistentMnistStep: the flagship MirroredStrategy MNIST CNN trained ``n`` steps per launch.

Reference workload: notebooks/ml/Distributed_Training/mirrored_strategy/
mirroredstrategy_mnist_example.ipynb:189-222 (model, Adadelta(1.0) compile, fit on 32 images per
replica).  On one MI355X the whole training step — forward, softmax cross-entropy, backward and the
Adadelta update of all 1,394,282 parameters — runs inside ONE persistent kernel per
``steps_per_launch`` steps (csrc/ops/mnist_persist.hip): each of 169 workgroups owns one pooled
position and keeps its fc1 weight slice and Adadelta state in registers for the whole launch; 32 head
workgroups own one image each.  Four in-launch hand-offs per step replace six kernel launches and
the per-step HBM round trip of the 1.38 M fc1 parameters and their optimizer state.

Contract (same as TrainStep.run_resident on an HBM-resident epoch): every step trains on the next
batch of ``xs``/``ys`` (cycling), with dropout masks keyed on the device RNG counter, and the arena
(fp32 master, bf16 shadow, Adadelta accumulators), the optimizer's step count, the RNG counter and
the batch cursor are up to date in HBM when a launch returns.  The result is deterministic: no float
atomics, every cross-workgroup sum is a fixed-order loop.

Data parallel (world 2..8, one rank per GPU of one node): every rank runs the same persistent
kernel on its own 32 images and the replicas exchange, inside the launch, exactly what the update
needs over xGMI — each position's pooled activations and each rank's dh (the fc1 weight gradient is
their product, so 1.38 M gradient floats never cross the wire), the 1,418 head gradients and the
8,416 conv-gradient slice sums.  Producers push into the peers' uncached exchange buffers and raise a
flag word in the peers' flag pages; consumers poll their own page (csrc/ops/mnist_persist.hip,
"data-parallel exchange").  Every cross-rank sum runs in rank order, so the replicas stay
bit-identical; the loss is the mean over the global batch (MirroredStrategy semantics,
mirroredstrategy_mnist_example.ipynb:128-131).  ``loopback=world`` lets ONE process play every rank
(the peers' buffers are its own): the same code paths on one GPU, for tests.

Limits: batch 32 per replica, Adadelta, the MirroredMnistCNN architecture, ranks on distinct GPUs
(two kernels of 201 one-per-CU workgroups cannot be co-resident on one GPU).
``PersistentMnistStep.supported(...)`` says whether it applies.
"""
from __future__ import annotations

import os

import torch

_GEOM = None


def _ext():
    from ..ops import _C

    return _C.ext()


def geometry() -> dict:
    """Kernel geometry (csrc/ops/mnist_persist.hip constants)."""
    global _GEOM
    if _GEOM is None:
        g = _ext().mnist_persist_geom()
        _GEOM = dict(zip(["batch", "npos", "nhead", "grid", "nconv", "nslice", "slice", "pay", "flag_words",
                          "lds_bytes", "d_bytes", "x_bytes", "xflag_words", "max_ranks", "xo_pool", "xs_pool",
                          "xo_dht", "xs_dht", "xo_fc2", "xs_fc2", "xo_conv", "xs_conv"], g))
    return _GEOM


class PersistentError(RuntimeError):
    pass


def flagship_layers(model):
    """The (conv1, conv2, pool, fc1, fc2) layers when ``model`` has the structure of the reference's
    MirroredStrategy MNIST CNN (mirroredstrategy_mnist_example.ipynb:189-207) — Conv 1->32 k2 relu,
    Conv 32->64 k2 relu, MaxPool 2 (+ fused dropout), Dense 10816->128 relu, Dense 128->10, uint8 input
    affine on conv1 — matched on the layers, not on the class; else None."""
    from .. import nn as hnn
    from ..models.mnist import MirroredMnistCNN

    names = ("conv1", "conv2", "pool", "fc1", "fc2")
    L = [getattr(model, n, None) for n in names]
    if any(x is None for x in L):
        return None
    c1, c2, pool, f1, f2 = L

    def conv_ok(c, cin, cout):
        return (isinstance(c, hnn.Conv2d) and c.in_channels == cin and c.out_channels == cout
                and tuple(c.kernel_size) == (2, 2) and c.activation == "relu" and c.bias is not None
                and c.cfg.get("stride", 1) in (1, (1, 1)) and c.cfg.get("padding", 0) in (0, "valid", (0, 0))
                and c.cfg.get("dilation", 1) in (1, (1, 1)))

    def dense_ok(d, fin, fout, act):
        return (isinstance(d, hnn.Linear) and tuple(d.weight.shape) == (fout, fin) and d.activation == act
                and d.bias is not None)

    ok = (conv_ok(c1, 1, 32) and conv_ok(c2, 32, 64) and c1.in_affine is not None
          and isinstance(pool, hnn.MaxPool2d) and pool.k == 2 and pool.s in (None, 2) and not pool.p
          and 0.0 <= float(pool.dropout) < 1.0
          and dense_ok(f1, 13 * 13 * 64, 128, "relu") and dense_ok(f2, 128, 10, None))
    # the forward must be exactly that chain: the reference model class (or a subclass keeping its forward)
    return L if ok and type(model).forward is MirroredMnistCNN.forward else None


def _device_cus(dev) -> int:
    return int(torch.cuda.get_device_properties(dev).multi_processor_count)


def _occupancy(dp: bool) -> int:
    return int(_ext().mnist_persist_occupancy(int(dp)))


def launchable(dev, world: int = 1) -> tuple[bool, str]:
    """Can all of the persistent kernel's workgroups be resident at once on ``dev``?  Its workgroups
    hand data to each other inside the launch, so a partitioned GPU (fewer CUs than the grid) or a
    kernel too big for one workgroup per CU would spin until the hand-off timeout: refuse instead."""
    g = geometry()
    cus = _device_cus(dev)
    if cus < g["grid"]:
        return False, f"{cus} CUs < the persistent grid of {g['grid']} workgroups"
    occ = _occupancy(world > 1)
    if occ < 1:
        return False, f"occupancy {occ} workgroups per CU"
    return True, "ok"


class PersistentMnistStep:
    PARAMS = ("conv1.weight", "conv1.bias", "conv2.weight", "conv2.bias", "fc1.weight", "fc1.bias",
              "fc2.weight", "fc2.bias")

    @staticmethod
    def supported(model, opt, batch: int, world: int = 1) -> bool:
        """Local checks: the model's structure (``flagship_layers``), Adadelta over the whole arena, batch
        32 per replica, training mode, and a device that can hold every workgroup at once
        (``launchable``).  For world > 1 the caller also needs every rank on its own GPU of one node
        (``parallel.oneshot._colocation``) and a passing ``selftest()``; ``HOPSX_PERSIST=0`` /
        ``HOPSX_PERSIST_DP=0`` keep runs on TrainStep."""
        from ..optim import Adadelta

        if os.environ.get("HOPSX_PERSIST", "1") != "1":
            return False
        if world > 1 and (os.environ.get("HOPSX_PERSIST_DP", "1") != "1" or world > geometry()["max_ranks"]):
            return False
        a = getattr(opt, "arena", None)
        if not (isinstance(opt, Adadelta) and batch == 32 and a is not None and a.device.type == "cuda"
                and a.shadow is not None and opt._sl.start == 0 and opt._sl.stop >= a.numel and model.training
                and flagship_layers(model) is not None):
            return False
        return launchable(a.device, world)[0]

    def __init__(self, model, opt, steps_per_launch: int = 32, debug_stamps: bool = False, world: int | None = None,
                 loopback: int = 0, timeout_s: float | None = None, exchange=None):
        """``world``: replicas (default: the process group's size; 1 without one).  ``loopback``: play
        that many ranks in this one process (tests).  ``exchange``: a simulated exchange
        (runtime/persist_sim.py ExchangeSim) — the real data-parallel instantiation (loopback off), whose
        peer buffers / flag pages the simulator owns, so one process can play ranks that hold DIFFERENT
        batches.  ``timeout_s``: how long a hand-off waits before
        the launch is declared failed (default 2 s on one GPU, ``HOPSX_PERSIST_TIMEOUT_S`` or 60 s
        across ranks, whose launches can start far apart)."""
        from ..ops.functional import rng_state
        from ..parallel import dist as hdist

        a = opt.arena
        self.model, self.opt, self.arena = model, opt, a
        dev = a.device
        self.device = dev
        g = geometry()
        self.geom = g
        named = dict(model.named_parameters())
        self.offs = [int(named[n]._hx_off) for n in self.PARAMS]
        self.s1 = a.state("adadelta_s0")
        self.s2 = a.state("adadelta_s1")
        self.spl = max(1, int(os.environ.get("HOPSX_PERSIST_STEPS", steps_per_launch)))
        f32 = dict(device=dev, dtype=torch.float32)
        B, npos, nh = g["batch"], g["npos"], g["nhead"]
        self.slabA = torch.empty(2 * npos * B * 128, **f32)
        self.slabB = torch.empty(2 * nh * g["pay"], **f32)
        self.slabC = torch.empty(2 * npos * g["nconv"], **f32)
        self.slabD = torch.empty(2 * g["d_bytes"] // 4, **f32)
        self.flags = torch.zeros(g["flag_words"], device=dev, dtype=torch.int32)
        self.err = torch.zeros(4, device=dev, dtype=torch.int32)
        self.out = torch.zeros(2 * self.spl, **f32)
        self.cursor = torch.zeros(1, device=dev, dtype=torch.int64)
        self.rng = rng_state(dev)
        self.dbg = torch.zeros(g["grid"] * self.spl * 16, device=dev, dtype=torch.int64) if debug_stamps else None
        self.acquire = int(os.environ.get("HOPSX_PERSIST_ACQUIRE", "0"))
        self.loopback = int(loopback)
        # system-scope release fence before raising peer flags: the payload stores are themselves
        # system-scope write-through and drained before the flag, which is the release for them; the
        # fence only writes back OTHER dirty L2 lines (measured +3 us / step at 8 loopback ranks)
        self.xfence = int(os.environ.get("HOPSX_PERSIST_XFENCE", "0"))
        if exchange is not None:
            self.world, self.rank = int(exchange.world), 0
        elif self.loopback > 1:
            self.world, self.rank = self.loopback, 0
        else:
            self.world = int(world) if world is not None else hdist.world_size()
            self.rank = hdist.rank() if self.world > 1 else 0
        if self.world > g["max_ranks"]:
            raise ValueError(f"the persistent step supports <= {g['max_ranks']} ranks")
        default_t = "60" if self.world > 1 else "2"
        self.timeout_ms = int(1000 * float(timeout_s or os.environ.get("HOPSX_PERSIST_TIMEOUT_S", default_t)))
        self._xptrs: list[int] = []
        self._owned: list[int] = []
        self._opened: list[int] = []
        self.exchange = exchange
        self.selftest_report: dict | None = None
        if exchange is not None:
            self.xstep = torch.zeros(1, device=self.device, dtype=torch.int64)
            exchange.attach(self)
        elif self.world > 1:
            self._setup_exchange()
        self.use_graph = False
        self.steps_per_execution = self.spl
        self._last = None
        self._n = 0

    # ------------------------------------------------------------------ data parallel
    def _setup_exchange(self) -> None:
        """Allocate this rank's uncached exchange buffer + flag page, map every peer's (IPC handles
        through the default process group), make the replicas identical (rank 0's weights)."""
        import torch.distributed as dist

        from ..parallel import oneshot

        C = oneshot.ext()
        g = self.geom
        local = self.loopback > 1
        err = None
        from ..parallel import dist as hdist

        hdist.register(self)  # ordered teardown (close: local) at shutdown / interpreter exit
        try:
            buf, hb = C.alloc(int(g["x_bytes"]), True)
            self._owned.append(buf)
            flg, hf = C.alloc(int(g["xflag_words"]) * 4, True)
            self._owned.append(flg)
        except Exception as e:  # every rank must learn of it before the handle exchange
            err, hb, hf = repr(e), None, None
        self.xstep = torch.zeros(1, device=self.device, dtype=torch.int64)
        if local:
            if err:
                raise RuntimeError(f"persistent DP exchange setup failed: {err}")
            bufs, flags = [buf] * self.world, [flg] * self.world
        else:
            objs = [None] * self.world
            dist.all_gather_object(objs, (self.rank, None if err else bytes(hb), None if err else bytes(hf), err))
            bad = [(o[0], o[3]) for o in objs if o[3]]
            if bad:
                self.close()
                raise RuntimeError(f"persistent DP exchange setup failed on ranks {bad}")
            bufs, flags = [0] * self.world, [0] * self.world
            try:
                for r, b, f, _ in objs:
                    if r == self.rank:
                        bufs[r], flags[r] = buf, flg
                    else:
                        bufs[r] = C.open(b)
                        self._opened.append(bufs[r])
                        flags[r] = C.open(f)
                        self._opened.append(flags[r])
            except Exception as e:
                err = repr(e)
            oks = [None] * self.world
            dist.all_gather_object(oks, err)
            if any(oks):
                self.close()
                raise RuntimeError(f"persistent DP: mapping a peer's exchange buffer failed: {oks}")
            # replicas start from rank 0's parameters and optimizer state
            a = self.arena
            for t in (a.master, self.s1, self.s2):
                dist.broadcast(t, 0)
            a.shadow.copy_(a.master.to(a.shadow.dtype))
            dist.broadcast(self.opt.step_count, 0)
            torch.cuda.synchronize(self.device)
            dist.barrier()
        self._xptrs = [self.xstep.data_ptr()] + bufs + flags

    def close(self) -> None:
        """Unmap the peers' buffers and free this rank's (collective in spirit: call on every rank
        after the last launch has finished)."""
        if not self._owned:
            return
        from ..parallel import oneshot

        C = oneshot.ext()
        torch.cuda.synchronize(self.device)
        for p in self._opened:
            C.close(p)
        for p in self._owned:
            C.free(p)
        self._opened, self._owned, self._xptrs = [], [], []

    def param_digest(self) -> tuple[float, int]:
        """(sum, integer bit-sum) of the fp32 master: equal on every replica iff the replicas agree."""
        m = self.arena.master
        return float(m.double().sum()), int(m.view(torch.int32).long().sum())

    def verify_replicas(self) -> dict:
        """Collective: do all replicas hold bit-identical parameters?"""
        import torch.distributed as dist

        d = self.param_digest()
        if self.world <= 1 or self.loopback > 1:
            return {"identical": True, "digests": [d]}
        objs = [None] * self.world
        dist.all_gather_object(objs, d)
        return {"identical": all(o == objs[0] for o in objs), "digests": objs}

    def views(self) -> dict:
        """name -> (fp32 master, Adadelta E[g^2], E[dx^2]) views of every parameter in the arena."""
        named = dict(self.model.named_parameters())
        out = {}
        for k in self.PARAMS:
            t = named[k]
            o, n = int(t._hx_off), t.numel()
            out[k] = tuple(x[o:o + n].view(t.shape) for x in (self.arena.master, self.s1, self.s2))
        return out

    def _state(self):
        a = self.arena
        return (a.master, a.shadow, self.s1, self.s2, self.opt.step_count, self.rng, self.cursor)

    def numeric_probe(self, xs=None, ys=None, reduce=None, tries: int = 6) -> dict:
        """One data-parallel training step of the kernel on a scratch copy of the state (optimizer
        accumulators zeroed, so E[g^2] after the step is 0.05 g^2 exactly), checked against fp64:
        this replica's bf16-emulating fp64 gradient of its share of the global-batch loss
        (``reference_grads``), summed over the replicas by ``reduce`` (default: an all-reduce over the
        process group), one fp64 Adadelta step, ``compare_update``.  ``xs``/``ys``: this replica's batch
        [1, 32, 28, 28, 1] / [1, 32] (default: a random batch, redrawn while an fc1 ReLU input sits
        within 2e-5 of 0, where fp32-vs-fp64 accumulation can flip it).  With a simulated exchange
        (``exchange``) the step is ExchangeSim.step over W random batches and the reference sums the W
        replicas' gradients in-process.  The real state is restored.  Returns compare_update's report
        plus "err" (the launch's error word)."""
        import torch.distributed as dist

        B = self.geom["batch"]
        V = self.views()
        P0 = {k: v[0].detach().to(torch.float64).clone() for k, v in V.items()}
        pool = self.model.pool
        drop = float(pool.dropout) if pool.training else 0.0
        seed, ctr = int(self.rng[0].item()) & ((1 << 64) - 1), int(self.rng[1].item())
        scale, shift = self.model.conv1.in_affine
        denom = self.world * B
        rf = dict(xscale=float(scale), xshift=float(shift), emulate_bf16=True)

        def draw(rank, xs=None, ys=None):
            g = torch.Generator().manual_seed(0x5E1F + 7919 * rank)
            for t in range(tries if xs is None else 1):
                if xs is None or t > 0:
                    xs = torch.randint(0, 256, (1, B, 28, 28, 1), dtype=torch.uint8, generator=g).to(self.device)
                    ys = torch.randint(0, 10, (1, B), dtype=torch.int64, generator=g).to(self.device)
                P = {k: v.clone().requires_grad_(True) for k, v in P0.items()}
                mg = []
                grads, _ = reference_grads(P, xs[0], ys[0], seed, ctr, int(pool.salt), drop, rank * B, denom,
                                           margins=mg, **rf)
                if mg[0]["fc1"] > 2e-5:
                    break
            return xs, ys, torch.cat([gr.flatten() for gr in grads])

        sim = self.exchange
        if sim is not None:
            batches = [draw(r) for r in range(self.world)]
            flat = sum(b[2] for b in batches)
        else:
            xs, ys, flat = draw(self.rank, xs, ys)
            if reduce is not None:
                flat = reduce(flat)
            elif self.loopback > 1:
                flat = flat * self.world  # every simulated peer holds this rank's batch (and masks)
            elif self.world > 1:
                dist.all_reduce(flat)
        grads, o = [], 0
        for k, v in P0.items():
            grads.append(flat[o:o + v.numel()].view_as(v))
            o += v.numel()
        S1r = {k: torch.zeros_like(v) for k, v in P0.items()}
        S2r = {k: torch.zeros_like(v) for k, v in P0.items()}
        opt = self.opt
        opt.sync_hp()
        lr, _, _, rho, eps = [float(v) for v in opt._hp()][:5]
        Pr = adadelta_ref(P0, S1r, S2r, grads, lr, rho, eps)
        saved = [t.clone() for t in self._state()]
        try:
            self.s1.zero_()
            self.s2.zero_()
            if sim is not None:
                sim.step([b[0] for b in batches], [b[1] for b in batches])
            else:
                self._launch(xs, ys, 1, 1)
            torch.cuda.synchronize(self.device)
            err = int(self.err[0].item())
            V = self.views()
            P1 = {k: v[0].detach().clone() for k, v in V.items()}
            S1k = {k: v[1].detach().clone() for k, v in V.items()}
        finally:
            for t, sv in zip(self._state(), saved):
                t.copy_(sv)
            torch.cuda.synchronize(self.device)
        rep = compare_update(P0, P1, S1k, Pr, S1r)
        rep["err"] = err
        rep["ok"] = rep["ok"] and err == 0
        return rep

    def selftest(self, steps: int = 3, numeric: bool = True) -> bool:
        """Collective pre-flight of the cross-rank exchange on a scratch copy of the model state.
        (1) ``numeric_probe``: one step on this rank's own random batch must match the fp64
        reference of the GLOBAL batch — every replica's gradient, all-reduced over the process group
        (RCCL) — per parameter tensor (update cosine >= 0.999, E[g^2] within 2 %): a dropped peer, a
        wrong world-size scale or a mis-ordered slot fails here even when every rank is wrong the same
        way.  (2) a few launches, then every rank must report no hand-off error and bit-identical
        scratch parameters.  The real state (arena, optimizer, RNG counter, cursor) is untouched.
        Returns the verdict every rank agrees on; ``selftest_report`` keeps the details."""
        import torch.distributed as dist

        B = self.geom["batch"]
        saved = [t.clone() for t in self._state()]
        ok, rep = True, None
        # the self-test's launches start together (right after a collective): a hand-off that has not
        # arrived within a few seconds never will, so a broken exchange costs seconds here, not the
        # 60 s a training launch waits for a late peer (HOPSX_PERSIST_SELFTEST_TIMEOUT_S)
        t_run = self.timeout_ms
        self.timeout_ms = min(t_run, int(1000 * float(os.environ.get("HOPSX_PERSIST_SELFTEST_TIMEOUT_S", "8"))))
        try:
            if numeric:
                rep = self.numeric_probe()
                ok = rep["ok"]
            xs = torch.randint(0, 256, (2, B, 28, 28, 1), dtype=torch.uint8, device=self.device)
            ys = torch.randint(0, 10, (2, B), dtype=torch.int64, device=self.device)
            if int(self.err[0].item()) == 0 and self.exchange is None:
                for k in (steps, 1):
                    self._launch(xs, ys, 2, k)
            torch.cuda.synchronize(self.device)
            ok = ok and int(self.err[0].item()) == 0
            dig = self.param_digest()
        except Exception as e:
            ok, dig = False, None
            rep = dict(rep or {}, exception=repr(e)[:300])
        finally:
            self.timeout_ms = t_run
            for t, sv in zip(self._state(), saved):
                t.copy_(sv)
            torch.cuda.synchronize(self.device)
        if self.world > 1 and self.loopback <= 1 and self.exchange is None:
            objs = [None] * self.world
            dist.all_gather_object(objs, (ok, dig))
            ok = all(o[0] for o in objs) and all(o[1] == objs[0][1] for o in objs)
        self.selftest_report = {"ok": ok, "numeric": rep}
        if ok:
            self.err.zero_()
        return ok

    # ------------------------------------------------------------------ launch
    def _check_data(self, xs, ys):
        chk = getattr(self, "_checked", None)
        if chk is not None and chk[0] is xs and chk[1] is ys and chk[2] == (xs.data_ptr(), ys.data_ptr()):
            return chk[3]  # the same resident epoch as the last call (the common case: every launch)
        B = self.geom["batch"]
        if xs.dtype != torch.uint8 or not xs.is_contiguous() or xs.device != self.device:
            raise ValueError("xs must be a contiguous uint8 tensor on the model's device")
        if xs.numel() % (B * 784) or xs.dim() < 3 or xs.shape[1] != B:
            raise ValueError(f"xs must be [nbatch, {B}, 28, 28(, 1)], got {tuple(xs.shape)}")
        nb = xs.shape[0]
        if ys.dtype != torch.int64 or tuple(ys.shape) != (nb, B) or not ys.is_contiguous() or ys.device != self.device:
            raise ValueError(f"ys must be a contiguous int64 [{nb}, {B}] tensor on the model's device")
        self._checked = (xs, ys, (xs.data_ptr(), ys.data_ptr()), nb)
        return nb

    def _launch(self, xs, ys, nb: int, k: int) -> None:
        from ..ops import _C

        opt = self.opt
        opt.sync_hp()
        hp = [float(v) for v in opt._hp()]  # lr gscale wd rho eps
        # the argument vectors are built once per launch shape (_arg_slot): at bench.py's 20 steps per launch
        # the host-side preparation would be in the timed window while the GPU idles.  The launch before
        # this one with the same epoch tensors, step count, hyper-parameters and dropout state reuses its
        # slot without rebuilding the key (the host issue cost is in the timed window too)
        pool = self.model.pool
        fast = (xs, ys, xs.data_ptr(), k, hp, pool.training, pool.dropout)
        last = getattr(self, "_last_launch", None)
        if last is not None and last[0] is xs and last[1] is ys and last[2:-1] == fast[2:]:
            sid = last[-1]
        else:
            sid = self._arg_slot(self._launch_key(xs, ys, nb, k, hp), xs, ys, nb, k, hp)
            self._last_launch = fast + (sid,)
        rc = self._ext.mnist_persist_slot(sid, _C.stream())
        if rc == 720:  # hipErrorCooperativeLaunchTooLarge
            raise PersistentError("mnist_persist: cooperative launch refused — the device cannot hold all "
                                  f"{self.geom['grid']} workgroups at once")
        _C.check(rc, "mnist_persist")

    def _launch_key(self, xs, ys, nb: int, k: int, hp: list):
        pool = self.model.pool
        return (xs.data_ptr(), ys.data_ptr(), nb, k, float(pool.dropout) if pool.training else 0.0, int(pool.salt),
                tuple(hp), self.acquire, self.xfence, self.timeout_ms, id(self.dbg), id(self.cursor), id(self.rng),
                id(self.arena.master), id(self.s1), self.world, self.rank, tuple(self._xptrs))

    def _arg_slot(self, key, xs, ys, nb: int, k: int, hp: list) -> int:
        """The C++-side argument slot of this launch shape: built once per key (a few launch shapes per run:
        warm-up steps, steps_per_launch, the remainder), a launch then passes the slot id and the stream."""
        slots = self.__dict__.setdefault("_slots", {})
        sid = slots.get(key)
        if sid is None:
            free = -1
            if len(slots) >= 8:  # reuse the oldest slot id (and forget the launch fast path, which may hold it)
                free = slots.pop(next(iter(slots)))
                self._last_launch = None
            sid = self._ext.mnist_persist_store(free, *self._build_args(xs, ys, nb, k, hp))
            slots[key] = sid
        return sid

    def _build_args(self, xs, ys, nb: int, k: int, hp: list):
        opt, a, m = self.opt, self.arena, self.model
        ptrs = [a.master.data_ptr(), a.shadow.data_ptr(), self.s1.data_ptr(), self.s2.data_ptr(), xs.data_ptr(),
                ys.data_ptr(), self.cursor.data_ptr(), self.rng.data_ptr(), opt.step_count.data_ptr(),
                opt._hp_dev.data_ptr() if opt._hp_dev is not None else 0, self.slabA.data_ptr(),
                self.slabB.data_ptr(), self.slabC.data_ptr(), self.slabD.data_ptr(), self.flags.data_ptr(),
                self.err.data_ptr(), self.out.data_ptr(), self.dbg.data_ptr() if self.dbg is not None else 0]
        ptrs += self._xptrs
        pool = m.pool
        drop = float(pool.dropout) if pool.training else 0.0
        scale, shift = m.conv1.in_affine
        iv = self.offs + [nb, int(pool.salt), int(k), self.geom["batch"], self.acquire, self.world, self.rank,
                          1 if self.loopback > 1 else 0, self.timeout_ms, self.xfence]
        fv = [drop, float(scale), float(shift)] + (hp + [0.0] * 5)[:5]
        return ptrs, iv, fv

    @property
    def _ext(self):
        return _ext()

    def run_resident(self, xs, ys, n: int):
        """``n`` training steps on the resident epoch, ``steps_per_launch`` per launch.  Returns the
        last step's {"loss", "correct", "count"} as device tensors (no host sync)."""
        nb = self._check_data(xs, ys)
        k = 0
        while n > 0:
            k = min(n, self.spl)
            self._launch(xs, ys, nb, k)
            n -= k
            self._n += k
        if k:
            self._last = {"loss": self.out[2 * (k - 1)], "correct": self.out[2 * k - 1],
                          "count": self.geom["batch"]}
        return self._last

    def step_resident(self, xs, ys):
        return self.run_resident(xs, ys, 1)

    def __call__(self, x, y):
        """One step on an explicit batch (TrainStep API): x uint8 [32, 28, 28(, 1)], y int64 [32] — a
        resident epoch of one batch.  Prefer ``run_resident`` on a device-resident epoch: one launch
        then runs ``steps_per_launch`` steps."""
        xs = x.reshape(1, *x.shape) if x.is_contiguous() else x.contiguous().reshape(1, *x.shape)
        return self.run_resident(xs, y.reshape(1, -1).contiguous(), 1)

    def eager(self, x, y):
        return self(x, y)

    def prepare_resident(self, xs, ys, n=None) -> None:
        """TrainStep API parity (there is no graph to capture): validates the epoch and builds the launch
        arguments of the launch shapes ``run_resident(xs, ys, n)`` will use (``steps_per_launch`` and the
        remainder), so none of that host work falls inside a timed run."""
        nb = self._check_data(xs, ys)
        if n:
            self.opt.sync_hp()
            hp = [float(v) for v in self.opt._hp()]
            for k in {min(int(n), self.spl), int(n) % self.spl} - {0}:
                self._arg_slot(self._launch_key(xs, ys, nb, k, hp), xs, ys, nb, k, hp)

    def losses(self, k: int) -> torch.Tensor:
        """[k, 2] (mean loss, correct) of the last launch's first k steps."""
        return self.out[: 2 * k].view(k, 2)

    def check(self) -> None:
        """Raise if a hand-off of any launch timed out or was aborted (sticky device error word)."""
        e = int(self.err[0].item()) & 0xFFFFFFFF
        if e:
            # a launch that gave up left flag epochs behind without advancing the epoch base: clear them,
            # so a later launch (after the caller resets err) cannot match a stale flag
            self.flags.zero_()
            phase, step, wg = (e >> 24) & 0x7F, (e >> 12) & 0xFFF, e & 0xFFF
            if phase == 12:
                raise PersistentError(f"mnist_persist: the grid's workgroups were not co-resident (workgroup {wg} "
                                      "waited out step 0's local hand-off: another kernel holds CUs this launch "
                                      "needs); arena state of the failed launch is partial")
            raise PersistentError(f"mnist_persist: hand-off wait timed out (phase {phase}, step {step}, "
                                  f"workgroup {wg}); arena state of the failed launch is partial")

    def phase_stamps(self, k: int) -> torch.Tensor:
        """[grid, k, 16] wall-clock stamps (100 MHz ticks) of the last launch (debug_stamps=True).
        Position workgroups: 0 step start, 1 conv fwd done, 2 A published, 3 B ready, 4 pool bwd done,
        5 conv bwd done, 6 C published, 7 C ready (slice owners), 8 D published (owners), 9 fc1 slice
        updated, 10 D ready, 11 step end.  Heads: 0 A ready, 1 B published, 2 fc2 update done."""
        if self.dbg is None:
            raise RuntimeError("construct with debug_stamps=True")
        return self.dbg.view(self.geom["grid"], self.spl, 16)[:, :k]


# ---------------------------------------------------------------------------------------------
# fp64 PyTorch reference of the same training steps (numerics tests, tools/persist_check.py)
# ---------------------------------------------------------------------------------------------
_M32 = 0xFFFFFFFF


def _mix32(x: torch.Tensor) -> torch.Tensor:
    x = x ^ (x >> 16)
    x = (x * 0x7FEB352D) & _M32
    x = x ^ (x >> 15)
    x = (x * 0x846CA68B) & _M32
    return x ^ (x >> 16)


def dropout_keep(seed: int, ctr: int, salt: int, idx: torch.Tensor, p: float) -> torch.Tensor:
    """The kernels' counter-based dropout mask (common.h drop_key / hash_u32 / uniform01) for int64
    element indices < 2**32: True where the element is kept."""
    m64 = (1 << 64) - 1
    key = (seed ^ ((salt * 0xD1B54A32D192ED03) & m64) ^ ((ctr * 0x8CB92BA72F3D8DD7) & m64)) & m64
    ka, kb = key & _M32, key >> 32
    h = _mix32((_mix32((idx & _M32) ^ ka) + kb) & _M32)
    return (h & 0xFFFFFF).to(torch.float64) * (1.0 / 16777216.0) >= p


class _RoundFwd(torch.autograd.Function):
    """x -> bf16(x) in the forward, gradient passed straight through (an operand the kernel reads as bf16)."""

    @staticmethod
    def forward(ctx, x):
        return x.to(torch.bfloat16).to(x.dtype)

    @staticmethod
    def backward(ctx, g):
        return g


class _RoundGrad(torch.autograd.Function):
    """identity in the forward; the incoming gradient is rounded to bf16 (a gradient the kernel stores as a
    bf16 MFMA operand)."""

    @staticmethod
    def forward(ctx, x):
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        return g.to(torch.bfloat16).to(g.dtype)


def reference_grads(P: dict, x_u8: torch.Tensor, y: torch.Tensor, seed: int, ctr: int, salt: int, drop_p: float,
                    image_offset: int = 0, denom: int | None = None, xscale: float = 1.0 / 255.0,
                    xshift: float = -0.5, emulate_bf16: bool = False, margins: list | None = None):
    """fp64 gradient of ONE replica's share of the MirroredStrategy loss: ``sum_b CE(image b) / denom``
    over this replica's images ``x_u8`` [B, 28, 28(, 1)], whose dropout masks are those of global images
    ``image_offset .. image_offset + B - 1`` (the kernel keys a mask on the global image index
    rank * 32 + b).  ``denom`` = the global batch (default B).  Summing every replica's result is the
    gradient of the global-batch mean — what an all-reduce of the replicas' gradients produces
    (mirroredstrategy_mnist_example.ipynb:128-131).  P: name -> fp64 tensor with requires_grad.
    Returns (grads in P's order, sum of this replica's CE losses).  ``emulate_bf16`` / ``margins``: see
    ``reference_steps``."""
    import torch.nn.functional as F

    rf = _RoundFwd.apply if emulate_bf16 else (lambda t: t)
    rg = _RoundGrad.apply if emulate_bf16 else (lambda t: t)
    B = y.shape[0]
    denom = B if denom is None else int(denom)
    x = x_u8.reshape(B, 1, 28, 28).to(torch.float64) * xscale + xshift
    z1 = F.conv2d(x, P["conv1.weight"].permute(0, 3, 1, 2), P["conv1.bias"])
    h = rf(F.relu(z1))
    z2 = F.conv2d(h, rf(P["conv2.weight"]).permute(0, 3, 1, 2), P["conv2.bias"])
    h = rg(rf(F.relu(z2)))
    h = F.max_pool2d(h, 2).permute(0, 2, 3, 1).reshape(B, -1)  # NHWC flatten
    if drop_p > 0:
        per = 169 * 64
        po = torch.arange(B * per, dtype=torch.int64, device=x_u8.device) + int(image_offset) * per
        keep = dropout_keep(seed, ctr, salt, po, drop_p).reshape(B, -1)
        h = h * keep.to(h.dtype) / (1.0 - drop_p)
    z3 = rg(F.linear(rf(h), rf(P["fc1.weight"]))) + P["fc1.bias"]
    h = F.relu(z3)
    if margins is not None:
        margins.append({k: float(z.detach().abs().min()) for k, z in (("conv1", z1), ("conv2", z2), ("fc1", z3))})
    logits = F.linear(h, P["fc2.weight"], P["fc2.bias"])
    loss = F.cross_entropy(logits, y, reduction="sum")
    grads = torch.autograd.grad(loss / denom, list(P.values()))
    return grads, float(loss.detach())


def adadelta_ref(P: dict, S1: dict, S2: dict, grads, lr: float, rho: float, eps: float) -> dict:
    """One fp64 Adadelta step (optim_core.h upd<3>) in place on S1 / S2; returns the new parameters."""
    out = {}
    with torch.no_grad():
        for (k, w), g in zip(list(P.items()), grads):
            S1[k].mul_(rho).addcmul_(g, g, value=1 - rho)
            d = (S2[k] + eps).sqrt() / (S1[k] + eps).sqrt() * g
            S2[k].mul_(rho).addcmul_(d, d, value=1 - rho)
            out[k] = w.detach() - lr * d
    return out


def compare_update(P0: dict, P1: dict, S1k: dict, Pr: dict, S1r: dict, cos_min: float = 0.999,
                   srel_max: float = 2e-2) -> dict:
    """Per parameter tensor: the cosine between the kernel's update P1 - P0 and the reference's Pr - P0,
    and the relative L2 error of the kernel's Adadelta E[g^2] against the reference's.  E[g^2] carries
    the gradient's MAGNITUDE (the first Adadelta steps are nearly sign(g) x const, so the update's
    direction alone misses a gradient that is scaled wrong, e.g. by the wrong world size); the update
    cosine carries its direction.  Returns {"ok": bool, "tensors": {name: (cos, srel)}}."""
    rep, ok = {}, True
    for k in P0:
        dk = (P1[k].double() - P0[k].double()).flatten()
        dr = (Pr[k].double() - P0[k].double()).flatten()
        cos = float(torch.nn.functional.cosine_similarity(dk, dr, dim=0))
        sk, sr = S1k[k].double().flatten(), S1r[k].double().flatten()
        srel = float((sk - sr).norm() / sr.norm().clamp_min(1e-300))
        rep[k] = (cos, srel)
        ok = ok and cos >= cos_min and srel <= srel_max
    return {"ok": ok, "tensors": rep}


def reference_steps(params: dict, s1: dict, s2: dict, xs: torch.Tensor, ys: torch.Tensor, cursor: int, n: int,
                    seed: int, ctr: int, salt: int, drop_p: float, lr: float, rho: float, eps: float,
                    xscale: float = 1.0 / 255.0, xshift: float = -0.5, emulate_bf16: bool = False,
                    margins: list | None = None):
    """``n`` fp64 training steps of MirroredMnistCNN with the kernel's data order, dropout masks,
    loss (mean sparse CE) and Adadelta.  params / s1 / s2: name -> tensor (hopsx layouts: conv OHWI,
    dense [out, in]).  Returns fp64 (params, s1, s2, losses).  A data-parallel step of W replicas is
    this with the replicas' batches concatenated along the batch axis (replica r's images are global
    images r * 32 .. r * 32 + 31, the kernel's dropout key).

    ``emulate_bf16``: round exactly the tensors the persistent kernel stores as bf16 MFMA operands —
    conv1 output, conv2 weight, the relu'd conv2 output (before the max-pool, as the kernel ties it),
    the pooled+dropout activations, the fc1 weight, dh (fc1 output gradient, not its bias gradient) and
    the conv2 output gradient — and nothing else, so the kernel differs from it only by fp32 vs fp64
    accumulation (and the rare relu / max-pool tie that rounding flips).

    ``margins``: a list that receives, per step, the smallest |pre-activation| of each ReLU (conv1,
    conv2, fc1) — how close the step came to a tie that fp32-vs-fp64 accumulation can flip.  A flip
    at fc1 moves a whole fc1 row's gradient and, through dh, every conv gradient."""
    P = {k: v.detach().to(torch.float64).clone() for k, v in params.items()}
    S1 = {k: v.detach().to(torch.float64).clone() for k, v in s1.items()}
    S2 = {k: v.detach().to(torch.float64).clone() for k, v in s2.items()}
    nb, B = ys.shape
    losses = []
    for s in range(n):
        bt = (cursor + s) % nb
        for v in P.values():
            v.requires_grad_(True)
        grads, lsum = reference_grads(P, xs[bt], ys[bt], seed, ctr + s, salt, drop_p, 0, B, xscale, xshift,
                                      emulate_bf16, margins)
        losses.append(lsum / B)
        P = adadelta_ref(P, S1, S2, grads, lr, rho, eps)
    return {k: v.detach() for k, v in P.items()}, S1, S2, losses
