"""TrainStep: a training step (forward, fused loss, backward, gradient all-reduce,
fused optimizer, RNG advance) that is captured into hipGraphs after warm-up.

The reference runs the equivalent step inside ``model.fit`` (TF) or a Python
loop (PyTorch) — notebooks/ml/Experiment/PyTorch/mnist.ipynb:136-154.  On
MI355X the small reference models are launch-bound (a 32-image MNIST step is
~1-3 GFLOP), so after warm-up the whole step is replayed from a hipGraph: one
host call per step instead of ~30 kernel launches plus autograd bookkeeping.

world_size == 1 : one graph  = fwd + bwd + optimizer + rng
world_size  > 1 : P2P path (parallel/oneshot.py, one node): one graph = fwd + bwd + the fused
                  reduce-scatter / sharded-update / all-gather kernel (or P2P all-reduce +
                  optimizer), replayed steps_per_execution at a time like one GPU;
                  RCCL path: graph A = fwd + bwd (the RCCL all-reduce of the flat grad
                  buckets runs between the graphs, on RCCL's stream), graph B = optimizer + rng;
                  HOPSX_GRAPH_COLLECTIVES=1 captures the RCCL collectives too (one graph).

Every path — eager, one-step graph, multi-step graph — runs the same step tail (``_tail``):
gradient exchange, optimizer, the engine's post-step (sharded PS all-gather).  Hyper-parameters
live on the device (optim.FusedOptimizer.sync_hp before every replay), so lr changes after a
capture take effect on replay.

``run_resident(xs, ys, n)`` (single GPU, HBM-resident epoch) also captures ``steps_per_execution``
consecutive steps into ONE graph — Keras' ``compile(steps_per_execution=...)``.  Every step is
still a full forward / loss / backward / optimizer step on the next batch (the optimizer kernel's
tail prefetches it and advances the device cursor); only the per-replay launch gap (~8 us on
MI355X, ~9% of a 32-image MNIST step) is paid once per U steps instead of once per step.
"""
from __future__ import annotations

import os

import torch

from .capture import graph as _capture_graph

from ..ops import functional as HF
from ..parallel import dist as hdist
from . import health


def _mark_ready(p):
    r = HF.COLAUNCH["ready"]
    if r is not None:
        r.add(id(p))


def _clone(x):
    return tuple(t.clone() for t in x) if isinstance(x, (tuple, list)) else x.clone()


def _shape(x):
    return tuple(t.shape for t in x) if isinstance(x, (tuple, list)) else x.shape


def _same_storage(a, b):
    if isinstance(a, (tuple, list)):
        return all(u.data_ptr() == v.data_ptr() for u, v in zip(a, b))
    return a.data_ptr() == b.data_ptr()


def _copy_into(dst, src):
    if isinstance(dst, (tuple, list)):
        for d, s_ in zip(dst, src):
            d.copy_(s_, non_blocking=True)
    else:
        dst.copy_(src, non_blocking=True)


class TrainStep:
    """``x`` may be a tensor or a tuple of tensors (e.g. dense + categorical inputs)."""

    def __init__(self, model, optimizer, loss_kind: str = "sparse_ce", dp=None, graph: bool = True, warmup: int = 3,
                 forward_fn=None, steps_per_execution: int = 8):
        self.model, self.opt, self.loss_kind, self.dp = model, optimizer, loss_kind, dp
        self.forward_fn = forward_fn or (lambda m, x: m(x))
        dev = optimizer.arena.device
        self.device = dev
        self.use_graph = bool(graph) and dev.type == "cuda" and os.environ.get("HOPSX_GRAPH", "1") == "1"
        self.warmup = warmup
        self.graph_collectives = os.environ.get("HOPSX_GRAPH_COLLECTIVES", "0") == "1"
        self._n = 0
        self._g1 = self._g2 = None
        self._sx = self._sy = None
        self._out = None
        self._rn = 0
        self._resident = None
        self._cursor = None
        self._pf_opt = None
        self._pf_pending = None
        self.defer_head = os.environ.get("HOPSX_DEFER_HEAD", "1") == "1"
        self._head_defer = None
        self._prehead_w = None
        self.steps_per_execution = max(1, int(os.environ.get("HOPSX_STEPS_PER_EXEC", steps_per_execution)))
        self._gU = None
        self._outU = None
        self._gR: dict = {}  # remainder graphs: U -> (graph, outputs)
        self._outs_of: dict = {}  # id(multi-step graph) -> every captured step's outputs
        self._pool = None
        if dp is not None:
            optimizer.grad_scale = dp.grad_scale()
            if hasattr(dp, "bind_optimizer"):
                dp.bind_optimizer(optimizer)  # fused P2P step tail when the engine supports it
            if getattr(dp, "capturable", lambda: False)():
                self.graph_collectives = True  # P2P kernels capture like any other

    # ------------------------------------------------------------- eager path
    def _forward(self, x):
        """Model forward.  The first CUDA step probes whether the logits layer's output is exactly
        the model output (nothing else reads it); from then on that layer's forward is deferred
        into the fused loss kernel (functional.HEAD, loss.hip head_ce_k forward mode)."""
        if self.device.type != "cuda" or not self.defer_head:
            return self.forward_fn(self.model, x)
        if self._head_defer is None:
            HF.HEAD["probe"] = []
            HF.HEAD["last_lin"] = HF.HEAD["prehead_w"] = None
            try:
                out = self.forward_fn(self.model, x)
                probe = HF.HEAD["probe"]
                prehead = HF.HEAD["prehead_w"]
            finally:
                HF.HEAD["probe"] = None
                HF.HEAD["last_lin"] = HF.HEAD["prehead_w"] = None
            self._head_defer = len(probe) == 1 and probe[0] is out
            # the Dense layer feeding the logits layer runs inside the loss kernel too (mlp_head)
            self._prehead_w = prehead if (self._head_defer and os.environ.get("HOPSX_DEFER_PREHEAD", "1") == "1") \
                else None
            return out
        HF.HEAD["defer"] = self._head_defer
        HF.PREHEAD["w"] = self._prehead_w
        try:
            return self.forward_fn(self.model, x)
        finally:
            HF.HEAD["defer"] = False
            HF.PREHEAD["w"] = None

    def _colaunch_ok(self) -> bool:
        """One GPU, a single fused optimizer over the arena: the last backward launch may carry the
        optimizer's update of the layers whose gradients are already final (functional.COLAUNCH;
        HOPSX_OPT_COLAUNCH=1)."""
        from ..optim import FusedOptimizer

        # opt-in: measured slower on the flagship (profiles/r3s7_flagship_ab.txt: the optimizer
        # workgroups compete with the pair's 2-per-CU workgroups for slots, 0.0817 vs 0.0751 ms/step)
        return (self.device.type == "cuda" and self.dp is None and isinstance(self.opt, FusedOptimizer)
                and os.environ.get("HOPSX_OPT_COLAUNCH", "0") == "1")

    def _fwd_bwd(self, x, y):
        # every step starts from zeroed gradients (the optimizer / fused DP step zeroes them): a weight
        # used once in this forward may STORE its gradient instead of adding it (functional.STEP)
        HF.STEP["overwrite"] = self.device.type == "cuda" and os.environ.get("HOPSX_DW_STORE", "1") == "1"
        HF.STEP["uses"] = {}
        co = self._colaunch_ok()
        if co:
            from . import hooks

            HF.COLAUNCH.update(opt=self.opt, ready=set(), lo=None)
            hooks.subscribe(_mark_ready)
        try:
            out = self._forward(x)
            loss, correct, count, root, grad = HF.loss_and_grad_root(out, y, self.loss_kind)
            root.backward(grad)
        finally:
            HF.STEP["overwrite"] = False
            HF.STEP["uses"] = {}
            if co:
                hooks.unsubscribe(_mark_ready)
                HF.COLAUNCH["ready"] = None  # the optimizer step below still sees opt / lo
        HF.join_side_streams()  # gradients complete before all-reduce / optimizer
        return {"loss": loss, "correct": correct, "count": count}

    def _opt(self):
        try:
            self.opt.step()
        finally:
            HF.COLAUNCH.update(opt=None, ready=None, lo=None)
        if self.device.type != "cuda" or getattr(self.opt, "rng", None) is None:
            HF.advance_rng(self.device)  # on the GPU the optimizer kernel advances the RNG itself

    def _post(self):
        if self.dp is not None and hasattr(self.dp, "post_step"):
            self.dp.post_step()  # sharded PS: all-gather the updated weights

    def _fused(self) -> bool:
        return self.dp is not None and getattr(self.dp, "fuses_optimizer", lambda o: False)(self.opt)

    def _tail(self, eager: bool = False):
        """Gradient exchange + optimizer + post-step: the one step tail every path runs."""
        if self._fused():
            self.dp.fused_update(self.opt)  # reduce-scatter + sharded update + all-gather, one kernel
            return
        if self.dp is not None:
            if eager:
                self.dp.finish()  # completes the bucket all-reduces overlapped with backward
            else:
                self.dp.allreduce_all()
        self._opt()
        self._post()

    def _sync_hp(self):
        if hasattr(self.opt, "sync_hp"):
            self.opt.sync_hp()

    def _after_replay(self):
        if self.dp is not None and hasattr(self.dp, "poll"):
            self.dp.poll()  # P2P failure flag, checked asynchronously every poll_every steps

    def eager(self, x, y):
        r = self._fwd_bwd(x, y)
        self._tail(eager=True)
        self._after_replay()  # the P2P failure flag is polled on the eager path too
        return r

    # ------------------------------------------------------------- graph path
    def _capture(self, x, y):
        self._sx = _clone(x)
        self._sy = y.clone()
        if self._pf_pending is not None and not isinstance(self._sx, (tuple, list)):
            xs, ys = self._pf_pending
            self._pf_opt.prefetch = ([(xs, self._sx), (ys, self._sy)], self._cursor)
        world = hdist.world_size()
        overlap = None
        if self.dp is not None and hasattr(self.dp, "_on_ready"):
            overlap, self.dp.overlap = self.dp.overlap, False
            from . import hooks

            hooks.unsubscribe(self.dp._on_ready)
        pool = self._pool = torch.cuda.graph_pool_handle()
        g1 = torch.cuda.CUDAGraph()
        one_graph = world == 1 or self.dp is None or self.graph_collectives
        self._sync_hp()
        with _capture_graph(g1, pool=pool):
            out = self._fwd_bwd(self._sx, self._sy)
            if one_graph:
                self._tail()
        self._g1 = g1
        if not one_graph:
            g2 = torch.cuda.CUDAGraph()
            with _capture_graph(g2, pool=pool):
                self._opt()
            self._g2 = g2
        self._out = out
        if self._pf_opt is not None:
            self._pf_opt.prefetch = None  # only the captured optimizer kernel carries the prefetch
        if overlap is not None:
            self.dp.overlap = overlap

    def step_resident(self, xs, ys):
        """One step on an HBM-resident dataset (xs [nbatch, B, ...], ys [nbatch, B]), cycling through
        its batches.  Once the step is a replayed hipGraph, the NEXT batch is copied into the static
        input buffers by the optimizer kernel's tail (fused prefetch, optim.hip) and a device cursor
        advances in-kernel: no copy launch and no host work per step beyond the replay."""
        nb = xs.shape[0]
        if self._g1 is None or self._resident is None or self._resident[0] is not xs or self._resident[1] is not ys:
            i = self._rn % nb
            self._rn += 1
            if self.use_graph and self._n == self.warmup and self._g1 is None:
                self._arm_prefetch(xs, ys, i)
            r = self(xs[i], ys[i])
            if self._g1 is not None and self._resident is None:
                self._resident = (xs, ys)  # the graph exists and its optimizer carries the prefetch
            return r
        self._n += 1
        health.beat(self._n)
        self._replay()
        return self._out

    def _replay(self):
        self._sync_hp()
        self._g1.replay()
        if self._g2 is not None:
            self.dp.allreduce_all()
            self._g2.replay()
            self._post()
        self._after_replay()

    def _multi_ok(self, xs, ys) -> bool:
        return (self.steps_per_execution > 1 and self._g2 is None and self._g1 is not None
                and self._resident is not None and self._resident[0] is xs and self._resident[1] is ys
                and self._pf_opt is not None and self._cursor is not None)

    def _capture_multi(self, xs, ys, U: int | None = None):
        """U (default steps_per_execution) resident steps in one graph (same pool and static buffers
        as the one-step graph; each captured optimizer kernel prefetches the batch the next step
        reads).  Returns (graph, last step's outputs)."""
        U = U or self.steps_per_execution
        torch.cuda.synchronize()
        self._pf_opt.prefetch = ([(xs, self._sx), (ys, self._sy)], self._cursor)
        self._sync_hp()
        try:
            g = torch.cuda.CUDAGraph()
            outs = []
            with _capture_graph(g, pool=self._pool):
                for _ in range(U):
                    out = self._fwd_bwd(self._sx, self._sy)
                    outs.append(out)  # every step's outputs stay valid in the graph's pool (run_resident on_out)
                    self._tail()  # the same tail as the one-step graph (incl. the PS post-step)
        finally:
            self._pf_opt.prefetch = None
        torch.cuda.synchronize()
        self._outs_of[id(g)] = outs
        if U == self.steps_per_execution:
            self._gU, self._outU = g, out
        return g, out

    def prepare_resident(self, xs, ys, n: int | None = None) -> None:
        """Capture (not run) the steps_per_execution graph once the one-step graph exists, and, when
        the caller says how many steps follow (``n``), a graph for the remainder n % steps_per_execution
        — what Keras does with an epoch that is not a multiple of steps_per_execution (a 20-step run
        at 8 per execution replays 8 + 8 + 4 instead of 8 + 8 + 1 + 1 + 1 + 1)."""
        if self._gU is None and self._multi_ok(xs, ys):
            self._capture_multi(xs, ys)
        if n is not None and self._multi_ok(xs, ys):
            rem = n % self.steps_per_execution
            if rem > 1 and rem not in self._gR:
                self._gR[rem] = self._capture_multi(xs, ys, rem)

    def _replay_multi(self, g, U: int, on_out=None):
        health.beat_range(self._n + 1, U)  # one heartbeat (and fault check) for the U replayed steps
        self._n += U
        self._sync_hp()
        g.replay()
        self._after_replay()
        if on_out is not None:
            on_out(self._outs_of[id(g)])

    def run_resident(self, xs, ys, n: int, on_out=None):
        """``n`` consecutive steps on the resident epoch (see step_resident); returns the last
        step's outputs.  Single-GPU and P2P data-parallel graph steps run ``steps_per_execution`` at
        a time (a prepared remainder graph takes the tail).  ``on_out(list of outputs)`` receives EVERY
        step's outputs, once per launch (a replayed graph's U steps together), right after it (device
        tensors: e.g. keras.fit's epoch loss / accuracy totals, a few small ops per launch)."""
        r = None
        rem = n % self.steps_per_execution
        if n > self.steps_per_execution and rem in self._gR and self._multi_ok(xs, ys):
            # the short remainder graph first: its launch is cheaper, so the GPU starts sooner and the
            # full graphs are issued while it runs
            g, r = self._gR[rem]
            self._replay_multi(g, rem, on_out)
            n -= rem
        while n > 0:
            if n in self._gR and n < self.steps_per_execution and self._multi_ok(xs, ys):
                g, r = self._gR[n]
                self._replay_multi(g, n, on_out)
                n = 0
                continue
            if n < self.steps_per_execution or not self._multi_ok(xs, ys):
                r = self.step_resident(xs, ys)
                if on_out is not None:
                    on_out([r])
                n -= 1
                continue
            if self._gU is None:
                self._capture_multi(xs, ys)
            self._replay_multi(self._gU, self.steps_per_execution, on_out)
            n -= self.steps_per_execution
            r = self._outU
        return r

    def _arm_prefetch(self, xs, ys, i):
        opt = self.opt.opts[-1] if hasattr(self.opt, "opts") else self.opt
        if not hasattr(opt, "prefetch") or xs.device.type != "cuda":
            return
        # the capture clones xs[i] / ys[i] into the static buffers; the cursor says which batch they hold
        self._cursor = torch.full((1,), i, device=xs.device, dtype=torch.int64)
        self._pf_opt = opt
        self._pf_pending = (xs, ys)

    def __call__(self, x, y):
        self._n += 1
        health.beat(self._n)  # progress heartbeat for the launcher's watchdog (+ HOPSX_FAULT injection)
        if not self.use_graph or self._n <= self.warmup or (
                self._sx is not None and (_shape(x) != _shape(self._sx) or y.shape != self._sy.shape)):
            return self.eager(x, y)  # warm-up, or a ragged (e.g. last) batch the graph was not captured for
        if self._g1 is None:
            torch.cuda.synchronize()
            self._capture(x, y)
            torch.cuda.synchronize()
        if not _same_storage(x, self._sx):
            _copy_into(self._sx, x)
            self._sy.copy_(y, non_blocking=True)
        self._replay()
        return self._out


def make_step(model, optimizer, loss_kind: str = "sparse_ce", dp="auto", graph: bool = True, batch: int | None = None,
              **kw):
    """The training-step engine for ``model``: the persistent whole-step kernel
    (runtime/persist.py PersistentMnistStep: one launch per 32 steps, ~3x the multi-kernel engine on the
    reference's MirroredStrategy MNIST CNN) whenever ``PersistentMnistStep.supported`` holds for this
    model / optimizer / per-replica ``batch`` / world size and the ranks drive distinct GPUs — with N
    ranks it exchanges activations and gradients over xGMI inside the launch, after a collective
    self-test; otherwise a :class:`TrainStep` (hipGraph replays, fused optimizer, ``dp``).

    ``dp``: "auto" builds the engine of ``HOPSX_DP_MODE`` (``parallel.ps.make``: DataParallel, or ShardedPS
    for parameter_server, which never takes the persistent path) when the process group has > 1 rank and
    the TrainStep path is taken; None or an engine object is passed through to TrainStep as is.
    ``engine.kind`` says which one was built ("persistent" / "trainstep")."""
    from ..parallel import dist as hdist

    world = hdist.world_size()
    note = None
    if isinstance(dp, str) and dp == "auto" and os.environ.get("HOPSX_DP_MODE", "mirrored") == "parameter_server":
        from ..parallel import ps

        dp = ps.make(model, optimizer) if world > 1 else None
        note = "parameter_server mode"
    dev = getattr(getattr(optimizer, "arena", None), "device", None)
    if (batch is not None and graph and loss_kind == "sparse_ce" and dev is not None and dev.type == "cuda"
            and (dp is None or (isinstance(dp, str) and dp == "auto"))):
        from .persist import PersistentMnistStep, flagship_layers, launchable

        if PersistentMnistStep.supported(model, optimizer, int(batch), world):
            from ..parallel import oneshot

            if world == 1 or oneshot._colocation(dev) == 1:
                try:
                    eng = PersistentMnistStep(model, optimizer, steps_per_launch=int(kw.get("steps_per_execution", 32)))
                except RuntimeError as e:  # raised on every rank alike (collective setup)
                    eng, note = None, f"persistent setup failed: {e}"[:300]
                if eng is not None and (world == 1 or eng.selftest()):
                    eng.kind, eng.note = "persistent", None
                    return eng
                if eng is not None:
                    eng.close()
                    note = "persistent selftest failed"
            else:
                note = "ranks share a GPU: the persistent step needs one GPU per rank"
        elif flagship_layers(model) is not None:
            ok, why = launchable(dev, world)
            note = f"persistent step not launchable: {why}" if not ok else "persistent step not supported here"
    if isinstance(dp, str) and dp == "auto":
        from ..parallel import ps

        dp = ps.make(model, optimizer) if world > 1 else None
    st = TrainStep(model, optimizer, loss_kind, dp=dp, graph=graph, **kw)
    st.kind, st.note = "trainstep", note
    return st
