"""Fused optimizers over a ParamArena: ONE kernel launch per step for the
whole model (update + bf16 shadow refresh + gradient zeroing), with the step
counter on the device so the step can be captured into a hipGraph.

Defaults follow the frameworks the reference notebooks use:
Keras ``Adadelta(1.0)`` (rho 0.95, eps 1e-7; notebooks/ml/Experiment/Tensorflow/mnist.ipynb:176),
``torch.optim.SGD(lr=0.01, momentum=0.5)`` (notebooks/ml/Experiment/PyTorch/mnist.ipynb:207),
Keras ``Adam`` / ``RMSprop(0.2)`` (notebooks/ml/Benchmarks/benchmark.ipynb:154),
TF ``FtrlOptimizer`` for the census LinearClassifier (feature-bias-whatif.ipynb:458-463).
"""
from __future__ import annotations

import math

import torch

from .ops._C import OPTIM
from .runtime.arena import ALIGN, ParamArena

ARRIVE_WORDS = 9 * 32  # csrc/ops/optim_core.h kArriveWords


def _arena_of(obj) -> ParamArena:
    if isinstance(obj, ParamArena):
        return obj
    if isinstance(obj, torch.nn.Module):
        a = getattr(obj, "_hx_arena", None)
        if a is not None:
            return a
        params = [p for p in obj.parameters() if p.requires_grad]
        a = getattr(params[0], "_hx_arena", None) if params else None
        if a is not None and all(getattr(p, "_hx_arena", None) is a for p in params):
            return a  # a sub-module of a model whose arena already exists
        return ParamArena.from_module(obj)
    params = list(obj)
    arenas = {id(getattr(p, "_hx_arena", None)) for p in params}
    if len(arenas) == 1 and getattr(params[0], "_hx_arena", None) is not None:
        return params[0]._hx_arena
    return ParamArena(params)


def _range_of(arena: ParamArena, obj) -> slice:
    """The contiguous slice of the arena an optimizer owns: everything, or the span of a
    sub-module / parameter subset (wide & deep: FTRL on the wide part, Adagrad on the deep)."""
    if isinstance(obj, ParamArena) or (isinstance(obj, torch.nn.Module) and getattr(obj, "_hx_arena", None) is arena):
        return slice(0, arena.numel)
    params = [p for p in (obj.parameters() if isinstance(obj, torch.nn.Module) else obj) if p.requires_grad]
    ids = {id(p) for p in params}
    if ids == {id(p) for p in arena.params}:
        return slice(0, arena.numel)
    lo = min(p._hx_off for p in params)
    hi = max(p._hx_off + -(-p.numel() // ALIGN) * ALIGN for p in params)
    for p, o, _ in arena.ranges():
        if lo <= o < hi and id(p) not in ids:
            raise ValueError("optimizer parameter subset must be contiguous in the arena (register it as one "
                             "sub-module)")
    return slice(lo, hi)


class FusedOptimizer:
    kind = "sgd"
    nstate = 0

    def __init__(self, params, lr, weight_decay=0.0, **hp):
        self.arena = _arena_of(params)
        self._sl = _range_of(self.arena, params)
        self.lr = float(lr)
        self.weight_decay = float(weight_decay)
        self.hp = hp
        self.grad_scale = 1.0
        self.prefetch = None  # (pairs, cursor): fused next-batch copy of a resident dataset (TrainStep)
        dev = self.arena.device
        self.step_count = torch.zeros(1, device=dev, dtype=torch.float32)
        # arrival counter of the in-kernel step bookkeeping: 8 per-XCD shards + top word (optim_core.h)
        self._arrive = torch.zeros(ARRIVE_WORDS, device=dev, dtype=torch.int32)
        # device RNG state advanced by the optimizer kernel's last workgroup (dropout masks)
        self.rng = None
        if dev.type == "cuda":
            from .ops.functional import rng_state

            self.rng = rng_state(dev)
        self._states = [self.arena.state(f"{self.kind}_s{i}")[self._sl] for i in range(self.nstate)]
        self.param_groups = [{"params": self.arena.params, "lr": self.lr}]
        # device copy of the hyper-parameter vector: the kernel reads it at run time, so a step
        # replayed from a hipGraph sees lr / grad_scale changes made after the capture (sync_hp)
        self._hp_dev = torch.zeros(8, device=dev, dtype=torch.float32) if dev.type == "cuda" else None
        self._hp_up = None

    def restrict(self, sl: slice) -> "FusedOptimizer":
        """Own only ``sl`` of the arena (sharded parameter-server mode: each rank updates its shard)."""
        self._sl = sl
        self._states = [self.arena.state(f"{self.kind}_s{i}")[sl] for i in range(self.nstate)]
        return self

    # hyper-parameter vector in the kernel's layout: lr, gscale, wd, a..e
    def _hp(self) -> list[float]:
        raise NotImplementedError

    def sync_hp(self) -> None:
        """Upload the hyper-parameters if they changed since the last upload (stream-ordered; never
        during a hipGraph capture — TrainStep calls this before every replay)."""
        if self._hp_dev is None:
            return
        self.lr = self.param_groups[0]["lr"]
        hp = [float(v) for v in self._hp()]
        # (compared first: the capture query is a runtime call, and this runs before every launch / replay)
        if hp != self._hp_up and not torch.cuda.is_current_stream_capturing():
            self._hp_dev.copy_(torch.tensor((hp + [0.0] * 8)[:8], dtype=torch.float32))
            self._hp_up = hp

    def step(self, closure=None):
        from .ops.functional import join_side_streams

        join_side_streams()  # weight gradients still running on the parallel branch
        loss = closure() if closure is not None else None
        self.lr = self.param_groups[0]["lr"]
        a = self.arena
        s = self._states + [None] * (3 - len(self._states))
        if self._sl.stop <= self._sl.start:  # empty shard (sharded PS mode): nothing to update
            self.step_count += 1
            return loss
        if a.device.type == "cuda":
            from .ops import functional as HF
            from .ops import kernels as K

            sl = self._sl
            if HF.COLAUNCH["opt"] is self and HF.COLAUNCH["lo"] is not None:
                # the slice [lo, stop) was updated by the last backward launch (optim_slice.h):
                # this launch updates the prefix and does the step bookkeeping / prefetch
                lo = HF.COLAUNCH["lo"]
                HF.COLAUNCH["lo"] = None
                s = [t[: lo - sl.start] if t is not None else None for t in s]
                sl = slice(sl.start, lo)
            self.sync_hp()
            K.optim_step(OPTIM[self.kind], a.master[sl], a.grad[sl], s[0], s[1], s[2],
                         a.shadow[sl] if a.shadow is not None else None, self._hp(), self.step_count,
                         zero_grad=True, arrive=self._arrive, rng=self.rng, prefetch=self.prefetch,
                         hp_dev=self._hp_dev)
        else:
            self.step_count += 1
            sl = self._sl
            with torch.no_grad():
                self._cpu_step(a.master[sl], a.grad[sl] * self.grad_scale, s, float(self.step_count.item()))
                a.grad[sl].zero_()
            if a.shadow is not None:
                a.refresh_shadow()
        return loss

    def zero_grad(self, set_to_none: bool = False):
        self.arena.zero_grad()

    def state_dict(self):
        return {"step": self.step_count.cpu(), "lr": self.lr, "states": [t.cpu() for t in self._states]}

    def load_state_dict(self, sd):
        self.step_count.copy_(sd["step"])
        self.lr = sd["lr"]
        self.param_groups[0]["lr"] = self.lr
        for t, v in zip(self._states, sd["states"]):
            t.copy_(v)

    def _cpu_step(self, p, g, s, t):  # pragma: no cover - overridden
        raise NotImplementedError


class SGD(FusedOptimizer):
    kind, nstate = "sgd", 1

    def __init__(self, params, lr=0.01, momentum=0.0, dampening=0.0, nesterov=False, weight_decay=0.0):
        super().__init__(params, lr, weight_decay, momentum=momentum, dampening=dampening, nesterov=nesterov)

    def _hp(self):
        h = self.hp
        return [self.lr, self.grad_scale, self.weight_decay, h["momentum"], h["dampening"], float(h["nesterov"])]

    def _cpu_step(self, p, g, s, t):
        h = self.hp
        g = g + self.weight_decay * p
        if h["momentum"]:
            s[0].mul_(h["momentum"]).add_(g, alpha=1 - h["dampening"])
            g = g + h["momentum"] * s[0] if h["nesterov"] else s[0]
        p.sub_(self.lr * g)


class Adam(FusedOptimizer):
    kind, nstate = "adam", 2

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0):
        super().__init__(params, lr, weight_decay, b1=betas[0], b2=betas[1], eps=eps)

    def _hp(self):
        h = self.hp
        return [self.lr, self.grad_scale, self.weight_decay, h["b1"], h["b2"], h["eps"]]

    def _cpu_step(self, p, g, s, t):
        h = self.hp
        if self.kind == "adam":
            g = g + self.weight_decay * p
        else:
            p.mul_(1 - self.lr * self.weight_decay)
        s[0].mul_(h["b1"]).add_(g, alpha=1 - h["b1"])
        s[1].mul_(h["b2"]).addcmul_(g, g, value=1 - h["b2"])
        bc1, bc2 = 1 - h["b1"] ** t, 1 - h["b2"] ** t
        p.sub_(self.lr * (s[0] / bc1) / ((s[1] / bc2).sqrt() + h["eps"]))


class AdamW(Adam):
    kind = "adamw"

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2):
        super().__init__(params, lr, betas, eps, weight_decay)


class Adadelta(FusedOptimizer):
    kind, nstate = "adadelta", 2

    def __init__(self, params, lr=1.0, rho=0.95, eps=1e-7, weight_decay=0.0):
        super().__init__(params, lr, weight_decay, rho=rho, eps=eps)

    def _hp(self):
        return [self.lr, self.grad_scale, self.weight_decay, self.hp["rho"], self.hp["eps"]]

    def _cpu_step(self, p, g, s, t):
        rho, eps = self.hp["rho"], self.hp["eps"]
        g = g + self.weight_decay * p
        s[0].mul_(rho).addcmul_(g, g, value=1 - rho)
        delta = (s[1] + eps).sqrt() / (s[0] + eps).sqrt() * g
        s[1].mul_(rho).addcmul_(delta, delta, value=1 - rho)
        p.sub_(self.lr * delta)


class RMSprop(FusedOptimizer):
    kind, nstate = "rmsprop", 3

    def __init__(self, params, lr=1e-3, alpha=0.9, eps=1e-7, momentum=0.0, centered=False, weight_decay=0.0):
        super().__init__(params, lr, weight_decay, alpha=alpha, eps=eps, momentum=momentum, centered=centered)

    def _hp(self):
        h = self.hp
        return [self.lr, self.grad_scale, self.weight_decay, h["alpha"], h["eps"], h["momentum"], float(h["centered"])]

    def _cpu_step(self, p, g, s, t):
        h = self.hp
        g = g + self.weight_decay * p
        s[0].mul_(h["alpha"]).addcmul_(g, g, value=1 - h["alpha"])
        if h["centered"]:
            s[2].mul_(h["alpha"]).add_(g, alpha=1 - h["alpha"])
            avg = (s[0] - s[2] * s[2]).clamp_min(0).sqrt() + h["eps"]
        else:
            avg = s[0].sqrt() + h["eps"]
        if h["momentum"]:
            s[1].mul_(h["momentum"]).add_(g / avg)
            p.sub_(self.lr * s[1])
        else:
            p.sub_(self.lr * g / avg)


class Adagrad(FusedOptimizer):
    kind, nstate = "adagrad", 1

    def __init__(self, params, lr=0.01, eps=1e-10, initial_accumulator_value=0.0, weight_decay=0.0):
        super().__init__(params, lr, weight_decay, eps=eps)
        self.initial_accumulator_value = float(initial_accumulator_value)  # the accumulator's floor
        if initial_accumulator_value:
            self._states[0].fill_(initial_accumulator_value)

    def _hp(self):
        return [self.lr, self.grad_scale, self.weight_decay, self.hp["eps"]]

    def _cpu_step(self, p, g, s, t):
        g = g + self.weight_decay * p
        s[0].addcmul_(g, g)
        p.sub_(self.lr * g / (s[0].sqrt() + self.hp["eps"]))


class Ftrl(FusedOptimizer):
    """FTRL-proximal with lr_power = -0.5 (TF FtrlOptimizer defaults)."""

    kind, nstate = "ftrl", 2

    def __init__(self, params, lr=0.2, l1=0.0, l2=0.0, beta=0.0, initial_accumulator_value=0.1):
        super().__init__(params, lr, 0.0, l1=l1, l2=l2, beta=beta)
        self._states[1].fill_(initial_accumulator_value)

    def _hp(self):
        h = self.hp
        return [self.lr, self.grad_scale, 0.0, h["l1"], h["l2"], h["beta"]]

    def _cpu_step(self, p, g, s, t):
        h = self.hp
        nn_ = s[1] + g * g
        sigma = (nn_.sqrt() - s[1].sqrt()) / self.lr
        s[0].add_(g - sigma * p)
        s[1].copy_(nn_)
        z = s[0]
        new = -(z - torch.sign(z) * h["l1"]) / ((h["beta"] + nn_.sqrt()) / self.lr + 2 * h["l2"])
        p.copy_(torch.where(z.abs() <= h["l1"], torch.zeros_like(p), new))


class Chain:
    """Several fused optimizers over disjoint slices of one arena, stepped together
    (one kernel launch each) — e.g. FTRL for a wide part + Adagrad for a deep part."""

    def __init__(self, *opts: FusedOptimizer):
        self.opts = list(opts)
        self.arena = opts[0].arena
        self.rng = opts[0].rng
        self.param_groups = [g for o in opts for g in o.param_groups]

    @property
    def grad_scale(self):
        return self.opts[0].grad_scale

    @grad_scale.setter
    def grad_scale(self, v):
        for o in self.opts:
            o.grad_scale = v

    def sync_hp(self) -> None:
        for o in self.opts:
            o.sync_hp()

    def restrict(self, sl: slice) -> "Chain":
        for o in self.opts:
            lo, hi = max(o._sl.start, sl.start), min(o._sl.stop, sl.stop)
            o.restrict(slice(lo, max(lo, hi)))
        return self

    def step(self, closure=None):
        loss = closure() if closure is not None else None
        for o in self.opts:
            o.step()
        return loss

    def zero_grad(self, set_to_none: bool = False):
        self.arena.zero_grad()

    def state_dict(self):
        return {"opts": [o.state_dict() for o in self.opts]}

    def load_state_dict(self, sd):
        for o, s in zip(self.opts, sd["opts"]):
            o.load_state_dict(s)


_BY_NAME = {"sgd": SGD, "adam": Adam, "adamw": AdamW, "adadelta": Adadelta, "rmsprop": RMSprop, "adagrad": Adagrad,
            "ftrl": Ftrl}


def get(name: str, params, **kw) -> FusedOptimizer:
    return _BY_NAME[name.lower()](params, **kw)


def cosine_lr(base, step, total, warmup=0):
    if step < warmup:
        return base * (step + 1) / warmup
    return 0.5 * base * (1 + math.cos(math.pi * (step - warmup) / max(1, total - warmup)))
