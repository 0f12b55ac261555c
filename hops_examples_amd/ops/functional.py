"""Autograd-integrated ops backed by the gfx950 kernels.

GPU path (tensors on ``cuda``): bf16 NHWC activations, MFMA kernels, weight
gradients accumulated straight into the ParamArena grad buffer (the Function
returns ``None`` for arena-managed weights and notifies the data-parallel
engine that the gradient is ready, so bucketed all-reduce can start while the
rest of the backward runs).

CPU path: plain fp32 PyTorch with the same NHWC semantics — used by the CPU
test-suite and the ``experiment.launch`` CPU config (BASELINE.json config 1).
"""
from __future__ import annotations

import os
import weakref

import torch
import torch.nn.functional as F

from ..runtime import arena as _arena
from ..runtime import hooks
from . import kernels as K
from ._C import ACT, LOSS

BF16 = torch.bfloat16
F32 = torch.float32


def _cpu_act(y, act):
    a = ACT[act] if not isinstance(act, int) else act
    if a == 1:
        return F.relu(y)
    if a == 2:
        return torch.sigmoid(y)
    if a == 3:
        return torch.tanh(y)
    return y


def _wgrad_buf(p):
    g = _arena.grad_target(p)
    if g is None:
        # a zero-at-rest buffer the weight's producer keeps (the padded image-stem weight, _PadCinFn),
        # else a fresh zeroed one
        g = getattr(p, "_hx_wbuf", None)
        if g is None:
            g = torch.zeros(p.shape, device=p.device, dtype=torch.float32)
    return g


def _ret_grad(p, buf):
    """Return value for a weight's gradient: None when it went into the arena."""
    if p is None or not p.requires_grad:
        return None
    hooks.grad_ready(p)
    return None if _arena.grad_target(p) is buf else buf


# ------------------------------------------------- parallel weight gradients (graph branches)
# In a layer's backward the weight gradient and the input gradient are independent GEMMs over the
# same dY.  At small batch each is a latency-bound launch, so the weight gradient is issued on a
# side stream (fork: side waits for the main stream) and runs concurrently with the dgrad chain
# of the main stream; captured into a hipGraph this becomes a parallel branch.  The branch is
# joined before anything reads the gradients (FusedOptimizer.step, TrainStep, DP all-reduce).
# Only kernels that keep no shared workspace / ticket counter go on the side stream, and none
# when DP overlap hooks are subscribed (those fire per gradient on the main stream).
_SIDE: dict = {}
_PENDING: dict = {}  # device -> the main stream that forked (joined back by join_side_streams)


def _side_stream(device):
    if device.type != "cuda" or hooks._subscribers or "par_wgrad" in _disabled():
        return None
    s = _SIDE.get(device)
    if s is None:
        s = torch.cuda.Stream(device=device)
        _SIDE[device] = s
    return s


_PAR_MIN_FLOP = float(os.environ.get("HOPSX_PAR_WGRAD_MIN_FLOP", "2e9"))


class _on_side:
    """``with _on_side(dev, *tensors, flop=F):`` runs the block on the side stream when the weight
    gradient is big enough to win (F >= HOPSX_PAR_WGRAD_MIN_FLOP, default 2 GFLOP), else inline.
    Measured: a cross-queue dependency in a replayed hipGraph costs ~10 us and a multi-queue graph
    loses the back-to-back dispatch of its single-queue chain, so latency-bound models (MNIST at
    batch 32, CIFAR ResNets) stay single-stream while ResNet-50 at batch 64 gains ~6 %."""

    def __init__(self, device, *tensors, flop: float = float("inf")):
        self.side = _side_stream(device) if flop >= _PAR_MIN_FLOP else None
        self.tensors = [t for t in tensors if t is not None]
        self.device = device

    def __enter__(self):
        if self.side is None:
            return self
        self.main = torch.cuda.current_stream(self.device)
        self.side.wait_stream(self.main)
        for t in self.tensors:
            t.record_stream(self.side)
        self._ctx = torch.cuda.stream(self.side)
        self._ctx.__enter__()
        return self

    def __exit__(self, *exc):
        if self.side is not None:
            self._ctx.__exit__(*exc)
            if self.device not in _PENDING:
                _PENDING[self.device] = self.main
                try:  # join at the end of this backward pass (also inside user-captured graphs)
                    torch.autograd.Variable._execution_engine.queue_callback(join_side_streams)
                except RuntimeError:
                    pass  # not inside a backward pass: the caller joins (optimizer / TrainStep)
        return False


def join_side_streams() -> None:
    """Make the forking (main) stream wait for every outstanding side-stream weight gradient."""
    while _PENDING:
        dev, main = _PENDING.popitem()
        main.wait_stream(_SIDE[dev])


def to_compute(x: torch.Tensor) -> torch.Tensor:
    """Move an activation to the compute dtype of its device (bf16 on GPU)."""
    if x.is_cuda and x.dtype != BF16:
        if x.dtype == torch.uint8:
            return K.u8_normalize(x.contiguous(), 1.0, 0.0)
        return x.to(BF16)
    return x.contiguous()


# ===================================================================== Linear
# Single-contribution weight gradients (set by runtime.step.TrainStep around one step's forward +
# backward, whose gradients start zeroed): "uses" counts the forward uses of each weight, and a
# Linear whose weight was used once STORES its dW instead of adding it with float atomics.
STEP = {"overwrite": False, "uses": {}}


def _note_use(w) -> None:
    if STEP["overwrite"]:
        STEP["uses"][id(w)] = STEP["uses"].get(id(w), 0) + 1


def _sole_use(w) -> bool:
    return STEP["overwrite"] and STEP["uses"].get(id(w), 0) == 1


class _LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, act, out_f32, pool=None):
        ctx.pool = pool
        _note_use(w)
        x2 = x.reshape(-1, x.shape[-1]).contiguous()
        wb = _arena.weight_bf16(w)
        if PREHEAD["arm"]:
            # deferred: the fused loss kernel (mlp_head) fills y before anything reads it
            y = torch.empty(x2.shape[0], w.shape[0], device=x2.device, dtype=BF16)
            PREHEAD["last"] = (x2, wb, b, act, y)
        else:
            y = K.linear_fwd(x2, wb, b, act=act, out_f32=out_f32)
        ctx.save_for_backward(x2, y)
        ctx.w, ctx.b, ctx.act, ctx.xshape = w, b, act, x.shape
        return y.view(*x.shape[:-1], y.shape[-1])

    @staticmethod
    def backward(ctx, dy):
        x2, y = ctx.saved_tensors
        w, b, act = ctx.w, ctx.b, ctx.act
        dy2 = dy.reshape(-1, dy.shape[-1])
        if dy2.dtype != BF16:
            dy2 = dy2.to(BF16)
        dy2 = dy2.contiguous()
        gb = _wgrad_buf(b) if b is not None else None
        # the activation backward is fused into the A-operand staging of both GEMMs and
        # the bias gradient falls out of the weight-gradient GEMM (no elementwise passes)
        ymask = y if (act and y.dtype == BF16) else None
        dx = None
        gw = _wgrad_buf(w)
        wflop = 2.0 * dy2.numel() * x2.shape[1]
        if ctx.needs_input_grad[0] and wflop < _PAR_MIN_FLOP and "bwd_pair" not in _disabled():
            # small layer: dgrad and wgrad (+ bias grad) as ONE launch (horizontal fusion); when the
            # input is a flattened max-pool output, the dgrad epilogue also does the pool backward
            # (4x4 and bigger windows: the separate per-input-pixel pool backward, maxpool_bwdv_k, writes the
            # pool input as 16-B vectors; the scatter's per-element window stores measured 18.6 vs 5.7 + 6.6 us
            # on the E1 model, profiles/r6_e1_fit_kernels.txt)
            pool = ctx.pool if "pool_scatter" not in _disabled() and (ctx.pool is None or
                                                                      ctx.pool[3][0] * ctx.pool[3][1] <= 4) else None
            r = K.linear_bwd_pair(dy2, _arena.weight_bf16(w), x2, gw, y=ymask, act=act, dbias=gb, pool=pool,
                                  dw_store=_sole_use(w) and gw is _arena.grad_target(w))
            if r is not False:
                if pool is not None:
                    # r is the pool-INPUT gradient: hand autograd an unfilled placeholder for this
                    # layer's input and let the pool backward return r (registry keyed by address)
                    ph = torch.empty(ctx.xshape, device=dy2.device, dtype=BF16)
                    _PRESCATTERED[ph.data_ptr()] = (weakref.ref(ph), r, bool(pool[8]))
                    dxr = ph
                else:
                    dxr = r.view(ctx.xshape)
                return (dxr, _ret_grad(w, gw), (_ret_grad(b, gb) if b is not None else None), None, None, None)
        with _on_side(dy2.device, dy2, x2, ymask, flop=wflop):  # wgrad || dgrad
            K.linear_wgrad(dy2, x2, gw, y=ymask, act=act, dbias=gb)
        if ctx.needs_input_grad[0]:
            dx = K.linear_dgrad(dy2, _arena.weight_bf16(w), y=ymask, act=act).view(ctx.xshape)
        return dx, _ret_grad(w, gw), (_ret_grad(b, gb) if b is not None else None), None, None, None


def linear(x, w, b=None, act=None, out_f32=False, drop_in=None):
    """y = act(x @ w.T + b); w is [out, in] (fp32 master; bf16 shadow used on GPU).  ``drop_in`` = (p, salt):
    a training-mode Dropout applied to ``x`` first (keras.Sequential hands a Dense -> Dropout -> logits Dense
    chain's dropout to the logits layer): when this layer's forward is deferred to the fused loss kernel,
    the kernel applies it (loss.hip head_ce_k dp), so neither dropout launch runs."""
    if drop_in is not None and drop_in[0] <= 0:
        drop_in = None
    if not x.is_cuda:
        if drop_in is not None:
            x = F.dropout(x.float(), drop_in[0], True)
        return _cpu_act(F.linear(x.float(), w, b), act)
    a = ACT[act] if not isinstance(act, int) else act
    xc = to_compute(x)
    src = x if hasattr(x, "_hx_pool") else getattr(x, "_base", None)
    pool = getattr(src, "_hx_pool", None) if src is not None and src.numel() == x.numel() else None
    head = (not a and x.dim() == 2 and w.shape[0] <= 32 and xc.dtype == BF16 and torch.is_grad_enabled()
            and w.requires_grad and _arena.grad_target(w) is not None
            and (b is None or _arena.grad_target(b) is not None))
    if head and HEAD["defer"] and "head_fwd" not in _disabled() and K.head_ce_ok(w.shape[0], x.shape[1]) and (
            drop_in is None or "head_drop" not in _disabled()):
        # deferred logits layer (TrainStep verified that these logits are the model's output and
        # only feed the loss): no forward launch — the loss kernel computes and stores the logits
        # (and applies the dropout on its input, drop_in)
        y = torch.empty(x.shape[0], w.shape[0], device=x.device, dtype=F32 if out_f32 else BF16)
        drop = (float(drop_in[0]), rng_state(x.device), int(drop_in[1])) if drop_in is not None else None
        y._hx_dense_head = (xc, w, b, out_f32, True, drop)
        return y
    if drop_in is not None:
        xc = dropout(xc, float(drop_in[0]), True, int(drop_in[1]))
    if PREHEAD["pending"] and xc.data_ptr() in PREHEAD["pending"]:
        flush_pending()  # a deferred pre-head output read by anything but the deferred head
    pre = (HEAD["defer"] and PREHEAD["w"] is w and not head and a in (0, 1) and xc.dim() == 2 and xc.dtype == BF16
           and xc.shape[0] <= 32 and not out_f32 and torch.is_grad_enabled() and "prehead" not in _disabled())
    PREHEAD["arm"] = pre
    try:
        y = _LinearFn.apply(xc, w, b, a, out_f32, pool)
    finally:
        PREHEAD["arm"] = False
    if pre:
        PREHEAD["pending"][y.data_ptr()] = PREHEAD.pop("last")
    if head and y.requires_grad:
        y._hx_dense_head = (xc, w, b, out_f32, False)  # logits layer: loss_and_grad can fuse its backward
        if HEAD["probe"] is not None:
            HEAD["probe"].append(y)
            last = HEAD.get("last_lin")
            # the layer right before the logits layer: a Linear whose output is exactly the head's input
            HEAD["prehead_w"] = last[0] if last is not None and last[1] is x else None
    elif HEAD["probe"] is not None:
        HEAD["last_lin"] = (w, y) if (a in (0, 1) and y.dim() == 2 and not out_f32) else None
    return y


# logits-layer deferral (set by runtime.step.TrainStep): "probe" collects the head-candidate
# outputs of one forward; "defer" lets linear() skip the head's forward launch (head_ce computes it)
HEAD = {"probe": None, "defer": False}

# Pre-head deferral (also TrainStep): the Linear layer whose output feeds ONLY the deferred logits
# layer (found by the probe: weight ``w``) launches nothing in its forward either; the loss call
# runs it together with the head as ONE kernel (loss.hip mlp_head_k).  ``pending`` maps the
# placeholder output's address to its forward operands until then; anything else that reads a
# placeholder first gets it computed (flush_pending).
PREHEAD = {"w": None, "arm": False, "pending": {}}

# Optimizer co-launch (set by runtime.step.TrainStep on one GPU with a fused optimizer): the last
# backward launch (the input-side conv pair) also runs the optimizer's update of the arena slice
# whose gradients are already final (csrc/ops/optim_slice.h); ``lo`` = where that slice starts once
# launched, so the optimizer's own launch updates only [start, lo).  ``ready``: ids of the
# parameters whose gradients are final (hooks.grad_ready during this backward).
COLAUNCH = {"opt": None, "ready": None, "lo": None, "launched": 0}


def _colaunch_slice(own):
    """(lo, slice tuple for K.conv2d_bwd_pair) when the registered optimizer can update the arena
    suffix whose gradients are final, excluding ``own`` (the params this launch produces)."""
    opt = COLAUNCH["opt"]
    if (opt is None or COLAUNCH["ready"] is None or COLAUNCH["lo"] is not None or _PENDING
            or "opt_colaunch" in _disabled()):
        return None
    arena, sl = opt.arena, opt._sl
    ready, own_ids = COLAUNCH["ready"], {id(p) for p in own if p is not None}
    lo = sl.stop
    for p, o, _ in sorted(arena.ranges(), key=lambda r: -r[1]):
        if o >= sl.stop:
            continue
        if o < sl.start or id(p) not in ready or id(p) in own_ids:
            break
        lo = o
    if lo >= sl.stop or lo % 64:
        return None
    from ._C import OPTIM

    opt.sync_hp()
    off = lo - sl.start
    st = [t[off:] for t in opt._states] + [None] * (3 - len(opt._states))
    sh = arena.shadow[lo:sl.stop] if arena.shadow is not None else None
    return lo, (OPTIM[opt.kind], arena.master[lo:sl.stop], arena.grad[lo:sl.stop], st[0], st[1], st[2], sh,
                opt._hp(), opt._hp_dev, opt.step_count)


def flush_pending() -> None:
    """Compute every deferred pre-head output now (the unfused path)."""
    while PREHEAD["pending"]:
        _, (x2, wb, b, act, y) = PREHEAD["pending"].popitem()
        K.linear_fwd(x2, wb, b, act=act, out=y)


# ===================================================================== Conv2d
def _pad_same(k, d=1):
    tot = d * (k - 1)
    return tot // 2


# HOPSX_PLAIN_GEMM=blaslt: the epilogue-free 1x1 convs' forward / dgrad on the vendor library GEMM
# (torch.mm -> hipBLASLt) instead of the hopsx kernels (gg engine where it fills the chip)
_PLAIN_LIB = os.environ.get("HOPSX_PLAIN_GEMM", "hopsx") == "blaslt"


def _plain_gemm_conv(g, b, act, in_affine, prev) -> bool:
    """A 1x1 / stride-1 / unpadded conv with no epilogue (bias, activation) and no fused input layer
    is a plain GEMM over [B*H*W, C] x [C, CO]: forward and dgrad run as dense GEMMs on the hopsx
    kernels (gg engine, gemm_glds.h; the dgrad epilogue adds a shortcut's gradient), or on the
    vendor library with HOPSX_PLAIN_GEMM=blaslt; the weight gradient (a K = B*H*W reduction) stays
    on the hopsx kernels (HOPSX_BLASLT_WGRAD=1 to compare the library's fp32-out path)."""
    B, H, W, C, OH, OW, CO, KH, KW, sh, sw, ph, pw = g[:13]
    return (KH == 1 and KW == 1 and sh == 1 and sw == 1 and ph == 0 and pw == 0 and b is None and not act
            and in_affine is None and prev is None and B * H * W >= _PLAIN_MIN_PX and C % 8 == 0 and CO % 8 == 0
            and "blaslt_1x1" not in _disabled())


class _Conv2dFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, stride, padding, dilation, act, in_affine=None, prev=None, pool=None, bnstats=False,
                gslot=None):
        g = K.conv_geom(x.shape, w.shape, stride, padding, dilation)
        ctx.pool = None
        ctx.give = None
        ctx.bnin = _take_bn_input(x)  # x is a training BN's output consumed only here (bn_sole_consumer)
        if isinstance(gslot, GiveGrad):
            ctx.give, gslot = gslot.slot, None
        # gslot: a dict through which a later-backpropagated consumer of x (a ResNet block's identity
        # shortcut, _BNFn) hands over its gradient of x; this dgrad adds it (in the epilogue where
        # the kernel has one) instead of autograd launching an add
        ctx.gslot = gslot
        fold = _take_bn_fold(x)  # x: a batch_norm(fold_next=True) output whose apply has not run yet
        if bnstats and x.dtype == BF16 and b is None and not act and in_affine is None and _bnstats_conv(g):
            # the output feeds a training BatchNorm: the conv epilogue accumulates its statistics
            # (no statistics pass over y); the BN then runs bn_fwd_apply_fin
            x = x.contiguous()
            y = None
            if fold is not None:
                # ... and x's own BN apply runs inside this conv's operand gather (x written here too); the
                # output's statistics then go to the alternate accumulator (x's are being read)
                y = K.conv2d_fwd_bnstats_inbn(fold[0], x, _arena.weight_bf16(w), g, fold[1])
                if y is None:
                    _bn_fold_apply(x, fold)
                fold = None
            if y is not None:
                ctx.save_for_backward(x, y)
                ctx.w, ctx.b, ctx.g, ctx.act, ctx.in_affine, ctx.prev = w, b, g, act, in_affine, prev
                ctx.plain = False
                ctx.set_materialize_grads(False)
                y._hx_bnstats = 2
                return y
            y = K.conv2d_fwd_bnstats(x, _arena.weight_bf16(w), g)
            if y is not None:
                ctx.save_for_backward(x, y)
                ctx.w, ctx.b, ctx.g, ctx.act, ctx.in_affine, ctx.prev = w, b, g, act, in_affine, prev
                ctx.plain = False
                ctx.set_materialize_grads(False)
                y._hx_bnstats = True
                return y
        if fold is not None:
            _bn_fold_apply(x, fold)
        if pool is not None:
            # conv + act + pk x pk max-pool (+ dropout) as one launch; only the pooled tensor and the
            # argmax exist afterwards (ReLU' is encoded in the argmax, see conv2d_fwd_pool)
            drop_p, salt = pool[:2]
            pk = pool[2] if len(pool) > 2 else 2
            x = x.contiguous()
            rng = rng_state(x.device) if drop_p > 0 else None
            y, am = K.conv2d_fwd_pool(x, _arena.weight_bf16(w), g, bias=b, act=act, drop_p=drop_p, rng=rng, salt=salt,
                                      pk=pk)
            ctx.save_for_backward(x, am)
            ctx.w, ctx.b, ctx.g, ctx.act, ctx.in_affine, ctx.prev = w, b, g, act, in_affine, prev
            ctx.plain = False
            ctx.pool = (drop_p, rng, salt, pk)
            ctx.set_materialize_grads(False)
            y._hx_pool = (am, False, (g[0], g[4], g[5], g[6]), (pk, pk), 0, rng, salt, drop_p, True)
            return y
        if x.dtype == BF16 and _plain_gemm_conv(g, b, act, in_affine, prev):
            x = x.contiguous()
            wb = _arena.weight_bf16(w)
            C, CO = g[3], g[6]
            if _PLAIN_LIB:
                y = torch.mm(x.view(-1, C), wb.view(CO, C).t()).view(g[0], g[4], g[5], CO)
            else:
                y = K.conv2d_fwd(x, wb, g)
            ctx.save_for_backward(x, y)
            ctx.w, ctx.b, ctx.g, ctx.act, ctx.in_affine, ctx.prev = w, b, g, act, in_affine, prev
            ctx.plain = True
            ctx.set_materialize_grads(False)
            return y
        ctx.plain = False
        x = x.contiguous()
        wb = _arena.weight_bf16(w)
        g = K.conv_geom(x.shape, w.shape, stride, padding, dilation)
        y = K.conv2d_fwd(x, wb, g, bias=b, act=act, in_affine=in_affine)
        ctx.save_for_backward(x, y)
        ctx.w, ctx.b, ctx.g, ctx.act, ctx.in_affine, ctx.prev = w, b, g, act, in_affine, prev
        # an input layer whose gradient was fused into the next conv receives no dY: do not
        # let autograd materialise (and this backward then reduce) a zero tensor
        ctx.set_materialize_grads(False)
        return y

    @staticmethod
    def backward(ctx, dy):
        grads = _Conv2dFn._backward(ctx, dy)
        give = getattr(ctx, "give", None)
        if give is not None and grads[0] is not None and not give.pop("late", False):
            give["g"] = grads[0]  # the other consumer of x adds it in its dgrad epilogue (GiveGrad)
            grads = (None,) + tuple(grads[1:])
        return grads

    @staticmethod
    def _backward(ctx, dy):
        if dy is None:
            return (None,) * 12
        if ctx.plain:  # 1x1 conv as library GEMMs: dX = dY W, dW += dY^T X (fp32 out, bf16 in)
            x, _ = ctx.saved_tensors
            w, g = ctx.w, ctx.g
            C, CO = g[3], g[6]
            dy2 = dy.to(BF16).contiguous().view(-1, CO)
            dx = None
            if ctx.needs_input_grad[0]:
                addend = _take_addend(ctx)
                if _PLAIN_LIB:
                    dx = torch.mm(dy2, _arena.weight_bf16(w).view(CO, C)).view(x.shape)
                    if addend is not None:
                        dx.add_(addend)
                else:  # the shortcut's gradient is added in the dgrad epilogue (no separate add launch)
                    add = None if addend is None else addend.to(BF16).contiguous().view(x.shape)
                    dx = _dgrad_bn(ctx, dy2.view(dy.shape), w, g, x, add, addend)
                    if dx is None:
                        dx = K.conv2d_dgrad(dy2.view(dy.shape), _arena.weight_bf16(w), g, addend=add)
            gw = _wgrad_buf(w)
            if os.environ.get("HOPSX_BLASLT_WGRAD", "0") != "1":
                # the library's fp32-out tall-skinny reductions (K = B*H*W) measured slower than the
                # split-K MFMA kernel at ResNet-50 shapes: weight gradient stays on the hopsx kernel
                if K.conv_wgrad_uses_ticket(g):
                    K.conv2d_wgrad(dy2.view(dy.shape), x, g, gw)
                else:
                    with _on_side(dy2.device, dy2, x, flop=2.0 * dy2.numel() * C):
                        K.conv2d_wgrad(dy2.view(dy.shape), x, g, gw)
            else:
                gw.view(CO, C).add_(torch.mm(dy2.t(), x.view(-1, C), out_dtype=torch.float32))
            return (dx, _ret_grad(w, gw), None, None, None, None, None, None, None, None, None, None)
        w, b, g, act = ctx.w, ctx.b, ctx.g, ctx.act
        if ctx.pool is not None:
            x, am = ctx.saved_tensors
            y = None
            drop_p, rng, salt = ctx.pool[:3]
            pk = ctx.pool[3] if len(ctx.pool) > 3 else 2
            oshape = (g[0], g[4], g[5], g[6])
            ent = _PRESCATTERED.pop(dy.data_ptr(), None)
            if ent is not None and ent[0]() is not None and tuple(ent[1].shape) == oshape:
                dy = ent[1]  # the consuming Linear's dgrad epilogue already did the pool backward
            else:
                dy = K.maxpool2d_bwd(dy.to(BF16).contiguous(), am, oshape, (pk, pk), (pk, pk), (0, 0), drop_p=drop_p,
                                     rng=rng, salt=salt)
            premasked = True  # ReLU' rode on the argmax
        else:
            x, y = ctx.saved_tensors
            dy = dy.to(BF16).contiguous() if dy.dtype != BF16 else dy.contiguous()
            premasked = act == 1 and _take_premasked(dy)
        gb = _wgrad_buf(b) if b is not None else None
        ymask = y if (act and not premasked) else None
        if premasked:
            act = 0
        dx = None
        gw = _wgrad_buf(w)
        wflop = 2.0 * dy.numel() * g[7] * g[8] * g[3]
        if (wflop < _PAR_MIN_FLOP and (ctx.prev is not None or ctx.needs_input_grad[0])
                and dy.dtype == BF16 and x.dtype == BF16 and "bwd_pair" not in _disabled()):
            # small layer: dgrad and wgrad as ONE launch (horizontal fusion) instead of two
            pprev = None
            if ctx.prev is not None:
                w0, b0, g0, act0, aff0, x0 = ctx.prev
                pprev = (x0, g0, _arena.grad_target(w0), _arena.grad_target(b0), x, act0, aff0)
            addend = ctx.gslot.get("g") if (ctx.gslot is not None and pprev is None) else None
            co = _colaunch_slice((w, b) + ((ctx.prev[0], ctx.prev[1]) if ctx.prev is not None else ())) \
                if (ctx.prev is not None and addend is None) else None
            bn = _bn_sums_request(ctx, x, pprev, gb, addend)
            r = False
            if bn is not None and K.conv2d_bwd_pair_bn_ok(g):
                # dX is x's whole gradient (sole consumer; a shortcut's part is the addend): its dgrad
                # epilogue masks it and reduces the input BN's backward column sums
                r = K.conv2d_bwd_pair(dy, _arena.weight_bf16(w), g, x, gw, y=ymask, act=act, addend=addend, bn=bn)
                if r is not False and r is not None:
                    _BNPRE[r.data_ptr()] = weakref.ref(r)
            if r is False:
                r = K.conv2d_bwd_pair(dy, _arena.weight_bf16(w), g, x, gw, dbias=gb, y=ymask, act=act, prev=pprev,
                                      addend=addend, opt_slice=co[1] if co is not None else None)
            if co is not None and r is not False:
                COLAUNCH["lo"] = co[0]  # the optimizer's launch now updates only the prefix
                COLAUNCH["launched"] += 1
            if r is not False:
                if addend is not None:
                    ctx.gslot.pop("g", None)  # consumed by the launch
                elif r is not None:
                    r = _add_addend(ctx, r)
                if ctx.prev is not None:
                    hooks.grad_ready(ctx.prev[0])
                    hooks.grad_ready(ctx.prev[1])
                return (r, _ret_grad(w, gw), (_ret_grad(b, gb) if b is not None else None), None, None, None, None,
                        None, None, None, None, None)
        # wgrad || dgrad on a parallel branch (its kernels keep no shared ticket/workspace) — only when there
        # IS a dgrad to overlap: a layer whose input needs no gradient (the image stem) would only pay the
        # cross-queue join (ResNet-50 B=8: +4 % with the stem's weight gradient inline, r5_side_stream_ab.txt)
        side_ok = not K.conv_wgrad_uses_ticket(g, ctx.in_affine) and (ctx.prev is not None or ctx.needs_input_grad[0])
        if side_ok:
            with _on_side(dy.device, dy, x, ymask, flop=2.0 * dy.numel() * g[7] * g[8] * g[3]):
                K.conv2d_wgrad(dy, x, g, gw, dbias=gb, y=ymask, act=act, in_affine=ctx.in_affine)
        if ctx.prev is not None:
            # x is the output of the network's input layer: its weight/bias gradients are
            # produced by this dgrad launch directly, dX is never materialised and the input
            # layer's own backward is never reached (returning None for x)
            w0, b0, g0, act0, aff0, x0 = ctx.prev
            gw0, gb0 = _arena.grad_target(w0), _arena.grad_target(b0)
            K.conv2d_dgrad_fused_wgrad(dy, _arena.weight_bf16(w), g, x, act0, ymask, act, x0, g0, gw0, gb0,
                                       in_affine=aff0)
            hooks.grad_ready(w0)
            hooks.grad_ready(b0)
        elif ctx.needs_input_grad[0]:
            addend = _take_addend(ctx)  # a shortcut's gradient of x: added in the dgrad epilogue
            add = addend.to(BF16).contiguous().view(x.shape) if addend is not None else None
            dx = _dgrad_bn(ctx, dy, w, g, x, add, addend) if ymask is None else None
            if dx is None:
                dx = K.conv2d_dgrad(dy, _arena.weight_bf16(w), g, y=ymask, act=act, addend=add)
        if not side_ok:
            K.conv2d_wgrad(dy, x, g, gw, dbias=gb, y=ymask, act=act, in_affine=ctx.in_affine)
        return (dx, _ret_grad(w, gw), (_ret_grad(b, gb) if b is not None else None), None, None, None, None, None,
                None, None, None, None)


class GiveGrad:
    """``gslot=GiveGrad(slot)`` on a conv: its input gradient is handed to the slot instead of autograd,
    for the OTHER conv consuming the same input (``gslot=slot``, backpropagated later) to add in its
    dgrad epilogue — a projection-shortcut block's two convs of x, no autograd add.  Order-safe: a taker
    that runs first marks the slot "late" and the giver then returns its gradient normally."""
    __slots__ = ("slot",)

    def __init__(self, slot: dict):
        self.slot = slot


# BN backward column sums reduced by a consumer conv's dgrad epilogue (conv_mfma.hip DgradArgs bnacc):
# data_ptr of that dX -> weakref.  _BNFn.backward pops its dy here and then runs only the apply
# (K.bn_bwd_pre).  Written and consumed within one backward pass.
_BNPRE: dict = {}


def bn_sole_consumer(t):
    """Declare that the next hopsx conv applied to ``t`` (a training batch_norm output) is its ONLY autograd
    consumer — other consumers hand their gradient of ``t`` to that conv as an epilogue addend (gslot) —
    so the conv's backward may reduce the BN's backward column sums in its dgrad epilogue.  The ResNet
    blocks call this where the structure guarantees it."""
    if getattr(t, "_hx_bnsrc", None) is not None and "bn_dgrad_sums" not in _disabled():
        t._hx_bn_sole = True
    return t


def _take_bn_input(x):
    if not getattr(x, "_hx_bn_sole", False):
        return None
    x._hx_bn_sole = False  # one consumer
    return x._hx_bnsrc


def _bn_sums_request(ctx, x, pprev, gb, addend):
    """(z, mean, rstd, yprev, act) for a dgrad that can carry its input BN's column sums (K.conv2d_bwd_pair
    / K.conv2d_dgrad_bn bn=...), else None."""
    src = getattr(ctx, "bnin", None)
    if (src is None or pprev is not None or gb is not None or ctx.give is not None or not ctx.needs_input_grad[0]
            or (ctx.gslot is not None and addend is None)):  # a shortcut part not handed over yet: sums incomplete
        return None
    z2, mean, rstd, act, acc = src
    if z2.numel() != x.numel() or x.dtype != BF16:
        return None
    return (z2, mean, rstd, x if act else None, act, acc)


# The same on the separate (unpaired) dgrad launches (ResNet-50).  With the gg engine's per-element
# epilogue it measured slower (B=64 5.1 k vs 5.59 k img/s); with the 16-B LDS-staged BN epilogue
# (gemm_glds.h, EpiDgradBnBF16::store8_bn) it wins at every batch: B=8 1,530 -> 1,608, B=64 5.58-5.68 k ->
# 5.94-5.99 k, B=256 8,081 -> 8,503 img/s (profiles/r5_bn_dgrad_sums.txt).  HOPSX_BN_SUMS_SEPARATE_DGRAD=0: off
_BN_SEPARATE = os.environ.get("HOPSX_BN_SUMS_SEPARATE_DGRAD", "1") == "1"


def _dgrad_bn(ctx, dy, w, g, x, add, addend):
    """dX through K.conv2d_dgrad_bn when x is a sole-consumed BN output and the kernel covers the shape (the
    BN's backward column sums ride on the epilogue; registered for _BNFn.backward), else None."""
    if not _BN_SEPARATE:
        return None
    bn = _bn_sums_request(ctx, x, None, None, addend)
    if bn is None or dy.dtype != BF16:
        return None
    dx = K.conv2d_dgrad_bn(dy.contiguous(), _arena.weight_bf16(w), g, bn, addend=add)
    if dx is False:
        return None
    _BNPRE[dx.data_ptr()] = weakref.ref(dx)
    return dx


def _take_addend(ctx):
    if ctx.gslot is None:
        return None
    a = ctx.gslot.pop("g", None)
    if a is None:
        ctx.gslot["late"] = True  # (a giver that has not run yet returns its gradient to autograd itself)
    return a


def _add_addend(ctx, dx):
    addend = _take_addend(ctx)
    if addend is not None and dx is not None:
        dx.add_(addend.view(dx.shape))
    return dx


def conv2d_maxpool(x, w, b=None, stride=1, padding=0, dilation=1, act=None, pool_kernel=2, pool_stride=None,
                   pool_padding=0, dropout_p: float = 0.0, training: bool = True, salt: int = 0):
    """max_pool2d(conv2d(x, ...), ...) with the pool (+ its fused dropout) folded into the conv's
    epilogue when the pair qualifies (bf16 NHWC on the GPU, unpadded 2x2/2 or 4x4/4 pool, floor
    windows, ReLU or no activation): one launch, and neither the conv output nor a pool pass."""
    pk = (pool_kernel, pool_kernel) if isinstance(pool_kernel, int) else tuple(pool_kernel)
    ps = pk if pool_stride is None else ((pool_stride,) * 2 if isinstance(pool_stride, int) else tuple(pool_stride))
    pp = (pool_padding,) * 2 if isinstance(pool_padding, int) else tuple(pool_padding)
    a = ACT[act] if not isinstance(act, int) else act
    if (x.is_cuda and x.dtype == BF16 and pk in ((2, 2), (4, 4)) and ps == pk and pp == (0, 0)
            and "conv_pool" not in _disabled() and x.data_ptr() % 16 == 0
            and not (padding == "same" and (w.shape[1] % 2 == 0 or w.shape[2] % 2 == 0))):
        st = (stride, stride) if isinstance(stride, int) else tuple(stride)
        dl = (dilation, dilation) if isinstance(dilation, int) else tuple(dilation)
        if padding == "same":
            pd = (_pad_same(w.shape[1], dl[0]), _pad_same(w.shape[2], dl[1]))
        elif padding == "valid":
            pd = (0, 0)
        else:
            pd = (padding, padding) if isinstance(padding, int) else tuple(padding)
        if K.conv_fwd_pool_ok(K.conv_geom(x.shape, w.shape, st, pd, dl), a, pk[0]):
            return _conv_apply(x, w, b, st, pd, dl, a, None,
                               pool=(float(dropout_p) if training else 0.0, salt, pk[0]))
    y = conv2d(x, w, b, stride, padding, dilation, act)
    return max_pool2d(y, pool_kernel, pool_stride, pool_padding, dropout_p, training, salt)  # unfused


class _ConvInPoolFn(torch.autograd.Function):
    """pool(conv(input_layer(x0))) as ONE forward launch (conv_mfma.hip IN0: the input layer is
    evaluated inside the conv's operand gather and its output stored once for the backward).  The
    backward is the conv's own (_Conv2dFn), whose dgrad carries the input layer's weight and bias
    gradients (conv_mfma.hip K0) — the input layer has no backward node of its own."""

    @staticmethod
    def forward(ctx, x0, w0, b0, w, b, act0, aff0, g0, g, act, drop_p, salt, keep):
        rng = rng_state(x0.device) if drop_p > 0 else None
        y, am, y1 = K.conv2d_fwd_pool_in(x0, _arena.weight_bf16(w0), b0, act0, g0, _arena.weight_bf16(w), g, bias=b,
                                         act=act, drop_p=drop_p, rng=rng, salt=salt, in_affine=aff0, keep_y1=keep)
        ctx.save_for_backward(y1, am)
        ctx.w, ctx.b, ctx.g, ctx.act, ctx.in_affine = w, b, g, act, None
        ctx.prev = (w0, b0, g0, act0, aff0, x0)
        ctx.plain, ctx.gslot, ctx.pool = False, None, (drop_p, rng, salt)
        ctx.set_materialize_grads(False)
        y._hx_pool = (am, False, (g[0], g[4], g[5], g[6]), (2, 2), 0, rng, salt, drop_p, True)
        return y

    @staticmethod
    def backward(ctx, dy):
        r = _Conv2dFn.backward(ctx, dy)
        return (None, None, None, r[1], r[2]) + (None,) * 8


def _sym_pads(padding, ks, dl):
    """Symmetric (ph, pw) for a padding spec, or None ('same' with an even kernel pads one side)."""
    if padding == "valid":
        return (0, 0)
    if padding == "same":
        if ks[0] % 2 == 0 or ks[1] % 2 == 0:
            return None
        return (_pad_same(ks[0], dl[0]), _pad_same(ks[1], dl[1]))
    return (padding, padding) if isinstance(padding, int) else tuple(padding)


# opt-in (HOPSX_CONV_IN_POOL=1): one launch fewer and bit-identical, but measured 1-2 % slower on the
# flagship at the driver's 20-step setting (profiles/r3s7_flagship_ab.txt): the in-gather input layer
# lengthens conv2's operand phase by more than the separate launch costs
def _conv_in_pool_on() -> bool:
    return os.environ.get("HOPSX_CONV_IN_POOL", "0") == "1"


def conv_input_maxpool(x, w0, b0, act0, in_affine0, cfg0, w, b, act, cfg, pool_kernel=2, pool_stride=None,
                       pool_padding=0, dropout_p=0.0, training=True, salt=0):
    """max_pool2d(conv2d(conv2d(x, w0, b0, in_affine0), w, b)) for the network's input layer (raw uint8
    NHWC images, one channel) as ONE launch when the chain qualifies; returns None otherwise (the
    caller then runs the layers one by one).  Results equal the unfused chain's (same fp32 order in
    the input layer, same bf16 roundings)."""
    if (not x.is_cuda or x.dtype != torch.uint8 or x.dim() != 4 or x.shape[-1] != 1 or in_affine0 is None
            or float(in_affine0[0]) == 0.0 or not _conv_in_pool_on() or "conv_in_pool" in _disabled()
            or b0 is None):
        return None
    pk = (pool_kernel, pool_kernel) if isinstance(pool_kernel, int) else tuple(pool_kernel)
    ps = pk if pool_stride is None else ((pool_stride,) * 2 if isinstance(pool_stride, int) else tuple(pool_stride))
    pp = (pool_padding,) * 2 if isinstance(pool_padding, int) else tuple(pool_padding)
    if pk != (2, 2) or ps != (2, 2) or pp != (0, 0):
        return None
    geoms = []
    shape = tuple(x.shape)
    for wt, c in ((w0, cfg0), (w, cfg)):
        st = (c.get("stride", 1),) * 2 if isinstance(c.get("stride", 1), int) else tuple(c["stride"])
        dl = (c.get("dilation", 1),) * 2 if isinstance(c.get("dilation", 1), int) else tuple(c["dilation"])
        pd = _sym_pads(c.get("padding", 0), tuple(wt.shape[1:3]), dl)
        if pd is None or st != (1, 1) or dl != (1, 1):
            return None
        gg = K.conv_geom(shape, wt.shape, st, pd, dl)
        geoms.append(gg)
        shape = (gg[0], gg[4], gg[5], gg[6])
    g0, g = geoms
    a0 = ACT[act0] if not isinstance(act0, int) else act0
    a = ACT[act] if not isinstance(act, int) else act
    if not K.conv_u8_fusable(g0) or not K.conv_fwd_pool_in_ok(g0, g, a) or x.data_ptr() % 16:
        return None
    keep = torch.is_grad_enabled() and (w.requires_grad or w0.requires_grad)
    if keep and (not w0.requires_grad or _arena.grad_target(w0) is None or _arena.grad_target(b0) is None
                 or not K.conv_dgrad_fused_wgrad_ok(g, g0) or "fused_wgrad0" in _disabled()):
        return None  # the input layer's gradients must ride on this conv's dgrad
    aff = (float(in_affine0[0]), float(in_affine0[1]))
    return _ConvInPoolFn.apply(x.contiguous(), w0, b0, w, b, a0, aff, g0, g, a,
                               float(dropout_p) if training else 0.0, salt, keep)


def _fusable_input_layer(x, geom):
    """(w0, b0, geom0, act0, in_affine0, x0) when x is the output of the network's input layer
    and that layer's weight gradient can ride on this conv's dgrad (see conv_mfma.hip K0)."""
    prev = getattr(x, "_hx_input_layer", None)
    if prev is None or not torch.is_grad_enabled() or "fused_wgrad0" in _disabled():
        return None
    w0, b0, g0 = prev[0], prev[1], prev[2]
    if b0 is None or not w0.requires_grad or _arena.grad_target(w0) is None or _arena.grad_target(b0) is None:
        return None
    return prev if K.conv_dgrad_fused_wgrad_ok(geom, g0) else None


def _disabled() -> str:
    import os

    return os.environ.get("HOPSX_DISABLE", "")


def _conv_apply(x, w, b, st, pd, dl, a, in_affine, pool=None, bnstats=False, gslot=None):
    """Apply the conv Function; tag the output of an input layer (input needs no gradient) so
    the next conv can fuse this layer's weight gradient into its dgrad."""
    prev = _fusable_input_layer(x, K.conv_geom(x.shape, w.shape, st, pd, dl)) if x.requires_grad else None
    y = _Conv2dFn.apply(x, w, b, st, pd, dl, a, in_affine, prev, pool, bnstats, gslot)
    if pool is not None:
        return y
    if a:
        y._hx_act_out = a  # activation fused into this conv's epilogue (see max_pool2d premask)
    if not x.requires_grad and w.requires_grad and x.shape[-1] == 1:
        y._hx_input_layer = (w, b, K.conv_geom(x.shape, w.shape, st, pd, dl), a, in_affine, x)
    return y


class _PadCinFn(torch.autograd.Function):
    """A conv weight [CO, KH, KW, C] zero-padded to ``cp`` input channels, for an input whose channels
    C..cp-1 are zero (a 3-channel image stem laid out as 8 channels by kernels.u8_normalize_chan, so the
    conv takes the C % 8 == 0 MFMA paths instead of the generic narrow-channel gather).  The padded
    taps meet zeros, so the conv is unchanged; backward hands the first C channels of the padded
    weight's gradient to the parameter (into its arena gradient directly when it has one)."""

    @staticmethod
    def forward(ctx, w, cp):
        ctx.w = w
        if not w.is_cuda or "pad_cin" in _disabled():
            return torch.nn.functional.pad(w.detach(), (0, cp - w.shape[-1]))
        # GPU: one kernel writes the padded fp32 weight AND the bf16 copy the conv reads (tagged as its
        # shadow); its weight gradient goes into a zero-at-rest buffer kept on the parameter, which the
        # backward folds into the arena gradient and re-zeroes in one launch (no fill / copy / cast /
        # add launches of PyTorch's own in the step)
        out, out16 = K.pad_cin(w.detach(), cp)
        out._hx_shadow = out16
        wb = getattr(w, "_hx_padgrad", None)
        if wb is None or wb.shape != out.shape:
            wb = torch.zeros(out.shape, device=w.device, dtype=torch.float32)  # warm-up (eager), not in capture
            w._hx_padgrad = wb
        out._hx_wbuf = wb
        return out

    @staticmethod
    def backward(ctx, g):
        w = ctx.w
        tgt = _arena.grad_target(w)
        if g.is_cuda and g is getattr(w, "_hx_padgrad", None):
            # g is the zero-at-rest buffer: add its first C channels to the arena gradient (or a fresh
            # one) and re-zero it, one launch; accumulate BEFORE announcing (the DP overlap hook may
            # launch this bucket's reduction the moment the stem weight, the last gradient, is ready)
            out = tgt if tgt is not None else torch.zeros(w.shape, device=w.device, dtype=torch.float32)
            K.unpad_cin_add(g, w.shape[-1], out)
            hooks.grad_ready(w)
            return (None if tgt is not None else out), None
        gs = g[..., :w.shape[-1]]
        if tgt is not None:
            tgt.add_(gs)
            hooks.grad_ready(w)
            return None, None
        hooks.grad_ready(w)
        return gs.contiguous(), None


def pad_input_channels(w, cp: int):
    """``w`` padded with zero input channels to ``cp`` (autograd-aware, see _PadCinFn)."""
    return _PadCinFn.apply(w, int(cp))


def conv2d(x, w, b=None, stride=1, padding=0, dilation=1, act=None, in_affine=None, bnstats=False, gslot=None):
    """NHWC conv. x [B,H,W,C], w [CO,KH,KW,C]. padding: int, tuple, 'valid' or 'same' (stride 1).

    ``bnstats=True``: the output feeds a training-mode ``batch_norm`` next (models/resnet.py ConvBN);
    where the conv kernel has the epilogue, it accumulates the BN statistics itself and tags the
    output (``_hx_bnstats``) so the BN skips its statistics pass.  The tagged output must go to
    ``batch_norm`` before any other BN of the same width runs.  ``gslot``: see _Conv2dFn (GPU only).

    ``in_affine=(scale, shift)`` with a uint8 ``x``: the input layer's normalisation
    ``x * scale + shift``; on the GPU it is fused into the conv kernels when the layer
    qualifies (K.conv_u8_fusable), otherwise applied by one normalisation pass first."""
    st = (stride, stride) if isinstance(stride, int) else tuple(stride)
    dl = (dilation, dilation) if isinstance(dilation, int) else tuple(dilation)
    if padding == "valid":
        pd = (0, 0)
    elif padding == "same":
        pd = (_pad_same(w.shape[1], dl[0]), _pad_same(w.shape[2], dl[1]))
    else:
        pd = (padding, padding) if isinstance(padding, int) else tuple(padding)
    a = ACT[act] if not isinstance(act, int) else act
    if x.dtype == torch.uint8:
        sc, sh = in_affine or (1.0, 0.0)
        if not x.is_cuda:
            x = x.float() * sc + sh
        elif padding != "same" or (w.shape[1] % 2 == 1 and w.shape[2] % 2 == 1):
            g = K.conv_geom(x.shape, w.shape, st, pd, dl)
            if K.conv_u8_fusable(g):
                return _conv_apply(x, w, b, st, pd, dl, a, (float(sc), float(sh)))
            x = K.u8_normalize(x.contiguous(), float(sc), float(sh))
        else:
            x = K.u8_normalize(x.contiguous(), float(sc), float(sh))
    if not x.is_cuda:
        xr = x.float().permute(0, 3, 1, 2)
        if padding == "same" and (w.shape[1] % 2 == 0 or w.shape[2] % 2 == 0):
            # TF 'same' pads the extra row/col at the end for even kernels
            th, tw = dl[0] * (w.shape[1] - 1), dl[1] * (w.shape[2] - 1)
            xr = F.pad(xr, (tw // 2, tw - tw // 2, th // 2, th - th // 2))
            pd = (0, 0)
        y = F.conv2d(xr, w.permute(0, 3, 1, 2), b, st, pd, dl)
        return _cpu_act(y, a).permute(0, 2, 3, 1).contiguous()
    if padding == "same" and (w.shape[1] % 2 == 0 or w.shape[2] % 2 == 0):
        # TF 'same' with an even kernel: the extra row / column of padding goes at the end — an asymmetric
        # geometry (K.conv_geom), not a padded copy of x
        th, tw = dl[0] * (w.shape[1] - 1), dl[1] * (w.shape[2] - 1)
        pd = (th // 2, tw // 2, th - th // 2, tw - tw // 2)
    return _conv_apply(to_compute(x), w, b, st, pd, dl, a, None, bnstats=bnstats and x.is_cuda,
                       gslot=gslot if x.is_cuda else None)


def _bnstats_conv(g) -> bool:
    """Conv shapes whose BN statistics ride on the conv epilogue: everything except 1x1 convs above
    HOPSX_BNSTATS_MAX_1X1_FLOP, which run as plain GEMMs (_plain_gemm_conv: the hopsx gg engine, or
    hipBLASLt only under HOPSX_PLAIN_GEMM=blaslt) followed by a separate statistics pass."""
    if "bnstats" in _disabled() or not K.bn_prestats_ok(g[6]):
        return False
    B, H, W, C, OH, OW, CO, KH, KW = g[:9]
    if KH == 1 and KW == 1 and 2.0 * B * OH * OW * CO * C > _BNSTATS_MAX_1X1_FLOP:
        return False
    return C % 8 == 0


# 1x1 routing: above HOPSX_BNSTATS_MAX_1X1_FLOP a 1x1 conv leaves the stats-epilogue conv kernel for the
# plain-GEMM path + a BN statistics pass.  Round 2 set 1e8 when that path was hipBLASLt
# (profiles/r2s7_plain_1x1_ab.txt); with both paths on the gg engine the stats epilogue wins at every
# size (ResNet-50 B=8 / 64 / 256: +4.7 / +3-4 / +3.5 %, CIFAR flat; profiles/r4_launch_knobs_ab.txt),
# so the default is no limit
_BNSTATS_MAX_1X1_FLOP = float(os.environ.get("HOPSX_BNSTATS_MAX_1X1_FLOP", 1e30))
# fewest output pixels for which a plain 1x1 conv takes the plain-GEMM path
_PLAIN_MIN_PX = int(os.environ.get("HOPSX_PLAIN_MIN_PX", 256))


# ==================================================================== pooling
# data_ptrs of gradients that already carry the ReLU' mask of the tensor they are the gradient
# of (applied by the max-pool backward at its argmax scatter): the producing conv's backward
# then skips its own mask and never loads its activation output (half the dY traffic of its
# dgrad/wgrad).  Written and consumed within one backward pass (also during graph capture).
_PRESCATTERED: dict = {}  # placeholder data_ptr -> (weakref, pool-input gradient, premasked)
_PREMASKED: dict = {}  # data_ptr -> weakref of the pool's dX (a dead ref means the memory may be reused)


class _MaxPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s, p, drop_p, salt, premask):
        x = x.contiguous()
        rng = rng_state(x.device) if drop_p > 0 else None
        y, am = K.maxpool2d_fwd(x, k, s, p, drop_p=drop_p, rng=rng, salt=salt)
        if premask:
            ctx.save_for_backward(am, x)
        else:
            ctx.save_for_backward(am)
        ctx.cfg = (x.shape, k, s, p, drop_p, rng, salt, premask)
        B, H, W, C = x.shape
        if x.is_cuda and s == k and p == (0, 0) and H >= k[0] and W >= k[1] and k[0] * k[1] <= 255:
            # a Linear consuming the (flattened) output can do this backward in its dgrad epilogue
            # (floor windows: the remainder rows / columns get zeros there)
            y._hx_pool = (am, bool(premask), tuple(x.shape), k, "relu" if premask else 0,
                          rng, salt, drop_p, bool(premask))
        return y

    @staticmethod
    def backward(ctx, dy):
        shape, k, s, p, drop_p, rng, salt, premask = ctx.cfg
        ent = _PRESCATTERED.pop(dy.data_ptr(), None)
        if ent is not None and ent[0]() is not None and tuple(ent[1].shape) == tuple(shape):
            dx = ent[1]  # already produced by the consuming Linear's dgrad epilogue
            if ent[2]:
                _PREMASKED[dx.data_ptr()] = weakref.ref(dx)
            return dx, None, None, None, None, None, None
        dy = dy.to(BF16).contiguous()
        if premask:
            am, x = ctx.saved_tensors
            dx = K.maxpool2d_bwd(dy, am, shape, k, s, p, x=x, act="relu", drop_p=drop_p, rng=rng, salt=salt)
            _PREMASKED[dx.data_ptr()] = weakref.ref(dx)
        else:
            (am,) = ctx.saved_tensors
            dx = K.maxpool2d_bwd(dy, am, shape, k, s, p, drop_p=drop_p, rng=rng, salt=salt)
        return dx, None, None, None, None, None, None


def _take_premasked(dy) -> bool:
    ref = _PREMASKED.pop(dy.data_ptr(), None)
    src = ref() if ref is not None else None
    return src is not None and src.shape == dy.shape


def max_pool2d(x, kernel, stride=None, padding=0, dropout_p: float = 0.0, training: bool = True, salt: int = 0):
    """NHWC max-pool; ``dropout_p`` > 0 fuses a following Dropout into the same kernel (fwd and bwd)."""
    k = (kernel, kernel) if isinstance(kernel, int) else tuple(kernel)
    s = k if stride is None else ((stride, stride) if isinstance(stride, int) else tuple(stride))
    p = (padding, padding) if isinstance(padding, int) else tuple(padding)
    dp = float(dropout_p) if training else 0.0
    if not x.is_cuda:
        y = F.max_pool2d(x.permute(0, 3, 1, 2), k, s, p).permute(0, 2, 3, 1).contiguous()
        return F.dropout(y, dp, True) if dp > 0 else y
    # a ReLU conv output feeding the pool: apply ReLU' at the argmax scatter (idempotent, so it
    # stays correct if the conv output has other consumers whose gradients get added)
    premask = (getattr(x, "_hx_act_out", None) == 1 and x.requires_grad and x.dtype == BF16
               and "premask" not in _disabled())
    return _MaxPoolFn.apply(to_compute(x), k, s, p, dp, salt, premask)


class _GapFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        ctx.shape = x.shape
        return K.gap_fwd(x.contiguous())

    @staticmethod
    def backward(ctx, dy):
        return K.gap_bwd(dy.to(BF16).contiguous(), ctx.shape)


def global_avg_pool(x):
    if not x.is_cuda:
        return x.mean(dim=(1, 2))
    return _GapFn.apply(to_compute(x))


# ==================================================================== dropout
_RNG: dict = {}


def rng_state(device) -> torch.Tensor:
    """Per-device (seed, counter) int64 pair; advanced once per train step."""
    key = str(device)
    if key not in _RNG:
        seed = int(torch.randint(0, 2**62, (1,)).item())
        _RNG[key] = torch.tensor([seed, 0], dtype=torch.int64, device=device)
    return _RNG[key]


def seed_device_rng(seed: int, device) -> None:
    """Pin the device RNG.  Does not draw from torch's global generator (rng_state's lazy default
    does), so seeding before ``torch.manual_seed``-dependent init leaves that init unchanged."""
    key = str(device)
    if key in _RNG:
        _RNG[key].copy_(torch.tensor([seed, 0], dtype=torch.int64))
    else:
        _RNG[key] = torch.tensor([seed, 0], dtype=torch.int64, device=device)


def advance_rng(device) -> None:
    if torch.device(device).type == "cuda":
        K.rng_advance(rng_state(device))
    else:
        rng_state(device)[1] += 1


class _DropoutFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, p, salt):
        rng = rng_state(x.device)
        ctx.cfg = (p, salt, rng)
        return K.dropout(x.contiguous(), p, rng, salt)

    @staticmethod
    def backward(ctx, dy):
        p, salt, rng = ctx.cfg
        return K.dropout(dy.to(BF16).contiguous(), p, rng, salt), None, None


def dropout(x, p: float, training: bool = True, salt: int = 0):
    if not training or p <= 0:
        return x
    if not x.is_cuda:
        return F.dropout(x, p, True)
    return _DropoutFn.apply(to_compute(x), float(p), salt)


# ================================================================== batchnorm
class _BNFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, gamma, beta, rm, rv, momentum, eps, residual, act, prestats=False, gslot=None, fold=False):
        C = x.shape[-1]
        x2 = x.contiguous().view(-1, C)
        mean = torch.empty(C, device=x.device)
        rstd = torch.empty(C, device=x.device)
        r2 = residual.contiguous().view(-1, C) if residual is not None else None
        deferred = None
        if fold and prestats is True and residual is None and x2.dtype == BF16 and "bn_fold" not in _disabled():
            # the apply is folded into the consuming conv's operand gather (conv2d_fwd_bnstats_inbn), which
            # also writes y, mean / rstd and the running statistics; _Conv2dFn launches the apply instead
            # when its shape has no such path (_bn_fold_apply)
            y = torch.empty_like(x2)
            deferred = (x2, (gamma, beta, mean, rstd, rm, rv, momentum, eps, act))
        elif prestats:  # statistics accumulated by the producing conv's epilogue (2: the alternate buffer)
            y = K.bn_fwd_apply_fin(x2, gamma, beta, mean, rstd, rm, rv, momentum, eps, residual=r2, act=act,
                                   alt=prestats == 2)
        else:
            y = K.bn_fwd_train(x2, gamma, beta, mean, rstd, rm, rv, momentum, eps, residual=r2, act=act)
        ctx.save_for_backward(x2, y, mean, rstd)
        ctx.p = (gamma, beta, act, x.shape, residual is not None)
        ctx.gslot = gslot  # the residual's gradient goes to the conv that also consumes it (_Conv2dFn)
        out = y.view(x.shape)
        if x.is_cuda and out.dtype == BF16 and "bn_dgrad_sums" not in _disabled():
            # for a consumer conv's dgrad epilogue (bn_sole_consumer): the BN input, its batch statistics and
            # this BN's private sums accumulator
            out._hx_bnsrc = (x2, mean, rstd, act, K.bn_sums_acc(gamma, x.device, C))
        if deferred is not None:
            out._hx_bn_fold = deferred
        return out

    @staticmethod
    def backward(ctx, dy):
        x2, y, mean, rstd = ctx.saved_tensors
        gamma, beta, act, shape, has_res = ctx.p
        C = shape[-1]
        gg, gb = _wgrad_buf(gamma), _wgrad_buf(beta)
        ws = torch.empty(2 * C, device=dy.device)
        ent = _BNPRE.pop(dy.data_ptr(), None)
        src = ent() if ent is not None else None
        if src is not None and src.numel() == dy.numel() and dy.dtype == BF16 and dy.is_contiguous():
            # the consuming conv's dgrad already masked dy and reduced the column sums: apply only; the
            # masked dy IS the residual's gradient
            dy2 = dy.view(-1, C)
            dx = K.bn_bwd_pre(dy2, x2, gamma, mean, rstd, gg, gb, ws, K.bn_sums_acc(gamma, dy.device, C))
            dres = dy2 if has_res else None
            if has_res and ctx.gslot is not None:
                ctx.gslot["g"] = dres.view(shape)
                dres = None
            return (dx.view(shape), _ret_grad(gamma, gg), _ret_grad(beta, gb), None, None, None, None,
                    dres.view(shape) if dres is not None else None, None, None, None, None)
        dy2 = dy.to(BF16).contiguous().view(-1, C)
        dres = torch.empty_like(dy2) if has_res else None
        # no residual + ReLU: the backward recomputes the act' mask from x (no read of y; K.bn_bwd zbeta)
        zb = beta.detach() if (beta is not None and not has_res and K.act_id(act) == 1) else None
        dx = K.bn_bwd(dy2, x2, y, gamma, mean, rstd, gg, gb, ws, act=act, dresidual=dres, zbeta=zb)
        if has_res and ctx.gslot is not None:
            ctx.gslot["g"] = dres.view(shape)
            dres = None
        return (dx.view(shape), _ret_grad(gamma, gg), _ret_grad(beta, gb), None, None, None, None,
                dres.view(shape) if dres is not None else None, None, None, None, None)


def _bn_fold_apply(a, fold) -> None:
    """Launch the deferred apply of a fold_next batch_norm output ``a`` whose consumer could not fold it."""
    z2, (gamma, beta, mean, rstd, rm, rv, momentum, eps, act) = fold
    K.bn_fwd_apply_fin(z2, gamma, beta, mean, rstd, rm, rv, momentum, eps, act=act, out=a.view(z2.shape))


def _take_bn_fold(x):
    fold = getattr(x, "_hx_bn_fold", None)
    if fold is not None:
        x._hx_bn_fold = None
    return fold


def batch_norm(x, gamma, beta, running_mean, running_var, training=True, momentum=0.1, eps=1e-5, residual=None,
               act=None, gslot=None, fold_next=False):
    """NHWC batch norm with fused residual add + activation: act(bn(x) + residual).  ``gslot``: hand
    the residual's gradient to the conv that also consumes the residual (see _Conv2dFn) instead of
    returning it to autograd.  ``fold_next``: the output goes straight to a ``conv2d(bnstats=True)`` (its
    only consumer, next on the stream): with statistics from the producing conv and no residual, the
    apply is deferred into that conv's operand gather (conv_mfma.hip InBn) — one launch fewer."""
    a = ACT[act] if not isinstance(act, int) else act
    C = x.shape[-1]
    if not x.is_cuda:
        y = F.batch_norm(x.reshape(-1, C).float(), running_mean, running_var, gamma, beta, training, momentum, eps)
        y = y.view(x.shape)
        if residual is not None:
            y = y + residual
        return _cpu_act(y, a)
    pre = getattr(x, "_hx_bnstats", False)
    if pre:
        x._hx_bnstats = False  # the accumulated statistics are consumed (and re-zeroed) exactly once
        if not training:
            # the conv epilogue already accumulated this tensor's statistics: re-zero the shared
            # accumulator rows before raising, or every later training BN of this width folds them in
            K.bn_acc(x.device, C, alt=pre == 2).zero_()
            raise RuntimeError("conv2d(bnstats=True) output fed to an eval-mode batch_norm")
    x = to_compute(x)
    residual = to_compute(residual) if residual is not None else None
    if training:
        return _BNFn.apply(x, gamma, beta, running_mean, running_var, momentum, eps, residual, a, pre, gslot,
                           bool(fold_next))
    y = K.bn_fwd_infer(x.contiguous().view(-1, C), gamma, beta, running_mean, running_var, eps,
                       residual=None if residual is None else residual.contiguous().view(-1, C), act=a)
    return y.view(x.shape)


# ============================================================== embedding bag
class _EmbagFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, idx, offsets, table, mode, nbags, bag_len):
        out = torch.empty(nbags, table.shape[1], device=table.device, dtype=torch.float32)
        K.embedding_bag_fwd(table.detach(), idx, offsets, mode, out, bag_len=bag_len)
        ctx.save_for_backward(idx, offsets if offsets is not None else torch.empty(0, device=idx.device))
        ctx.p = (table, mode, nbags, offsets is not None, bag_len)
        return out

    @staticmethod
    def backward(ctx, dout):
        idx, offs = ctx.saved_tensors
        table, mode, nbags, has_offs, bag_len = ctx.p
        g = _wgrad_buf(table)
        K.embedding_bag_bwd(dout.float().contiguous(), idx, offs if has_offs else None, mode, g, nbags,
                            bag_len=bag_len)
        return None, None, _ret_grad(table, g), None, None, None


def embedding_bag(idx, table, offsets=None, mode="sum"):
    """Sum/mean of embedding rows per bag -> fp32 [bags, dim].

    idx: 1-D int64 with ``offsets`` (variable-length bags), [B] (one row per bag), or
    [B, L] (fixed-length bags of L rows, e.g. the L categorical columns of a wide model)."""
    m = {"sum": 0, "mean": 1}[mode]
    if not table.is_cuda:
        if offsets is None:
            e = F.embedding(idx, table)
            return e if idx.dim() == 1 else (e.sum(1) if m == 0 else e.mean(1))
        return F.embedding_bag(idx, table, offsets, mode=mode)
    bag_len = idx.shape[1] if (offsets is None and idx.dim() == 2) else 1
    idx = idx.long().contiguous()
    nb = (idx.numel() // bag_len) if offsets is None else offsets.numel()
    return _EmbagFn.apply(idx.reshape(-1), None if offsets is None else offsets.long().contiguous(), table, m, nb,
                          bag_len)


# ===================================================================== losses
class _LossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, target, kind, stats):
        B, C = logits.shape
        loss_sum = torch.empty(1, device=logits.device)  # the kernel overwrites / zero-fills itself
        correct = torch.empty(1, device=logits.device, dtype=torch.int32)
        dl = torch.empty(B, C, device=logits.device, dtype=torch.float32)
        K.loss_fwd_bwd(kind, logits.contiguous(), target.contiguous(), 1.0 / (B * (C if kind in (2, 3, 4) else 1)),
                       loss_sum, correct, dl)
        if stats is not None:
            stats["correct"] = correct
            stats["count"] = B * (C if kind in (2, 4) else 1)
        ctx.save_for_backward(dl)
        ctx.dtype = logits.dtype
        return loss_sum.squeeze(0)

    @staticmethod
    def backward(ctx, g):
        (dl,) = ctx.saved_tensors
        return (dl * g).to(ctx.dtype), None, None, None


def _cpu_loss(kind, logits, target, stats):
    logits = logits.float()
    if kind == 0:
        loss = F.cross_entropy(logits, target.long())
        corr = (logits.argmax(1) == target.long()).sum()
        cnt = logits.shape[0]
    elif kind == 1:
        loss = -(target * F.log_softmax(logits, 1)).sum(1).mean()
        corr = (logits.argmax(1) == target.argmax(1)).sum()
        cnt = logits.shape[0]
    elif kind == 2:
        loss = F.binary_cross_entropy_with_logits(logits, target.float())
        corr = ((logits > 0) == (target > 0.5)).sum()
        cnt = target.numel()
    elif kind == 3:
        loss = F.mse_loss(logits, target.float())
        corr, cnt = torch.zeros(()), 1
    else:
        p = logits.clamp(1e-7, 1 - 1e-7)
        loss = F.binary_cross_entropy(p, target.float())
        corr = ((logits > 0.5) == (target > 0.5)).sum()
        cnt = target.numel()
    if stats is not None:
        stats["correct"] = corr
        stats["count"] = cnt
    return loss


def loss_and_grad(logits, target, kind: str = "sparse_ce"):
    """Non-autograd fused loss for training loops that seed backward themselves:
    returns (mean loss [1], correct [1] int32, count, dlogits in the logits' dtype).
    ``logits.backward(dlogits)`` then runs the model backward with no extra
    elementwise kernels (the 1/count mean scaling is folded into the loss kernel)."""
    k = LOSS[kind]
    if logits.dim() == 1:
        logits = logits.unsqueeze(1)
    B, C = logits.shape
    cnt = B * (C if k in (2, 3, 4) else 1)
    if k in (2, 3, 4) and target.dim() == 1:
        target = target.unsqueeze(1)
    if not logits.is_cuda:
        lg = logits.detach().float().requires_grad_(True)
        st: dict = {}
        l = _cpu_loss(k, lg, target, st)
        (g,) = torch.autograd.grad(l, (lg,))
        return l.detach().view(1), torch.as_tensor(st["correct"]).view(1), st["count"], g.to(logits.dtype)
    target = target.long() if k == 0 else target.float()
    loss_sum = torch.empty(1, device=logits.device)
    correct = torch.empty(1, device=logits.device, dtype=torch.int32)
    dl = torch.empty(B, C, device=logits.device, dtype=logits.dtype)
    K.loss_fwd_bwd(k, logits.detach().contiguous(), target.contiguous(), 1.0 / cnt, loss_sum, correct, dl)
    return loss_sum, correct, (B if k in (0, 1) else cnt), dl


def loss_and_grad_root(logits, target, kind: str = "sparse_ce"):
    """Like :func:`loss_and_grad` but returns ``(loss, correct, count, root, grad)`` for
    ``root.backward(grad)``.  When ``logits`` come from a linear logits layer (tagged by
    :func:`linear`), ONE kernel computes the loss, that layer's weight and bias gradients and the
    gradient w.r.t. its input ``h`` (loss.hip head_ce_k), and backward starts at ``h``: the loss
    kernel and the head's two backward GEMMs collapse into one launch."""
    head = getattr(logits, "_hx_dense_head", None)
    k = LOSS[kind]
    drop = head[5] if head is not None and len(head) > 5 else None
    pend = PREHEAD["pending"].pop(head[0].data_ptr(), None) if (head is not None and head[4]) else None
    flush_pending()  # deferred outputs other than the head's input
    if (head is None or not logits.is_cuda or logits.dim() != 2 or "head_ce" in _disabled()
            or not K.head_ce_ok(logits.shape[1], head[0].shape[1])):
        if pend is not None:
            K.linear_fwd(pend[0], pend[1], pend[2], act=pend[3], out=pend[4])
        if head is not None and head[4]:  # deferred logits the fused kernel cannot take: compute them now
            hin = dropout(head[0], drop[0], True, drop[2]) if drop is not None else head[0]
            real = _LinearFn.apply(hin, head[1], head[2], 0, head[3], None)
            logits.copy_(real.detach())
            logits = real
        loss_, correct, count, dl = loss_and_grad(logits, target, kind)
        return loss_, correct, count, logits, dl
    h, w, b, _, deferred = head[:5]
    B, C = logits.shape
    cnt = B * (C if k in (2, 3, 4) else 1)
    if k in (2, 3, 4) and target.dim() == 1:
        target = target.unsqueeze(1)
    target = (target.long() if k == 0 else target.float()).contiguous()
    loss_sum = torch.empty(1, device=logits.device)
    correct = torch.empty(1, device=logits.device, dtype=torch.int32)
    if pend is not None:
        # the pre-head Dense layer + this head + the loss: one launch (loss.hip mlp_head_k)
        x2, wb, b1, act1, y = pend
        dh = K.mlp_head(x2, wb, b1.detach() if b1 is not None else None, act1, y, k, logits, target,
                        _arena.weight_bf16(w), b.detach() if b is not None else None, _arena.grad_target(w),
                        _arena.grad_target(b) if b is not None else None, 1.0 / cnt, loss_sum, correct, drop=drop)
        if dh is not False:
            hooks.grad_ready(w)
            if b is not None:
                hooks.grad_ready(b)
            return loss_sum, correct, (B if k in (0, 1) else cnt), h, dh
        K.linear_fwd(x2, wb, b1, act=act1, out=y)  # shape the fused kernel does not take
    dh = K.head_ce(k, logits if deferred else logits.detach().contiguous(), target, h.detach(),
                   _arena.weight_bf16(w), _arena.grad_target(w), _arena.grad_target(b) if b is not None else None,
                   1.0 / cnt, loss_sum, correct, bias=b.detach() if (deferred and b is not None) else None,
                   forward=deferred, drop=drop)
    hooks.grad_ready(w)
    if b is not None:
        hooks.grad_ready(b)
    return loss_sum, correct, (B if k in (0, 1) else cnt), h, dh


def loss(logits, target, kind: str = "sparse_ce", stats: dict | None = None):
    """Fused loss (+ gradient + correct-count in the same kernel).

    kind: sparse_ce (int labels), ce (one-hot/soft targets), bce_logits, bce (probabilities), mse.
    ``stats`` (optional dict) receives a device tensor ``correct`` and ``count``.
    """
    k = LOSS[kind]
    if logits.dim() == 1:
        logits = logits.unsqueeze(1)
    if k in (2, 3, 4) and target.dim() == 1:
        target = target.unsqueeze(1)
    if not logits.is_cuda:
        return _cpu_loss(k, logits, target, stats)
    if k == 0:
        target = target.long()
    else:
        target = target.float()
    return _LossFn.apply(logits, target, k, stats)
