"""Per-layer numerics of a training step on the hopsx kernels against fp64 (ResNets: conv / BN / GAP /
linear), with the kernels' own bf16 tensors as the reference's inputs.

Why teacher-forced.  A whole bf16 ResNet step compared with a free-running fp64 step drifts apart by
the network's own sensitivity: a last-bit difference in one BN mean grows ~2x per layer of a
random-init ResNet-20 (tests/test_bnstats_gpu.py), so a whole-step cosine (0.96) cannot tell one wrong
layer from accumulated rounding.  Here every recorded op is recomputed in fp64 FROM THE TENSORS THE
KERNELS ACTUALLY READ (their bf16 activations, the bf16 weight shadows) and the reference graph carries
the kernel's output value forward (value = kernel output, derivative = the exact fp64 op derivative at
that point: ``y_ref + (y_kernel - y_ref).detach()``).  So

  * each op's FORWARD is checked in isolation (its output vs fp64 of the same op on the same inputs);
  * the fp64 backward through that graph — optionally rounding every activation gradient to bf16 where
    the kernels store it (``round_grads``) — gives every parameter's gradient at the kernels' own
    operating point, and the kernels' gradients are compared per parameter tensor.

A layer whose kernel computes a wrong gradient shows up as that tensor's cosine, not as noise spread
over the network.  Reference: notebooks/ml/Benchmarks/benchmark.ipynb:144 (the BN ResNets of E7) and
BASELINE config 5.
"""
from __future__ import annotations

import contextlib

import torch
import torch.nn.functional as F

from .persist import _RoundFwd, _RoundGrad


def _key(t):
    return (t.data_ptr(), tuple(t.shape), t.dtype)


class Recorder:
    """Context manager recording the forward calls of the hopsx autograd ops (conv, BN, GAP, linear,
    padded stem weight) in execution order."""

    def __init__(self):
        self.ops: list[tuple] = []
        self._saved = []

    def __enter__(self):
        from ..ops import functional as HF

        rec = self.ops

        def wrap(cls, kind, pick):
            orig = cls.forward

            def fwd(ctx, *args):
                out = orig(ctx, *args)
                rec.append((kind, pick(args), out))
                return out

            self._saved.append((cls, orig))
            cls.forward = staticmethod(fwd)

        # (x, w, stride, padding, dilation, act, in_affine) / (x, gamma, beta, eps, residual, act) / ...
        wrap(HF._Conv2dFn, "conv", lambda a: (a[0], a[1], a[2], a[3], a[4], a[5], a[6], a[7] if len(a) > 7 else None))
        wrap(HF._BNFn, "bn", lambda a: (a[0], a[1], a[2], a[6], a[7], a[8]))
        wrap(HF._GapFn, "gap", lambda a: (a[0],))
        wrap(HF._LinearFn, "linear", lambda a: (a[0], a[1], a[2], a[3]))
        wrap(HF._PadCinFn, "pad", lambda a: (a[0], a[1]))
        return self

    def __exit__(self, *exc):
        for cls, orig in self._saved:
            cls.forward = orig
        self._saved = []
        return False


def _act(t, a):
    return t.relu() if a == 1 else t


def _cos(a, b):
    a, b = a.double().flatten(), b.double().flatten()
    return float(F.cosine_similarity(a, b, dim=0)) if a.norm() > 0 and b.norm() > 0 else float(torch.equal(a, b))


def reference(model, ops, target, round_grads: bool = True):
    """Build the teacher-forced fp64 graph of the recorded ``ops``, backpropagate the mean cross-entropy
    of the last op's output against ``target``.  Returns (per-op forward report, {param name: fp64 grad})."""
    names = {id(p): n for n, p in model.named_parameters()}
    P = {n: p.detach().double().clone().requires_grad_(True) for n, p in model.named_parameters()}
    env: dict = {}
    wpad: dict = {}
    fwd = []
    rf = _RoundFwd.apply
    rg = _RoundGrad.apply if round_grads else (lambda t: t)

    def act_in(t):
        return env.get(_key(t), None) if t is not None else None

    def get(t):
        v = act_in(t)
        return v if v is not None else t.detach().double()  # a graph input (the normalised image)

    def weight(w):
        if id(w) in wpad:
            return rf(wpad[id(w)])
        return rf(P[names[id(w)]])  # the kernels read the bf16 shadow of the fp32 master

    def force(name, ref, out):
        k = out.detach().double()
        fwd.append((name, _cos(k, ref.detach()), float((k - ref.detach()).abs().max() / ref.detach().abs().max().clamp_min(1e-30))))
        conn = ref + (k - ref).detach()
        if out.dtype == torch.bfloat16:
            conn = rg(conn)  # its gradient is stored as bf16 by the consuming backward
        env[_key(out)] = conn
        return conn

    nconv = nbn = 0
    last = None
    for kind, a, out in ops:
        if kind == "pad":
            w, cp = a
            wpad[id(out)] = F.pad(P[names[id(w)]], (0, int(cp) - w.shape[-1]))
        elif kind == "conv":
            x, w, b, stride, padding, dilation, act, in_aff = a
            xs = get(x).permute(0, 3, 1, 2)
            ws = weight(w).permute(0, 3, 1, 2)
            st = stride if isinstance(stride, (tuple, list)) else (stride, stride)
            pd = padding if isinstance(padding, (tuple, list)) else (padding, padding)
            y = F.conv2d(xs, ws, None, tuple(st), tuple(pd), tuple(dilation) if isinstance(dilation, (tuple, list))
                         else dilation)
            if b is not None:
                y = y + P[names[id(b)]].view(1, -1, 1, 1)
            y = _act(y.permute(0, 2, 3, 1), act)
            last = force(f"conv{nconv}", y, out)
            nconv += 1
        elif kind == "bn":
            x, gamma, beta, eps, residual, act = a
            xs = get(x)
            C = xs.shape[-1]
            x2 = xs.reshape(-1, C)
            mean = x2.mean(0)
            var = x2.var(0, unbiased=False)
            y = (xs - mean) * torch.rsqrt(var + eps) * P[names[id(gamma)]] + P[names[id(beta)]]
            if residual is not None:
                y = y + get(residual)
            last = force(f"bn{nbn}", _act(y, act), out)
            nbn += 1
        elif kind == "gap":
            last = force("gap", get(a[0]).mean((1, 2)), out)
        elif kind == "linear":
            x, w, b, act = a
            y = get(x).reshape(-1, x.shape[-1]) @ weight(w).t()
            if b is not None:
                y = y + P[names[id(b)]]
            last = force("linear", _act(y, act).view(*x.shape[:-1], -1), out)
    F.cross_entropy(last, target).backward()
    return fwd, {n: (p.grad if p.grad is not None else torch.zeros_like(p)) for n, p in P.items()}


def check_step(model, x, y, round_grads: bool = True) -> dict:
    """One forward / backward of ``model`` (training mode) on the kernels, recorded, against the teacher-
    forced fp64 reference.  Returns {"forward": [(op, cos, max rel err)], "grads": {name: (cos, rel L2)}}.
    The model's gradients are left as the step produced them (call ``zero_grad`` before the next)."""
    with Recorder() as rec:
        logits = model(x)
    loss = F.cross_entropy(logits.float(), y)
    loss.backward()
    fwd, ref = reference(model, rec.ops, y, round_grads=round_grads)
    grads = {}
    for n, p in model.named_parameters():
        g = p.grad
        if g is None:
            continue
        r = ref[n]
        grads[n] = (_cos(g, r), float((g.double() - r).norm() / r.norm().clamp_min(1e-30)))
    return {"forward": fwd, "grads": grads, "loss": float(loss.detach())}


def resnet20_check(batch: int = 16, flags: str = "", seed: int = 0) -> dict:
    """``check_step`` of a random-init CIFAR ResNet-20 (training mode) on a random uint8 batch with
    HOPSX_DISABLE=``flags``; adds "min_grad_cos" / "min_fwd_cos" (the worst tensor / op)."""
    from ..models.resnet import cifar_resnet

    with disabled(flags):
        torch.manual_seed(seed)
        m = cifar_resnet(20).to("cuda").train()
        g = torch.Generator().manual_seed(batch + seed)
        x = torch.randint(0, 256, (batch, 32, 32, 3), dtype=torch.uint8, generator=g).to("cuda")
        y = torch.randint(0, 10, (batch,), generator=g).to("cuda")
        r = check_step(m, x, y)
    r["min_grad_cos"] = min(c for c, _ in r["grads"].values())
    r["min_fwd_cos"] = min(c for _, c, _ in r["forward"])
    return r


@contextlib.contextmanager
def disabled(flags: str):
    """HOPSX_DISABLE for the duration (the fusion on/off variants of a check)."""
    import os

    old = os.environ.get("HOPSX_DISABLE", "")
    os.environ["HOPSX_DISABLE"] = flags
    try:
        yield
    finally:
        os.environ["HOPSX_DISABLE"] = old
