#!/usr/bin/env python3
"""Locate the fused-BN-statistics vs unfused gap of one CIFAR ResNet-20 step, layer by layer.

Run with HOPSX_DETERMINISTIC=1 so that each path is bit-reproducible (every remaining difference is
systematic, not float-atomic order): prints, per module, the relative difference of the forward output
and of the output gradient, and per parameter the cosine of the two paths' gradients.

  HOPSX_DETERMINISTIC=1 python tools/bn_gap.py
"""
from __future__ import annotations

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

dev = torch.device("cuda", 0)


def run(disable: str):
    from hops_examples_amd.models.resnet import cifar_resnet

    os.environ["HOPSX_DISABLE"] = disable
    torch.manual_seed(0)
    m = cifar_resnet(20).to(dev).train()
    g = torch.Generator().manual_seed(3)
    x = torch.randint(0, 256, (16, 32, 32, 3), dtype=torch.uint8, generator=g).to(dev)
    y = torch.randint(0, 10, (16,), generator=g).to(dev)
    acts, grads, names = {}, {}, []

    def fwd_hook(name):
        def h(mod, inp, out):
            if isinstance(out, torch.Tensor):
                acts[name] = out.detach().float().clone()
                if out.requires_grad:
                    out.register_hook(lambda gr: grads.__setitem__(name, gr.detach().float().clone()))
        return h

    for n, mod in m.named_modules():
        if n and not list(mod.children()):
            names.append(n)
            mod.register_forward_hook(fwd_hook(n))
    loss = F.cross_entropy(m(x).float(), y)
    loss.backward()
    torch.cuda.synchronize()
    pg = {n: p.grad.detach().float().clone() for n, p in m.named_parameters() if p.grad is not None}
    os.environ["HOPSX_DISABLE"] = ""
    return names, acts, grads, pg, float(loss)


def rel(a, b):
    return float((a - b).double().norm() / b.double().norm().clamp_min(1e-30))


def main():
    names, a0, g0, p0, l0 = run("bnstats")
    _, a1, g1, p1, l1 = run("")
    print(f"loss unfused {l0:.6f} fused {l1:.6f}")
    print(f"{'module':40s} {'fwd rel':>10s} {'dout rel':>10s}")
    for n in names:
        fr = rel(a1[n], a0[n]) if n in a0 and n in a1 and a0[n].shape == a1[n].shape else float("nan")
        gr = rel(g1[n], g0[n]) if n in g0 and n in g1 and g0[n].shape == g1[n].shape else float("nan")
        print(f"{n:40s} {fr:10.3e} {gr:10.3e}")
    print("parameter gradients (cos fused vs unfused):")
    for n in p0:
        c = float(F.cosine_similarity(p1[n].double().flatten(), p0[n].double().flatten(), dim=0))
        print(f"  {n:40s} cos {c:.6f} rel {rel(p1[n], p0[n]):.3e}")


if __name__ == "__main__":
    main()
