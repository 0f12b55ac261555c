#!/usr/bin/env python3
"""Deterministic-mode evidence (run with HOPSX_DETERMINISTIC=1; tests/test_deterministic_gpu.py runs it
in a subprocess): replays that the default mode only reproduces up to float-atomic order must be
bit-identical.  Prints one JSON object.

  HOPSX_DETERMINISTIC=1 python tools/det_check.py
"""
from __future__ import annotations

import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from hops_examples_amd import optim  # noqa: E402
from hops_examples_amd.models.mnist import MirroredMnistCNN  # noqa: E402
from hops_examples_amd.ops import _C  # noqa: E402
from hops_examples_amd.ops import functional as HF  # noqa: E402
from hops_examples_amd.runtime.arena import ParamArena  # noqa: E402
from hops_examples_amd.runtime.step import TrainStep  # noqa: E402

dev = torch.device("cuda", 0)


def _data(nb=6, B=32, seed=5):
    g = torch.Generator().manual_seed(seed)
    xs = torch.randint(0, 256, (nb, B, 28, 28, 1), dtype=torch.uint8, generator=g).to(dev)
    ys = torch.randint(0, 10, (nb, B), generator=g).to(dev)
    return xs, ys


def _model(seed=0, salt=7919):
    HF.seed_device_rng(11, dev)
    torch.manual_seed(seed)
    m = MirroredMnistCNN().to(dev)
    m.pool.salt = salt
    ParamArena.from_module(m, dev)
    return m


def mnist_replay(mode: str, n=15):
    """mode: 'u' = steps_per_execution graph (run_resident), '1' = one-step graph replays, 'eager'."""
    xs, ys = _data()
    m = _model()
    w0 = m._hx_arena.master.clone()
    st = TrainStep(m, optim.SGD(m, lr=0.05), "sparse_ce", graph=mode != "eager", steps_per_execution=8)
    losses = []
    if mode == "u":
        r = st.run_resident(xs, ys, n)
        losses.append(float(r["loss"].reshape(-1)[0]))
    else:
        for _ in range(n):
            r = st.step_resident(xs, ys)
        losses.append(float(r["loss"].reshape(-1)[0]))
    torch.cuda.synchronize()
    return m._hx_arena.master - w0, losses


def mnist_adadelta(colaunch: str, steps=6):
    os.environ["HOPSX_OPT_COLAUNCH"] = colaunch
    xs, ys = _data()
    m = _model()
    w0 = m._hx_arena.master.clone()
    st = TrainStep(m, optim.Adadelta(m, lr=1.0), "sparse_ce", graph=True, warmup=2)
    for i in range(steps):
        r = st(xs[i % xs.shape[0]], ys[i % ys.shape[0]])
    torch.cuda.synchronize()
    return m._hx_arena.master - w0, float(r["loss"].reshape(-1)[0])


def resnet_step(disable: str):
    from hops_examples_amd.models.resnet import cifar_resnet

    os.environ["HOPSX_DISABLE"] = disable
    torch.manual_seed(0)
    m = cifar_resnet(20).to(dev).train()
    g = torch.Generator().manual_seed(3)
    x = torch.randint(0, 256, (16, 32, 32, 3), dtype=torch.uint8, generator=g).to(dev)
    y = torch.randint(0, 10, (16,), generator=g).to(dev)
    loss = F.cross_entropy(m(x).float(), y)
    loss.backward()
    torch.cuda.synchronize()
    os.environ["HOPSX_DISABLE"] = ""
    return torch.cat([p.grad.float().reshape(-1) for p in m.parameters() if p.grad is not None])


def rel(a, b):
    return float((a - b).double().norm() / b.double().norm().clamp_min(1e-30))


def main():
    out = {"deterministic": _C.deterministic()}
    a1, l1 = mnist_replay("1")
    a2, l2 = mnist_replay("1")
    out["mnist_1step_replays_bitwise"] = bool(torch.equal(a1, a2)) and l1 == l2
    u1, lu1 = mnist_replay("u")
    u2, lu2 = mnist_replay("u")
    out["mnist_ugraph_replays_bitwise"] = bool(torch.equal(u1, u2)) and lu1 == lu2
    out["mnist_ugraph_vs_1step_bitwise"] = bool(torch.equal(u1, a1))
    out["mnist_ugraph_vs_1step_rel"] = rel(u1, a1)
    e1, _ = mnist_replay("eager")
    out["mnist_eager_vs_graph_bitwise"] = bool(torch.equal(e1, a1))
    out["mnist_eager_vs_graph_rel"] = rel(e1, a1)
    c1, lc1 = mnist_adadelta("1")
    c1b, _ = mnist_adadelta("1")
    c0, lc0 = mnist_adadelta("0")
    c0b, _ = mnist_adadelta("0")
    out["adadelta_graph_replays_bitwise"] = bool(torch.equal(c0, c0b)) and bool(torch.equal(c1, c1b))
    out["adadelta_colaunch_vs_unfused_bitwise"] = bool(torch.equal(c1, c0))
    out["adadelta_colaunch_vs_unfused_rel"] = rel(c1, c0)
    g1 = resnet_step("bnstats")
    g2 = resnet_step("bnstats")
    g3 = resnet_step("")
    g4 = resnet_step("")
    out["resnet20_unfused_bitwise"] = bool(torch.equal(g1, g2))
    out["resnet20_bnstats_bitwise"] = bool(torch.equal(g3, g4))
    out["resnet20_bnstats_vs_unfused_cos"] = float(F.cosine_similarity(g3.double(), g1.double(), dim=0))
    out["det_turns_lost"] = int(_C.ext().det_lost())
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
