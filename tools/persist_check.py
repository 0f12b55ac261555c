#!/usr/bin/env python3
"""Persistent flagship step: numerics vs the fp64 reference and per-phase timing from in-kernel
wall-clock stamps (runtime/persist.py, csrc/ops/mnist_persist.hip).

  python tools/persist_check.py [--steps 8] [--timing 32]
"""
from __future__ import annotations

import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from hops_examples_amd import optim  # noqa: E402
from hops_examples_amd.models.mnist import MirroredMnistCNN  # noqa: E402
from hops_examples_amd.runtime import persist  # noqa: E402
from hops_examples_amd.runtime.arena import ParamArena  # noqa: E402


def setup(seed, spl, stamps=False, nb=8, loopback=0):
    torch.manual_seed(seed)
    dev = torch.device("cuda", 0)
    m = MirroredMnistCNN().to(dev)
    ParamArena.from_module(m, dev)
    opt = optim.Adadelta(m, lr=1.0)
    xs = torch.randint(0, 256, (nb, 32, 28, 28, 1), dtype=torch.uint8, device=dev)
    ys = torch.randint(0, 10, (nb, 32), dtype=torch.int64, device=dev)
    return m, opt, persist.PersistentMnistStep(m, opt, steps_per_launch=spl, debug_stamps=stamps,
                                                                  loopback=loopback), xs, ys


def numerics(n):
    m, opt, eng, xs, ys = setup(0, 32)
    named = dict(m.named_parameters())
    sl = lambda t, k: t[named[k]._hx_off:named[k]._hx_off + named[k].numel()].view_as(named[k]).clone()  # noqa: E731
    P0 = {k: named[k].detach().clone() for k in eng.PARAMS}
    S10 = {k: sl(eng.s1, k) for k in eng.PARAMS}
    S20 = {k: sl(eng.s2, k) for k in eng.PARAMS}
    rng0 = eng.rng.clone().cpu()
    eng.run_resident(xs, ys, n)
    torch.cuda.synchronize()
    eng.check()
    lk = eng.losses(n)[:, 0].cpu().tolist()
    print("loss kernel        ", [round(v, 5) for v in lk])
    for emu in (False, True):
        Pr, S1r, S2r, lr_ = persist.reference_steps(P0, S10, S20, xs, ys, 0, n, int(rng0[0]) & ((1 << 64) - 1),
                                                    int(rng0[1]), int(m.pool.salt), float(m.pool.dropout), 1.0, 0.95,
                                                    1e-7, emulate_bf16=emu)
        print(f"loss ref (bf16={int(emu)})  ", [round(v, 5) for v in lr_])
        for k in eng.PARAMS:
            dk = (named[k].detach() - P0[k]).double().flatten()
            dr = (Pr[k] - P0[k].double()).flatten()
            cos = torch.nn.functional.cosine_similarity(dk, dr, dim=0).item()
            rel = ((dk - dr).norm() / dr.norm()).item()
            mx = (dk - dr).abs().max().item()
            big = ((dk - dr).abs() > 1e-4).double().mean().item()
            s1k = sl(eng.s1, k).double().flatten()
            srel = ((s1k - S1r[k].flatten()).norm() / S1r[k].norm()).item()
            print(f"  {k:14s} cos {cos:.6f} rel {rel:.5f} maxabs {mx:.3e} frac>1e-4 {big:.5f} "
                  f"|dref|max {dr.abs().max().item():.3e} s1 rel {srel:.6f}")


def timing(n, reps=5, loopback=0):
    m, opt, eng, xs, ys = setup(1, n, stamps=True, nb=64, loopback=loopback)
    eng.run_resident(xs, ys, n)  # warm
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        eng.run_resident(xs, ys, n)
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) / n * 1e6)
    eng.check()
    st = eng.phase_stamps(n).cpu().double() * 0.01  # us
    pos, head = st[:169], st[169:]
    own = pos[:162]
    step_us = (pos[:, 2:, 0] - pos[:, 1:-1, 0]).median().item()
    print(f"[loopback {loopback}] host wall {min(ts):.2f} us/step (best of {reps}), in-kernel step {step_us:.2f} us")
    # launch boundaries (stamps 13: workgroup entry in step 0, 14: write-back issued in the last step)
    entry, first = pos[:, 0, 13], pos[:, 0, 0]
    wb = pos[:, n - 1, 14]
    print(f"  launch: workgroup entry spread {(entry.max() - entry.min()).item():.2f} us; prologue (entry -> step 0) "
          f"median {(first - entry).median().item():.2f} max {(first - entry).max().item():.2f} us; step 0 "
          f"{(pos[:, 1, 0] - pos[:, 0, 0]).median().item():.2f} us; last step end -> write-back issued "
          f"{(wb - pos[:, n - 1, 11]).median().item():.2f} us; first entry -> last write-back "
          f"{(wb.max() - entry.min()).item():.2f} us = {(wb.max() - entry.min()).item() / n:.2f} us/step over {n} steps")

    def med(t, a, b):
        return (t[:, 1:, b] - t[:, 1:, a]).median().item()

    rows = [("conv fwd (input, conv1, conv2 MFMA, pool, dropout)", pos, 0, 1), ("fc1 partial + publish A", pos, 1, 2),
            ("wait B (heads)", pos, 2, 3), ("dh load + fc1 wgrad/dgrad + pool bwd", pos, 3, 4),
            ("conv2 wgrad/dgrad + conv1 wgrad", pos, 4, 5), ("publish C", pos, 5, 6),
            ("owner: wait C", own, 6, 7), ("owner: slice reduce + update + publish D", own, 7, 8),
            ("owner: fc1 slice Adadelta", own, 8, 9), ("wait D", pos, 9, 10), ("D load", pos, 10, 11)]
    for nm, t, a, b in rows:
        print(f"  {nm:48s} {med(t, a, b):7.2f} us")
    lastA = pos[:, 1:, 2].max(dim=0).values
    lastC = pos[:, 1:, 6].max(dim=0).values
    lastD = own[:, 1:, 8].max(dim=0).values
    print(f"  head: last A publish -> A ready {(head[:, 1:, 0] - lastA).median().item():.2f} us; head compute + "
          f"B publish {(head[:, 1:, 1] - head[:, 1:, 0]).median().item():.2f} us; fc2 update "
          f"{(head[:, 1:, 2] - head[:, 1:, 1]).median().item():.2f} us")
    print(f"  skew: C publish spread {(pos[:, 1:, 6].max(0).values - pos[:, 1:, 6].min(0).values).median().item():.2f} us; "
          f"last C publish -> owners' C ready {(own[:, 1:, 7] - lastC).median().item():.2f} us; "
          f"last D publish -> D ready {(pos[:, 1:, 10] - lastD).median().item():.2f} us")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--timing", type=int, default=32)
    ap.add_argument("--loopback", type=int, nargs="*", default=[],
                    help="also time the data-parallel instantiation playing these world sizes in-process")
    ap.add_argument("--timing-only", action="store_true")
    a = ap.parse_args()
    if not a.timing_only:
        numerics(1)
        numerics(a.steps)
    timing(a.timing)
    for w in a.loopback:
        timing(a.timing, loopback=w)
