#!/usr/bin/env python3
"""Per-element look at the persistent step's one-step update against the bf16-emulating and pure
fp64 references (tests/test_persist_gpu.py setup): which elements disagree, and how large their
gradients are (|g| from E[g^2] = (1 - rho) g^2 after one step).

  python tools/persist_diag.py [--seeds 0 1 2]
"""
from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))

import torch  # noqa: E402

import test_persist_gpu as T  # noqa: E402
from hops_examples_amd.runtime import persist  # noqa: E402


def one(seed):
    m, opt, eng, xs, ys = T._setup(seed)
    P0, S10, S20, _ = T._snapshot(m, eng)
    rng0 = eng.rng.clone().cpu()
    eng.run_resident(xs, ys, 1)
    torch.cuda.synchronize()
    eng.check()
    P1, S11, _, _ = T._snapshot(m, eng)
    lk = float(eng.losses(1)[0, 0])
    refs, mg = {}, []
    for emu in (True, False):
        refs[emu] = persist.reference_steps(P0, S10, S20, xs, ys, 0, 1, int(rng0[0]) & ((1 << 64) - 1), int(rng0[1]),
                                            int(m.pool.salt), float(m.pool.dropout), 1.0, 0.95, 1e-7,
                                            emulate_bf16=emu, margins=mg if emu else None)
    print(f"seed {seed}: loss kernel {lk:.7f} emu {refs[True][3][0]:.7f} fp64 {refs[False][3][0]:.7f} "
          f"relu margins {mg[0]} | rng {rng0.tolist()} salt {int(m.pool.salt)} "
          f"sum(P0) {sum(float(v.double().sum()) for v in P0.values()):.9f} sum(x) {int(xs.long().sum())}")
    for k in eng.PARAMS:
        dk = (P1[k] - P0[k]).double().flatten()
        de = (refs[True][0][k] - P0[k].double()).flatten()
        df = (refs[False][0][k] - P0[k].double()).flatten()
        ge = (refs[True][1][k].flatten() / 0.05).sqrt()
        gk = (S11[k].double().flatten() / 0.05).sqrt()
        e_ke, e_ef = (dk - de).abs(), (de - df).abs()
        cos = lambda a, b: torch.nn.functional.cosine_similarity(a, b, dim=0).item()  # noqa: E731
        print(f"  {k:14s} n {dk.numel():7d} kernel~emu cos {cos(dk, de):.6f} max {e_ke.max():.2e} "
              f">1e-4 {int((e_ke > 1e-4).sum()):4d} | emu~fp64 cos {cos(de, df):.6f} max {e_ef.max():.2e} "
              f">1e-4 {int((e_ef > 1e-4).sum()):4d} | kernel~fp64 cos {cos(dk, df):.6f} "
              f"| |g| median {ge.median():.2e}")
        if k == "conv1.weight" or int((e_ke > 1e-4).sum()) > dk.numel() // 1000:
            idx = torch.argsort(e_ke, descending=True)[:6]
            for i in idx.tolist():
                print(f"      [{i:5d}] dk {dk[i]:+.4e} demu {de[i]:+.4e} dfp64 {df[i]:+.4e} "
                      f"|g| kernel {gk[i]:.3e} emu {ge[i]:.3e}")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", type=int, nargs="+", default=[0, 1, 2])
    for s in ap.parse_args().seeds:
        one(s)
