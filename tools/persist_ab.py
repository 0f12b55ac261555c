"""Interleaved in-process A/B of persistent-flagship launch knobs (env variables read by the host wrapper at
every launch, e.g. HOPSX_PERSIST_POLLW_C): alternates the settings R times over the same engine and data,
each a timed run of N steps, and prints per-setting median / min ms per step — one box, one process, so
box-to-box variance cannot fake a difference.
usage (GPU): python tools/persist_ab.py "HOPSX_PERSIST_POLLW_C=1" "HOPSX_PERSIST_POLLW_C=4" [--reps 8 --steps 256]"""
import argparse
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("settings", nargs="+")
    ap.add_argument("--reps", type=int, default=8)
    ap.add_argument("--steps", type=int, default=256)
    a = ap.parse_args()
    from hops_examples_amd import optim
    from hops_examples_amd.models.mnist import MirroredMnistCNN
    from hops_examples_amd.runtime.arena import ParamArena
    from hops_examples_amd.runtime.step import make_step

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    m = MirroredMnistCNN().to(dev)
    ParamArena.from_module(m, dev)
    st = make_step(m, optim.Adadelta(m, lr=1.0), "sparse_ce", batch=32)
    assert st.kind == "persistent", st.note
    xs = torch.randint(0, 256, (1920, 32, 28, 28, 1), dtype=torch.uint8, device=dev)
    ys = torch.randint(0, 10, (1920, 32), device=dev)
    st.run_resident(xs, ys, 64)
    torch.cuda.synchronize()
    res = {s: [] for s in a.settings}
    base = dict(os.environ)
    for _ in range(a.reps):
        for s in a.settings:
            os.environ.clear()
            os.environ.update(base)
            for kv in s.split():
                k, v = kv.split("=", 1)
                os.environ[k] = v
            from hops_examples_amd.runtime.persist import _ext as persist_ext
            persist_ext().mnist_persist_reload_knobs()  # the host wrapper caches the knobs otherwise
            st.run_resident(xs, ys, 32)  # one untimed launch with the setting
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            st.run_resident(xs, ys, a.steps)
            torch.cuda.synchronize()
            res[s].append((time.perf_counter() - t0) / a.steps * 1e3)
    os.environ.clear()
    os.environ.update(base)
    st.check()
    for s, v in res.items():
        med = statistics.median(v)
        print(f"[{s}] median {med:.4f} ms/step ({32 / med * 1e3:,.0f} img/s)  min {min(v):.4f}  n={len(v)}")


if __name__ == "__main__":
    main()
