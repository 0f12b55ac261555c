#!/usr/bin/env python3
"""One rank of a data-parallel v2 taxi run (models/widedeep.py TaxiExchange + FusedWideDeepStep): every
rank trains on its own synthetic examples with the gradients exchanged inside the launch, then writes its
data, the initial and the final state to <out>/rank<r>.pt for tests/test_taxi_dp_gpu.py (which checks
the replicas bit-identical and against the fp64 reference of the global batch).  ``--bench K``: also
time K more steps (steps/s per rank, max over ranks) into <out>/bench.json.

Launch: python -c "from hops_examples_amd.parallel import launch; launch.launch(W, ['tools/taxi_dp_worker.py',
...], rehearse=True)" — W processes; on one GPU they share it (the step is one workgroup), gloo process group.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--steps", type=int, default=12)
    ap.add_argument("--spe", type=int, default=4)  # steps per launch
    ap.add_argument("--batch", type=int, default=40)
    ap.add_argument("--nb", type=int, default=4)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--bench", type=int, default=0)
    ap.add_argument("--phases", action="store_true", help="rank 0 prints the exchanging step's phase stamps")
    a = ap.parse_args()
    if a.phases:
        os.environ["HOPSX_PHASE_DBG"] = "1"
    import torch
    import torch.distributed as dist

    from hops_examples_amd.models import widedeep as WD
    from hops_examples_amd.parallel import dist as hdist
    from hops_examples_amd.runtime.arena import ParamArena

    rank, _, world = hdist.init()
    dev = hdist.device()
    torch.manual_seed(a.seed)
    m = WD.TaxiWideDeep()
    with torch.no_grad():
        m.wide.weight.normal_(0, 0.05)  # a trained-looking wide part (all-zero makes FTRL trivial)
    m = m.to(dev)
    ParamArena.from_module(m, dev)
    opt = WD.make_optimizer(m)
    B, nb = a.batch, a.nb
    dense, cat, label = WD.synth_taxi(nb * B, seed=a.seed + 100 + 7 * rank)
    dense, cat, label = dense.view(nb, B, -1), cat.view(nb, B, -1), label.view(nb, B, 1)
    xdp = WD.TaxiExchange(dev, world)
    fs = WD.FusedWideDeepStep(m, opt, xdp=xdp)
    assert fs.ok(B) and fs.kernel == "v2-dp", fs.kernel
    arena = m.wide.weight._hx_arena
    xdp.sync_replicas(arena)
    init = WD.reference_state(m, fs)
    xs, ys = (dense.to(dev), cat.to(dev)), label.to(dev)
    fs.steps_per_execution = a.spe
    fs.run_resident(xs, ys, a.steps)
    torch.cuda.synchronize()
    fs.check()
    final = {"master": arena.master.cpu(), "ada": arena.state("adagrad_s0").cpu(),
             "z": arena.state("ftrl_s0").cpu(), "n": arena.state("ftrl_s1").cpu(),
             "shadow": arena.shadow.float().cpu(), "loss": float(fs.loss.item()), "cursor": int(fs.cursor.item()),
             "steps_ada": float(opt.opts[1].step_count.item())}
    torch.save({"rank": rank, "world": world, "dense": dense, "cat": cat, "label": label, "init": init,
                "final": final, "digest": fs.digest(), "steps": a.steps}, os.path.join(a.out, f"rank{rank}.pt"))
    if a.bench:
        fs.steps_per_execution = 32
        fs.run_resident(xs, ys, 64)  # warm
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        fs.run_resident(xs, ys, a.bench)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        dist.barrier()
        fs.check()
        els = [None] * world
        dist.all_gather_object(els, el)
        digs = [None] * world
        dist.all_gather_object(digs, fs.digest())
        if rank == 0:
            mx = max(els)
            with open(os.path.join(a.out, "bench.json"), "w") as f:
                json.dump({"world": world, "steps": a.bench, "steps_per_sec_per_rank": round(a.bench / mx, 1),
                           "us_per_step": round(mx / a.bench * 1e6, 2), "replicas_identical": all(d == digs[0] for d in digs),
                           "kernel": fs.kernel}, f)
    if a.phases:
        # stamps (100 MHz): 7 last step start, 2 FWD, 3 B3, 4 B2, 5 B1, 6 B0 end, 31 pushes drained,
        # 25 peers' flags seen, 28 deep applied, 30 apply end; 1 prologue end, 19 launch end
        rows = [("FWD", 7, 2), ("B3", 2, 3), ("B2", 3, 4), ("B1", 4, 5), ("B0", 5, 6), ("drain+bar", 6, 31),
                ("flag wait", 31, 25), ("apply deep", 25, 28), ("apply wide+img", 28, 30), ("write-back", 30, 19)]
        acc = {}
        fs.steps_per_execution = 32
        for it in range(10):
            fs.run_resident(xs, ys, 32)
            torch.cuda.synchronize()
            t = fs.dbg.cpu().tolist()
            if it >= 2:
                acc.setdefault("per step (mean)", []).append((t[19] - t[1]) / 32 / 100.0)
                for name, a0, a1 in rows:
                    acc.setdefault(name, []).append((t[a1] - t[a0]) / 100.0)
        if rank == 0:
            with open(os.path.join(a.out, "phases.txt"), "w") as f:
                f.write(f"# taxi v2-dp, world {world} (ranks sharing one GPU), last step of a 32-step launch, us\n")
                for k, v in acc.items():
                    f.write(f"{k:18s} {sum(v) / len(v):8.3f}\n")
    xdp.close()
    hdist.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
