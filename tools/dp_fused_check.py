"""Multi-rank check of the fused P2P data-parallel step (csrc/comm/oneshot.hip dp_step_k,
parallel/dp.py fused_update) against the plain all-reduce engine.

Run under torch.distributed.run with N ranks.  On a one-GPU box the ranks share the device and
HOPSX_DIST_BACKEND=gloo carries the handle exchange, barriers and the reference all-reduce.

For the flagship model (MirroredMnistCNN) every rank trains two replicas from the same init on
its own data: A through DataParallel with the fused step (P2P required), B through DataParallel
with P2P off (process-group all-reduce + the fused optimizer kernel).  The comparison uses
SGD + momentum, whose update is linear in the gradient: Adadelta / Adam steps are nearly
sign(g) x const early on, so the last-bit noise of the fp32 atomic gradient accumulation flips
near-zero gradients and A and B legitimately differ by 2 x that constant (tools/dbg_dpfused.py).
Checks:
  * A's fp32 masters are bit-identical on every rank after eager, one-step-graph and
    steps_per_execution-graph steps (verify_replicas);
  * A matches B to fp32 rounding (same grads, same update rule; only the summation order of the
    process-group all-reduce differs);
  * checkpoint.save gathers the owner-only optimizer state: the saved momentum is every slice's
    owner copy.
Rank 0 prints one JSON line prefixed DPFUSED.
"""
import json
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

os.environ.setdefault("HOPSX_P2P", "1")

import torch  # noqa: E402

from hops_examples_amd import checkpoint, optim  # noqa: E402
from hops_examples_amd.models.mnist import MirroredMnistCNN  # noqa: E402
from hops_examples_amd.parallel import dist as hdist  # noqa: E402
from hops_examples_amd.parallel.dp import DataParallel  # noqa: E402
from hops_examples_amd.runtime.arena import ParamArena  # noqa: E402
from hops_examples_amd.runtime.step import TrainStep  # noqa: E402


def build(dev, p2p):
    torch.manual_seed(7)
    m = MirroredMnistCNN().to(dev)
    ParamArena.from_module(m, dev)
    opt = optim.SGD(m, lr=0.05, momentum=0.5)
    dp = DataParallel(m, p2p=p2p)
    return m, opt, dp, TrainStep(m, opt, "sparse_ce", dp=dp, warmup=2, steps_per_execution=4)


def main():
    rank, _, world = hdist.init()
    dev = hdist.device()
    B, nb = 32, 16
    g = torch.Generator(device="cpu").manual_seed(100 + rank)
    xs = torch.randint(0, 256, (nb, B, 28, 28, 1), dtype=torch.uint8, generator=g).to(dev)
    ys = torch.randint(0, 10, (nb, B), dtype=torch.int64, generator=g).to(dev)

    mA, optA, dpA, stA = build(dev, None)
    assert dpA.path.startswith("p2p-xgmi-fused-step"), dpA.path
    want = os.environ.get("HOPSX_DPCHECK_EXPECT")  # e.g. "-zerocopy-overlap": the gradient path under test
    assert want is None or dpA.path == "p2p-xgmi-fused-step" + want, (dpA.path, want)
    mB, optB, dpB, stB = build(dev, False)
    # dropout salts come from a per-instance counter: give B the same masks as A
    for ma, mb in zip(mA.modules(), mB.modules()):
        if hasattr(ma, "salt"):
            mb.salt = ma.salt
    assert dpB.path in ("rccl", "gloo"), dpB.path
    res = {"world": world, "path": dpA.path, "blocks": dpA._oneshot.blocks,
           "ranks_per_device": dpA._oneshot.ranks_per_device, "wire_bytes_per_param": dpA.wire_bytes_per_param,
           "master_sharded": dpA.master_sharded, "buckets": len(dpA.buckets),
           "grad_hbm_bytes_per_param": dpA.grad_hbm_bytes_per_param}

    # eager warm-up (2), capture + one-step replays, then one steps_per_execution replay (4 steps);
    # A then B from the same dropout-RNG state (the RNG tensor is per device, shared by both)
    from hops_examples_amd.ops.functional import rng_state

    rng0 = rng_state(dev).clone()
    init = optA.arena.master.clone()
    first = {}
    for name, st in (("A", stA), ("B", stB)):
        rng_state(dev).copy_(rng0)
        for i in range(6):
            st.step_resident(xs, ys)
            if i == 0:
                st.dp.sync_master()  # ZeRO-1 wire: reassemble the owners' fp32 slices
                torch.cuda.synchronize()
                first[name] = st.opt.arena.master.clone()
        st.run_resident(xs, ys, 4)
        torch.cuda.synchronize()
    # one step: the same gradients (up to the fp32 atomic-accumulation order), an update linear in
    # them -> A equals B to fp32 rounding
    d1 = float((first["A"] - first["B"]).abs().max())
    res["step1_max_abs_diff_vs_allreduce"] = d1
    assert d1 <= 1e-6 * max(1.0, float(first["B"].abs().max())), d1
    res["graph_multi"] = stA._gU is not None
    v = dpA.verify_replicas()
    res["replicas_identical"] = v["identical"]
    assert v["identical"], v
    # ten steps: last-bit differences re-round some bf16 compute weights and flip ReLU / max-pool
    # decisions, so trajectories drift apart chaotically — two runs of the SAME engine reach ~2.4%
    # relative drift by step 10 (tools/dbg_dpfused.py).  A wrong exchange (a missing 1/N, a stale
    # slice) is off by tens of percent from the first step.
    dpA.sync_master()
    dA, dB = optA.arena.master, optB.arena.master
    rel = float((dA - dB).norm() / (dB - init).norm())
    res["rel_drift_vs_allreduce_10_steps"] = rel
    assert rel < 0.1, rel
    assert torch.equal(optA.step_count, optB.step_count), (optA.step_count, optB.step_count)
    lossA = float(stA._outU["loss"].item())
    res["loss"] = round(lossA, 4)
    assert lossA == lossA

    # checkpoint: the moments of every slice (owner-only in fused mode) reach the file
    d = tempfile.mkdtemp(prefix="dpf_ckpt_") if rank == 0 else None
    obj = [d]
    torch.distributed.broadcast_object_list(obj, 0)
    d = obj[0]
    owners = dpA.owner_slices()  # per rank: its slice of every owner piece
    truth = {}
    for k, t in optA.arena.states.items():  # each slice as its owner holds it
        objs = [None] * world
        torch.distributed.all_gather_object(objs, [t[s].cpu() for s in owners[rank]])
        full = torch.empty_like(t).cpu()
        for r in range(world):
            for s, v in zip(owners[r], objs[r]):
                full[s] = v
        truth[k] = full
    p = checkpoint.save(d, mA, optA, step=10)
    if rank == 0:
        sd = torch.load(p, map_location="cpu", weights_only=True)
        for k, t in truth.items():
            assert torch.equal(sd["arena"][k], t), k
        res["ckpt_states_from_owners"] = sorted(truth)
    hdist.barrier()

    # lr change after capture reaches the replayed graph (device hyper-parameters)
    optA.param_groups[0]["lr"] = 0.0
    dpA.sync_master()
    before = optA.arena.master.clone()
    stA.run_resident(xs, ys, 4)
    dpA.sync_master()
    torch.cuda.synchronize()
    res["lr0_frozen"] = bool(torch.equal(before, optA.arena.master))
    assert res["lr0_frozen"]
    optA.param_groups[0]["lr"] = 0.05

    # timing of the fused tail alone (ranks share the GPU here: not an xGMI number)
    for _ in range(5):
        dpA.fused_update(optA)
    torch.cuda.synchronize()
    hdist.barrier()
    t0 = time.perf_counter()
    for _ in range(50):
        dpA.fused_update(optA)
    torch.cuda.synchronize()
    res["us_per_fused_step_tail_shared_gpu"] = round((time.perf_counter() - t0) / 50 * 1e6, 1)
    dpA.close()
    dpB.close()

    # fault injection: one rank's self-test verdict forced to "fail" -> EVERY rank falls back
    os.environ["HOPSX_P2P"] = "auto"
    os.environ["HOPSX_P2P_SELFTEST_FAIL"] = str(world - 1)
    _, _, dpC, _ = build(dev, None)
    res["forced_selftest_fail_path"] = dpC.path
    assert dpC.path in ("rccl", "gloo"), dpC.path
    dpC.close()
    del os.environ["HOPSX_P2P_SELFTEST_FAIL"]
    if rank == 0:
        res["ok"] = True
        print("DPFUSED " + json.dumps(res), flush=True)
    hdist.shutdown()


if __name__ == "__main__":
    main()
