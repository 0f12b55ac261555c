"""The persistent flagship's data-parallel exchange with DIFFERENT data on every rank
(runtime/persist_sim.py ExchangeSim, runtime/persist_peer.py), against a bf16-emulating fp64
reference of the MirroredStrategy global-batch step.

The loopback tests (test_persist_dp_gpu.py) feed every "peer" this rank's own batch, so they cannot
see a dropped peer, a wrong world-size scale or a mis-ordered slot.  Here one process plays W ranks
through the REAL (non-loopback) exchange code: each rank's payload is harvested from a launch as that
rank on its own batch, then injected into every other rank's exchange buffer; the W replicas' updates
must be bit-identical to each other and match the fp64 step of the concatenated global batch
(rank r's images are global images 32r..32r+31, the kernel's dropout key).  A second test moves the
peers into another PROCESS, whose payload pushes and flag stores go through IPC mappings of uncached
memory while the active kernel spins.

Reference workload: notebooks/ml/Distributed_Training/mirrored_strategy/
mirroredstrategy_mnist_example.ipynb:125-131 (global batch = 32 x replicas), :189-231.
"""
import json
import os
import subprocess
import sys
import time

import pytest
import torch

pytestmark = pytest.mark.gpu
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from hops_examples_amd import optim  # noqa: E402
from hops_examples_amd.models.mnist import MirroredMnistCNN  # noqa: E402
from hops_examples_amd.runtime import persist  # noqa: E402
from hops_examples_amd.runtime.arena import ParamArena  # noqa: E402
from hops_examples_amd.runtime.persist_sim import REGIONS, ExchangeSim  # noqa: E402

B = 32
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _setup(world, seed=1, nb=3):
    from hops_examples_amd.ops import functional as HF

    dev = torch.device("cuda", 0)
    torch.manual_seed(seed)
    HF.seed_device_rng(11, dev)
    m = MirroredMnistCNN().to(dev)
    m.pool.salt = 7919
    ParamArena.from_module(m, dev)
    opt = optim.Adadelta(m, lr=1.0)
    sim = ExchangeSim(world)
    eng = persist.PersistentMnistStep(m, opt, steps_per_launch=1, exchange=sim, timeout_s=5)
    return m, opt, eng, sim


def _snapshot(eng):
    V = eng.views()
    return ({k: v[0].detach().clone() for k, v in V.items()}, {k: v[1].detach().clone() for k, v in V.items()},
            {k: v[2].detach().clone() for k, v in V.items()})


def _batches(eng, world, nb, steps, base_seed, tries=24, need=4e-6):
    """Per-rank epochs whose first ``steps`` global batches keep every fc1 ReLU input clear of 0 in the
    reference (a tie there flips a whole fc1 row between fp32 and fp64 accumulation): of ``tries``
    candidate seeds the one with the largest smallest |fc1 input|, which must exceed the fp32
    accumulation error over K = 10816 (~1e-6).  W x 32 x 128 inputs per step make 2e-5-clear sets rare
    at W = 8, so the test takes the clearest instead of demanding a fixed margin."""
    dev = eng.device
    best = (-1.0, None)
    for s in range(base_seed, base_seed + tries):
        g = torch.Generator().manual_seed(s)
        xs = [torch.randint(0, 256, (nb, B, 28, 28, 1), dtype=torch.uint8, generator=g).to(dev) for _ in range(world)]
        ys = [torch.randint(0, 10, (nb, B), dtype=torch.int64, generator=g).to(dev) for _ in range(world)]
        P0, S10, S20 = _snapshot(eng)
        mg = []
        _ref(eng, P0, S10, S20, xs, ys, steps, margins=mg)
        m = min(x["fc1"] for x in mg)
        if m > best[0]:
            best = (m, (xs, ys))
        if m > 2e-5:
            break
    assert best[0] > need, f"no batch set clear of an fc1 ReLU tie (best margin {best[0]:.2e})"
    print(f"[batches] W={world} steps={steps} smallest |fc1 input| {best[0]:.2e}")
    return best[1]


def _ref(eng, P0, S10, S20, xs, ys, n, margins=None):
    rng = eng.rng.cpu()
    pool = eng.model.pool
    return persist.reference_steps(P0, S10, S20, torch.cat(xs, dim=1), torch.cat(ys, dim=1), int(eng.cursor.item()),
                                   n, int(rng[0]) & ((1 << 64) - 1), int(rng[1]), int(pool.salt),
                                   float(pool.dropout), 1.0, 0.95, 1e-7, emulate_bf16=True, margins=margins)


def _check_replicas(res):
    for r in res[1:]:
        for k in ("master", "shadow", "s1", "s2"):
            assert torch.equal(r[k], res[0][k]), f"replica state {k} differs"


def _step_and_check(eng, sim, xs, ys, world, tag, cmin_big=0.99999, cmin_small=0.9999, tie_margin=0.0):
    """One simulated DP step from the engine's CURRENT state against the fp64 one-step reference from
    that same state: replicas bit-identical, the global loss, and per tensor the update cosine, the
    off-by-more-than-7%-of-a-step element count and E[g^2] (the bounds of tests/test_persist_gpu.py).
    Returns the global-batch mean loss."""
    P0, S10, S20 = _snapshot(eng)
    mg = []
    Pr, S1r, _, lref = _ref(eng, P0, S10, S20, xs, ys, 1, margins=mg)
    # an fc1 ReLU input within tie_margin of 0 (from the kernel's own state): fp32-vs-fp64 accumulation may
    # flip it, which moves that fc1 row's gradient and, through dh, every conv gradient — such a step that
    # misses the strict bounds is held to cos > 0.999 instead (and reported as relaxed)
    tie = mg[0]["fc1"] < tie_margin
    res = sim.step(xs, ys)
    _check_replicas(res)
    P1, S11, _ = _snapshot(eng)
    # the replicas' local mean losses average to the global-batch mean
    gl = sum(r["loss"] for r in res) / world
    assert abs(gl - lref[0]) < 1e-5 * lref[0], (tag, gl, lref)
    assert len({r["loss"] for r in res}) > 1, "the replicas must have trained on different batches"
    bad, loose_bad = [], []
    for k in eng.PARAMS:
        dk = (P1[k] - P0[k]).double().flatten()
        dr = (Pr[k] - P0[k].double()).flatten()
        cos = float(torch.nn.functional.cosine_similarity(dk, dr, dim=0))
        err = (dk - dr).abs()
        nbad = int((err > 1e-4).sum())
        sk, sr = S11[k].double().flatten(), S1r[k].flatten()
        srel = float((sk - sr).norm() / sr.norm())
        print(f"[{tag}] {k:13s} cos {cos:.7f} max|err| {float(err.max()):.2e} E[g^2] rel {srel:.2e}")
        cmin = cmin_big if err.numel() >= 1024 else cmin_small
        # one element per tensor may sit on a ReLU / max-pool tie that fp32-vs-fp64 accumulation flips
        # (a 64-channel bias sums W x 32 x 144 conv2 output gradients: measured 1 of 64 at W=4, 1.1e-4)
        msg = f"{k}: cos {cos:.7f} off {nbad}/{err.numel()} max {float(err.max()):.3e} E[g^2] rel {srel:.5f}"
        if not (cos > cmin and nbad <= max(1, err.numel() // 1000) and float(err.max()) <= 2 * 1.42e-3 and srel < 1e-2):
            bad.append(msg)
        if not (cos > 0.999 and float(err.max()) <= 2 * 1.42e-3 and srel < 1e-2):
            loose_bad.append(msg)
    relaxed = bool(bad) and tie
    if relaxed:
        print(f"[{tag}] relaxed (fc1 input {mg[0]['fc1']:.1e} from a ReLU tie): " + "; ".join(bad))
    assert not (loose_bad if relaxed else bad), f"{tag}: " + "; ".join(loose_bad if relaxed else bad)
    return gl, relaxed


@pytest.mark.parametrize("world", [2, 4, 8])
def test_sim_one_step_matches_fp64_global_batch(world):
    """One MirroredStrategy step of W replicas on W different batches: bit-identical replicas, and every
    parameter tensor's update within fp32-vs-fp64 accumulation noise of the global-batch reference
    (the same bounds as the one-GPU test, tests/test_persist_gpu.py)."""
    m, opt, eng, sim = _setup(world)
    try:
        xs, ys = _batches(eng, world, 3, 1, 100 * world)
        _, tie = _step_and_check(eng, sim, xs, ys, world, f"1-step W={world}")
        assert not tie
    finally:
        sim.close()


@pytest.mark.parametrize("world", [2, 4, 8])
def test_sim_four_steps_track_fp64(world):
    """Four consecutive data-parallel steps (cursor, RNG counter, Adadelta state and cross-rank epochs
    carried from step to step): EVERY step, from the kernel's state at its start, meets the one-step
    bounds against fp64; replicas stay bit-identical; and the loss trajectory stays on the free-running
    fp64 reference.  (Over several steps the free-running references drift apart from the kernel by the
    same mechanism as on one GPU — Adadelta's nearly sign-like first steps amplify fp32-vs-fp64 noise in
    near-zero gradients — so the trajectory check uses test_persist_gpu.py's 1e-3, and the per-step
    anchoring carries the tight bounds.  A step that misses them while one of its fc1 inputs, from the
    kernel's own state, is within 1e-5 of a ReLU tie — at W = 8 there are 32,768 per step — is held to
    cos > 0.999 instead, and at most half the steps may be such.)"""
    n = 4
    m, opt, eng, sim = _setup(world, seed=2)
    try:
        # 4 steps x W x 32 x 128 fc1 inputs: at W = 8 the clearest of 40 seeds is ~3e-6 from a tie
        xs, ys = _batches(eng, world, 5, n, 1000 + world, tries=40, need=2e-6)
        P0, S10, S20 = _snapshot(eng)
        *_, lref = _ref(eng, P0, S10, S20, xs, ys, n)
        out = [_step_and_check(eng, sim, xs, ys, world, f"step {i + 1}/{n} W={world}", tie_margin=1e-5)
               for i in range(n)]
        losses = [o[0] for o in out]
        assert sum(o[1] for o in out) <= n // 2, "most steps must meet the strict bounds"
        assert torch.allclose(torch.tensor(losses, dtype=torch.float64), torch.tensor(lref, dtype=torch.float64),
                              rtol=1e-3, atol=0), (losses, lref)
        assert int(eng.cursor.item()) == n and float(opt.step_count.item()) == n
    finally:
        sim.close()


def test_selftest_is_numerical_and_catches_a_dropped_peer():
    """The self-test compares a DP step with the fp64 global-batch reference: it passes on a correct
    exchange and fails when one peer's contribution is dropped (every replica would be wrong the same
    way, so the old bit-identity check alone passed it)."""
    m, opt, eng, sim = _setup(4, seed=3)
    try:
        before = eng.param_digest()
        assert eng.selftest(), eng.selftest_report
        rep = eng.selftest_report["numeric"]
        assert min(c for c, _ in rep["tensors"].values()) > 0.999
        sim.drop = 2
        assert not eng.selftest()
        bad = eng.selftest_report["numeric"]["tensors"]
        assert max(s for _, s in bad.values()) > 0.1, bad  # E[g^2] far off: a quarter of the gradient missing
        assert eng.param_digest() == before  # the pre-flight leaves the real state untouched
    finally:
        sim.close()


def test_numeric_probe_catches_a_wrong_scale_in_loopback():
    """Loopback (every peer = this rank) against the probe: passes as is, and a reference that
    pretends the world is twice as large (the gradient scaled by the wrong world size) fails on E[g^2]."""
    from hops_examples_amd.ops import functional as HF

    dev = torch.device("cuda", 0)
    torch.manual_seed(4)
    HF.seed_device_rng(5, dev)
    mm = MirroredMnistCNN().to(dev)
    ParamArena.from_module(mm, dev)
    o = optim.Adadelta(mm, lr=1.0)
    eng = persist.PersistentMnistStep(mm, o, steps_per_launch=4, loopback=2, timeout_s=5)
    try:
        assert eng.numeric_probe()["ok"]
        bad = eng.numeric_probe(reduce=lambda f: f * 4)
        # E[g^2] ~ g^2: a gradient 2x off leaves the kernel's at 1/4 of the reference's (rel error 0.75)
        assert not bad["ok"] and max(s for _, s in bad["tensors"].values()) > 0.5
    finally:
        eng.close()


def _peer_proc():
    env = dict(os.environ, PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
    return subprocess.Popen([sys.executable, "-u", "-m", "hops_examples_amd.runtime.persist_peer"], cwd=ROOT, env=env,
                            stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True)


def _rd(p):
    line = p.stdout.readline()
    assert line, f"peer process ended (rc {p.poll()})"
    return json.loads(line)


def _wr(p, obj):
    p.stdin.write(json.dumps(obj) + "\n")
    p.stdin.flush()


@pytest.mark.parametrize("world", [2, 4])
def test_cross_process_peer(world, tmp_path):
    """Rank 0 runs the real DP kernel; ranks 1..W-1 are a second PROCESS on the same GPU that maps
    rank 0's uncached exchange buffer and flag page over IPC and, while rank 0's kernel spins, pushes
    their payloads with system-scope stores and then raises rank 0's flags.  Rank 0's kernel pushes into
    the second process's buffer.  Both directions must carry exactly the single-process payloads, and
    rank 0's update must be bit-identical to the single-process replica's."""
    from hops_examples_amd.parallel import oneshot

    C = oneshot.ext()
    m, opt, eng, sim = _setup(world, seed=5)
    p = _peer_proc()
    opened = []
    try:
        xs, ys = _batches(eng, world, 2, 1, 7000 + world)
        start = [t.clone() for t in eng._state()]
        res = sim.step(xs, ys)  # single-process: the payloads and the replica state to reproduce
        pay = sim.last_payload
        for t, s in zip(eng._state(), start):
            t.copy_(s)
        hello = _rd(p)
        f = str(tmp_path / "payload.pt")
        torch.save({"peers": {r: {n: pay[r][n].cpu() for n in REGIONS} for r in range(1, world)},
                    "expect": {n: pay[0][n].cpu() for n in REGIONS}}, f)
        _wr(p, {"hb": bytes(sim.own_h).hex(), "hf": bytes(sim.own_flags_h).hex(), "rank": 0, "payload": f})
        assert _rd(p).get("ready") == 1
        pb, pf = C.open(bytes.fromhex(hello["hb"])), C.open(bytes.fromhex(hello["hf"]))
        opened += [pb, pf]
        sim.peer_buf, sim.peer_flags = pb, pf
        sim._point(0)
        ep = int(eng.xstep.item()) + 1
        eng.timeout_ms = 20000
        t0 = time.perf_counter()
        eng._launch(xs[0], ys[0], 2, 1)  # spins on its flag page until the other process raises it
        _wr(p, {"go": ep, "delay_ms": 50})
        assert _rd(p).get("pushed") == 1
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        eng.check()
        assert torch.equal(eng.arena.master, res[0]["master"]) and torch.equal(eng.s1, res[0]["s1"])
        _wr(p, {"check": 1})
        chk = _rd(p)
        assert chk["match"], chk
        assert el < 10.0
        assert p.wait(timeout=60) == 0
    finally:
        if p.poll() is None:
            p.kill()
            p.wait()
        torch.cuda.synchronize()
        for x in opened:
            C.close(x)
        sim.close()


def test_not_coresident_fails_fast():
    """A concurrent kernel holding half the CUs: the persistent launch must not spin out its hand-off
    timeout.  Either the runtime serialises the cooperative launch behind the other kernel (the step
    then runs correctly), or step 0's local hand-off gives up within HOPSX_PERSIST_START_MS and the
    engine raises the co-residency error — never a 2 s hand-off timeout."""
    from hops_examples_amd.ops import functional as HF
    from hops_examples_amd.parallel import oneshot

    C = oneshot.ext()
    dev = torch.device("cuda", 0)
    torch.manual_seed(6)
    HF.seed_device_rng(5, dev)
    mm = MirroredMnistCNN().to(dev)
    ParamArena.from_module(mm, dev)
    o = optim.Adadelta(mm, lr=1.0)
    eng = persist.PersistentMnistStep(mm, o, steps_per_launch=2, timeout_s=2)
    xs = torch.randint(0, 256, (2, B, 28, 28, 1), dtype=torch.uint8, device=dev)
    ys = torch.randint(0, 10, (2, B), dtype=torch.int64, device=dev)
    eng.run_resident(xs, ys, 2)  # warm (code object loaded)
    torch.cuda.synchronize()
    side = torch.cuda.Stream(dev)
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    C.hog(1.0, cus // 2, 96 * 1024, 0, side.cuda_stream)  # one 96 KiB workgroup per CU on half the CUs
    time.sleep(0.05)
    t0 = time.perf_counter()
    outcome = "ok"
    try:
        eng.run_resident(xs, ys, 2)
        torch.cuda.current_stream().synchronize()
        el = time.perf_counter() - t0
        eng.check()
    except persist.PersistentError as e:
        el = time.perf_counter() - t0
        outcome = str(e)
    torch.cuda.synchronize()
    print(f"[coresident] outcome={outcome!r} elapsed={el:.3f}s")
    if outcome != "ok":
        assert "co-resident" in outcome or "cooperative" in outcome, outcome
        assert el < 0.9, el  # well before the hog ends (1 s) and the 2 s hand-off timeout
        eng.err.zero_()
    # the engine is usable afterwards
    eng.run_resident(xs, ys, 2)
    torch.cuda.synchronize()
    eng.check()
