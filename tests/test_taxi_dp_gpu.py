"""The data-parallel instantiation of the v2 taxi step (csrc/ops/taxi_step.hip DP, models/widedeep.py
TaxiExchange): each rank trains on its own batch, the dW accumulators and wide-row gradients are pushed
to every rank inside the launch and summed in rank order before the in-register Adagrad / FTRL updates.

* loopback (one process plays W ranks, every "peer" holds this rank's batch): at W = 2 every sum is
  x/2 + x/2 — exact — so the run must be bit-identical to the one-GPU kernel; at W = 8 it tracks it;
* W real PROCESSES sharing the GPU (the step is one workgroup, so they co-reside), each on different
  data, exchanging through IPC-mapped uncached buffers: the replicas must end bit-identical and match
  the bf16-emulating fp64 reference of the GLOBAL batch (MirroredStrategy semantics).

Reference: README.md:99-112 (the TFX Chicago-taxi trainer); BASELINE.json "steps/sec Chicago-taxi DNN at
1/2/4/8".
"""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from hops_examples_amd.models import widedeep as WD  # noqa: E402
from hops_examples_amd.runtime.arena import ParamArena  # noqa: E402

dev = torch.device("cuda", 0)
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(loopback, steps=12, spe=4, B=40, nb=4, seed=1):
    torch.manual_seed(seed)
    dense, cat, label = WD.synth_taxi(nb * B, seed=seed + 3)
    dense, cat, label = dense.view(nb, B, -1), cat.view(nb, B, -1), label.view(nb, B, 1)
    m = WD.TaxiWideDeep()
    with torch.no_grad():
        m.wide.weight.normal_(0, 0.05)
    m = m.to(dev)
    ParamArena.from_module(m, dev)
    opt = WD.make_optimizer(m)
    xdp = WD.TaxiExchange(dev, loopback=loopback, timeout_s=5) if loopback > 1 else None
    fs = WD.FusedWideDeepStep(m, opt, xdp=xdp)
    assert fs.kernel == ("v2-dp" if xdp else "v2")
    fs.steps_per_execution = spe
    fs.run_resident((dense.to(dev), cat.to(dev)), label.to(dev), steps)
    torch.cuda.synchronize()
    fs.check()
    a = m.wide.weight._hx_arena
    out = [a.master.clone(), a.state("adagrad_s0").clone(), a.state("ftrl_s0").clone(), a.state("ftrl_s1").clone(),
           float(fs.loss.item()), int(fs.cursor.item())]
    if xdp is not None:
        assert int(xdp.xstep.item()) == steps  # the exchange epochs carried across the launches
        xdp.close()
    return out


def test_loopback_two_ranks_bit_identical_to_one():
    one = _run(0)
    two = _run(2)
    assert one[4] == two[4] and one[5] == two[5] == 12 % 4
    for x, y in zip(one[:4], two[:4]):
        assert torch.equal(x, y)


def test_loopback_eight_ranks_tracks_one():
    one = _run(0, steps=8)
    eight = _run(8, steps=8)
    init = _run(0, steps=0)  # the initial state
    d1 = (one[0] - init[0]).double()
    d8 = (eight[0] - init[0]).double()
    cos = float(torch.nn.functional.cosine_similarity(d1, d8, dim=0))
    assert cos > 0.9999, cos
    assert abs(one[4] - eight[4]) < 1e-4 * abs(one[4]) + 1e-6


def _launch(world, out, steps, spe, bench=0):
    from hops_examples_amd.parallel import launch

    argv = [os.path.join(ROOT, "tools", "taxi_dp_worker.py"), "--out", str(out), "--steps", str(steps),
            "--spe", str(spe), "--bench", str(bench)]
    env = {"HOPSX_TAXI_DP_TIMEOUT_S": "20", "PYTHONPATH": ROOT + os.pathsep + os.environ.get("PYTHONPATH", "")}
    return launch.launch(world, argv, rehearse=True, timeout_s=240, extra_env=env)


def _update_err(got, ref, init):
    return float((got - ref).norm() / max(float((ref - init).norm()), 1e-12))


@pytest.mark.parametrize("world", [2, 4])
def test_processes_match_fp64_global_batch(world, tmp_path):
    steps = 12
    assert _launch(world, tmp_path, steps, 5) == 0
    rs = [torch.load(tmp_path / f"rank{r}.pt", weights_only=True) for r in range(world)]
    # the replicas: bit-identical after 12 steps on different data, every bookkeeping word advanced
    for r in rs[1:]:
        for k in ("master", "ada", "z", "n"):
            assert torch.equal(r["final"][k], rs[0]["final"][k]), k
    assert all(r["final"]["cursor"] == steps % 4 and r["final"]["steps_ada"] == steps for r in rs)
    assert len({r["final"]["loss"] for r in rs}) == world, "every replica trains on its own batch"
    # fp64 reference of the global batch (the replicas' batches side by side)
    W, b, w4, b4, wide, ada, z, n, hpa, hpf = rs[0]["init"]
    init = [w.clone() for w in W] + [x.clone() for x in b] + [w4.clone(), wide.clone()]
    dense = torch.cat([r["dense"] for r in rs], dim=1).double()
    cat = torch.cat([r["cat"] for r in rs], dim=1)
    label = torch.cat([r["label"] for r in rs], dim=1).double()
    ref_losses = WD.reference_steps(W, b, w4, b4, wide, ada, z, n, hpa, hpf, dense, cat, label, steps)
    gl = sum(r["final"]["loss"] for r in rs) / world
    assert abs(gl - ref_losses[-1]) < 2e-4 * abs(ref_losses[-1]) + 2e-5, (gl, ref_losses[-1])
    # the final parameters, read back through a model laid out like the workers'
    torch.manual_seed(1)
    mm = WD.TaxiWideDeep().to(dev)
    ParamArena.from_module(mm, dev)
    fs = WD.FusedWideDeepStep(mm, WD.make_optimizer(mm))
    mm.wide.weight._hx_arena.master.copy_(rs[0]["final"]["master"].to(dev))
    got = WD.reference_state(mm, fs)
    names = [f"W{l}" for l in range(4)] + [f"b{l}" for l in range(4)] + ["w4", "wide"]
    gots = list(got[0]) + list(got[1]) + [got[2], got[4]]
    refs = list(W) + list(b) + [w4, wide]
    for nm, g_, r_, i_ in zip(names, gots, refs, init):
        e = _update_err(g_, r_, i_)
        print(f"[W={world}] {nm}: relative update error {e:.2e}, max |err| {float((g_ - r_).abs().max()):.2e}")
        assert e < 5e-2 and float((g_ - r_).abs().max()) < 3e-3, (nm, e)
    torch.testing.assert_close(rs[0]["final"]["n"][int(mm.wide.weight._hx_off):][:wide.numel()].double(), n,
                               rtol=1e-4, atol=1e-7)
    assert torch.equal(rs[0]["final"]["shadow"], rs[0]["final"]["master"].to(torch.bfloat16).float())


def test_two_processes_bench(tmp_path):
    """Two ranks sharing the GPU for real (one workgroup each): steps/s per rank of the exchanging step."""
    import json

    assert _launch(2, tmp_path, 4, 4, bench=2000) == 0
    r = json.load(open(tmp_path / "bench.json"))
    print(f"[taxi dp bench] {r}")
    assert r["replicas_identical"] and r["kernel"] == "v2-dp"
    assert r["steps_per_sec_per_rank"] > 20_000, r
