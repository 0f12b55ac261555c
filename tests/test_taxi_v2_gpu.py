"""The v2 taxi step kernel (csrc/ops/taxi_step.hip: bf16 MFMA, LDS-resident model and wide table,
optimizer state in registers) against an fp64 reference that rounds to bf16 at exactly the kernel's
points (inputs, hidden activations, W images, the backward gradients), so the check is tight; plus
a loose check against the fp32 CPU TrainStep of the same model (the reference's own numerics)."""

import pytest
import torch

pytestmark = pytest.mark.gpu
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from hops_examples_amd.models import widedeep as WD  # noqa: E402
from hops_examples_amd.runtime.arena import ParamArena  # noqa: E402
from hops_examples_amd.runtime.step import TrainStep  # noqa: E402

dev = torch.device("cuda", 0)


reference_steps = WD.reference_steps


def _setup(B, nb, seed):
    torch.manual_seed(seed)
    dense, cat, label = WD.synth_taxi(nb * B, seed=seed + 3)
    dense, cat, label = dense.view(nb, B, -1), cat.view(nb, B, -1), label.view(nb, B, 1)
    m = WD.TaxiWideDeep()
    # a trained-looking wide part (the all-zero init makes the FTRL path trivial)
    with torch.no_grad():
        m.wide.weight.normal_(0, 0.05)
    state = {k: v.clone() for k, v in m.state_dict().items()}
    g = WD.TaxiWideDeep()
    g.load_state_dict(state)
    g = g.to(dev)
    ParamArena.from_module(g, dev)
    opt = WD.make_optimizer(g)
    fs = WD.FusedWideDeepStep(g, opt)
    return dense, cat, label, g, opt, fs


def _close_update(got, ref, init, name):
    """bf16 rounding flips make single elements drift: check the update as a whole (relative error of
    the applied change) plus a loose elementwise bound."""
    d = (got - ref).norm() / max(float((ref - init).norm()), 1e-12)
    print(f"{name}: relative update error {float(d):.2e}")
    assert d < 5e-2, (name, float(d))
    assert float((got - ref).abs().max()) < 3e-3, (name, float((got - ref).abs().max()))


def _ref_state(g, fs):
    return WD.reference_state(g, fs)


@pytest.mark.parametrize("B,graph,spe", [(40, True, 1), (40, False, 1), (48, True, 1), (13, True, 1), (40, True, 8)])
def test_taxi_v2_matches_bf16_reference(B, graph, spe):
    nb, steps = 4, 12
    dense, cat, label, g, opt, fs = _setup(B, nb, seed=1)
    assert fs.v2(B) and fs.kernel == "v2"
    W, bb, w4, b4, wide, ada, z, n, hpa, hpf = _ref_state(g, fs)
    init = [w.clone() for w in W] + [x.clone() for x in bb] + [w4.clone(), wide.clone()]
    ref_losses = reference_steps(W, bb, w4, b4, wide, ada, z, n, hpa, hpf, dense.double(), cat, label.double(), steps)
    xs, ys = (dense.to(dev), cat.to(dev)), label.to(dev)
    fs.steps_per_execution = spe
    losses = []
    if spe > 1:
        fs.run_resident(xs, ys, steps)  # 12 = one 8-step launch + a 4-step remainder launch (or single launches)
    else:
        for _ in range(steps):
            r = fs.step_resident(xs, ys, graph=graph)
            losses.append(float(r["loss"].reshape(-1)[0]))
    torch.cuda.synchronize()
    assert int(fs.cursor.item()) == steps % nb
    if losses:
        torch.testing.assert_close(torch.tensor(losses, dtype=torch.float64), torch.tensor(ref_losses, dtype=torch.float64),
                                   rtol=2e-4, atol=2e-5)
    else:
        assert float(fs.loss.item()) == pytest.approx(ref_losses[-1], rel=2e-4, abs=2e-5)
    a = g._hx_arena
    for l, m in enumerate(fs.lins[:4]):
        _close_update(m.weight.detach().double().cpu(), W[l], init[l], f"W{l}")
        _close_update(m.bias.detach().double().cpu(), bb[l], init[4 + l], f"b{l}")
    _close_update(fs.lins[4].weight.detach().double().cpu().reshape(-1), w4, init[8], "w4")
    wo, rows = int(g.wide.weight._hx_off), g.wide.weight.shape[0]
    _close_update(a.master[wo:wo + rows].double().cpu(), wide, init[9], "wide")
    torch.testing.assert_close(a.state("ftrl_s1")[wo:wo + rows].double().cpu(), n, rtol=1e-4, atol=1e-7)
    assert float(a.grad.abs().max()) == 0.0
    assert float(opt.opts[0].step_count.item()) == steps and float(opt.opts[1].step_count.item()) == steps
    torch.testing.assert_close(a.shadow.float(), a.master.to(torch.bfloat16).float())


def test_taxi_v2_tracks_fp32_training():
    """Against the fp32 CPU TrainStep (the reference's precision): the loss curve agrees to bf16 noise."""
    B, nb, steps = 40, 8, 40
    dense, cat, label, g, opt, fs = _setup(B, nb, seed=2)
    m = WD.TaxiWideDeep()
    m.load_state_dict({k: v.cpu() for k, v in g.state_dict().items()})
    ParamArena.from_module(m, "cpu")
    st = TrainStep(m, WD.make_optimizer(m), "bce_logits", graph=False, forward_fn=lambda mm, x: mm(*x))
    ref, got = [], []
    xs, ys = (dense.to(dev), cat.to(dev)), label.to(dev)
    for i in range(steps):
        j = i % nb
        ref.append(float(st((dense[j], cat[j]), label[j])["loss"].reshape(-1)[0]))
        got.append(float(fs.step_resident(xs, ys)["loss"].reshape(-1)[0]))
    diffs = [abs(a - b) for a, b in zip(ref, got)]
    # bf16 operands vs fp32: the curves agree to ~1e-3 on average, single steps to a few 1e-2
    assert sum(diffs) / len(diffs) < 5e-3 and max(diffs) < 3e-2, (diffs, ref[-5:], got[-5:])
    assert got[-1] < got[0]


def test_taxi_v2_multi_step_launch_matches_single_launches():
    """One 15-step launch (weights and wide table kept on chip between steps) == 15 one-step launches, bit
    for bit: every sum has a fixed order (no atomics), and a launch reloads exactly what the last stored."""
    B, nb, n = 40, 5, 16
    outs = []
    for spe in (n - 1, 1):
        dense, cat, label, g, opt, fs = _setup(B, nb, seed=5)
        fs.steps_per_execution = spe
        xs, ys = (dense.to(dev), cat.to(dev)), label.to(dev)
        if spe > 1:
            fs.step_resident(xs, ys)  # one step (captures the one-step graph), then ONE 15-step launch
            fs.prepare_resident(xs, ys, n - 1)
            fs.run_resident(xs, ys, n - 1)
            # direct launches: prepare_resident built the launch-argument slot; graph replays: the U-step graph
            assert len(fs._v2slots) >= 2 if fs._direct(xs[0]) else fs._graphU is not None
        else:
            for _ in range(n):
                fs.step_resident(xs, ys)
        torch.cuda.synchronize()
        a = g._hx_arena
        outs.append((float(fs.loss.item()), a.master.clone(), a.state("adagrad_s0").clone(),
                     a.state("ftrl_s0").clone(), a.state("ftrl_s1").clone()))
    assert outs[0][0] == outs[1][0]
    for x, y in zip(outs[0][1:], outs[1][1:]):
        assert torch.equal(x, y)


def test_taxi_v2_declines_other_shapes(monkeypatch):
    g = WD.TaxiWideDeep(hidden=[64, 32]).to(dev)
    ParamArena.from_module(g, dev)
    fs = WD.FusedWideDeepStep(g, WD.make_optimizer(g))
    assert not fs.v2(40) and fs.ok(40)  # the v1 kernel takes it
    g = WD.TaxiWideDeep().to(dev)
    ParamArena.from_module(g, dev)
    fs = WD.FusedWideDeepStep(g, WD.make_optimizer(g))
    assert fs.v2(40) and not fs.v2(49)
    monkeypatch.setenv("HOPSX_TAXI_KERNEL", "v1")
    assert not fs.v2(40) and fs.kernel == "v1"
