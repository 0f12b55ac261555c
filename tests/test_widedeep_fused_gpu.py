"""The fp32 v1 fused one-launch taxi training step (widedeep_step.hip) against the fp32 CPU TrainStep of
the same model/optimizers (FTRL wide + Adagrad deep, sigmoid cross-entropy).  The default taxi shape
runs the bf16 v2 kernel (tests/test_taxi_v2_gpu.py); this module pins HOPSX_TAXI_KERNEL=v1."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _v1(monkeypatch):
    monkeypatch.setenv("HOPSX_TAXI_KERNEL", "v1")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from hops_examples_amd.models import widedeep as WD  # noqa: E402
from hops_examples_amd.runtime.arena import ParamArena  # noqa: E402
from hops_examples_amd.runtime.step import TrainStep  # noqa: E402

dev = torch.device("cuda", 0)


def _cpu_reference(model_state, dense, cat, label, steps):
    m = WD.TaxiWideDeep()
    m.load_state_dict(model_state)
    ParamArena.from_module(m, "cpu")
    st = TrainStep(m, WD.make_optimizer(m), "bce_logits", graph=False, forward_fn=lambda mm, x: mm(*x))
    losses = []
    for i in range(steps):
        j = i % dense.shape[0]
        r = st((dense[j], cat[j]), label[j])
        losses.append(float(r["loss"].reshape(-1)[0]))
    return losses, m._hx_arena.master.clone()


@pytest.mark.parametrize("B,graph", [(40, True), (40, False), (48, True), (13, True)])
def test_fused_widedeep_step_matches_fp32_reference(B, graph):
    torch.manual_seed(0)
    nb, steps = 4, 10
    dense, cat, label = WD.synth_taxi(nb * B, seed=3)
    dense, cat, label = dense.view(nb, B, -1), cat.view(nb, B, -1), label.view(nb, B, 1)
    m = WD.TaxiWideDeep()
    state = {k: v.clone() for k, v in m.state_dict().items()}
    ref_losses, ref_master = _cpu_reference(state, dense, cat, label, steps)

    g = WD.TaxiWideDeep()
    g.load_state_dict(state)
    g = g.to(dev)
    ParamArena.from_module(g, dev)
    opt = WD.make_optimizer(g)
    fs = WD.FusedWideDeepStep(g, opt)
    assert fs.ok(B)
    xs = (dense.to(dev), cat.to(dev))
    ys = label.to(dev)
    losses = []
    for _ in range(steps):
        r = fs.step_resident(xs, ys, graph=graph)
        losses.append(float(r["loss"].reshape(-1)[0]))
    torch.cuda.synchronize()
    assert int(fs.cursor.item()) == steps % nb
    torch.testing.assert_close(torch.tensor(losses), torch.tensor(ref_losses), rtol=1e-4, atol=1e-5)
    a = g._hx_arena
    torch.testing.assert_close(a.master.cpu(), ref_master, rtol=1e-3, atol=1e-5)
    assert float(a.grad.abs().max()) == 0.0  # gradients never left the kernel / were claimed back to 0
    assert float(opt.opts[0].step_count.item()) == steps and float(opt.opts[1].step_count.item()) == steps
    # the bf16 shadow the layer kernels read follows the master weights
    torch.testing.assert_close(a.shadow.float(), a.master.to(torch.bfloat16).float())


def test_fused_widedeep_step_dp_gradients_match_layerwise():
    """apply_opt = 0 (the data-parallel form): the kernel leaves the summed gradients in the arena."""
    torch.manual_seed(0)
    B = 40
    dense, cat, label = WD.synth_taxi(B, seed=4)
    m = WD.TaxiWideDeep().to(dev)
    ParamArena.from_module(m, dev)
    fs = WD.FusedWideDeepStep(m, WD.make_optimizer(m))
    fs.dp = object()  # any non-None: gradients only (no optimizer in the kernel)
    fs._finish = lambda: None
    fs((dense.to(dev), cat.to(dev)), label.to(dev))
    torch.cuda.synchronize()
    fused = m._hx_arena.grad.clone()
    m._hx_arena.grad.zero_()
    # fp32 autograd of the same forward (CPU reference ops)
    mc = WD.TaxiWideDeep()
    mc.load_state_dict({k: v.cpu() for k, v in m.state_dict().items()})
    out = mc(dense, cat)
    loss = torch.nn.functional.binary_cross_entropy_with_logits(out, label)
    loss.backward()
    ref = torch.cat([p.grad.reshape(-1) for p in [mc.wide.weight] + [q for q in mc.deep.parameters()]])
    got = torch.cat([fused[p._hx_off:p._hx_off + p.numel()].cpu()
                     for p in [m.wide.weight] + [q for q in m.deep.parameters()]])
    torch.testing.assert_close(got, ref, rtol=1e-3, atol=1e-6)


def test_fused_widedeep_step_declines_batches_beyond_lds():
    """B > 48 pads to 64 rows, whose activations + gradients no longer fit one workgroup's 160 KB LDS:
    the fused step declines and bench_taxi / the trainer run the generic TrainStep path instead."""
    g = WD.TaxiWideDeep().to(dev)
    ParamArena.from_module(g, dev)
    fs = WD.FusedWideDeepStep(g, WD.make_optimizer(g))
    assert fs.ok(48) and not fs.ok(64)


def test_fused_widedeep_steps_per_execution_matches_single_launches():
    """run_resident replays U fused-step launches per graph: cursor, loss and weights equal those of
    U one-launch replays."""
    B, nb, n = 40, 5, 1 + 3 * 8 + 2
    dense, cat, label = WD.synth_taxi(nb * B, seed=9)
    xs = (dense.view(nb, B, -1).to(dev), cat.view(nb, B, -1).to(dev))
    ys = label.view(nb, B, 1).to(dev)
    state = {k: v.clone() for k, v in WD.TaxiWideDeep().state_dict().items()}
    runs = []
    for multi in (True, False):
        g = WD.TaxiWideDeep()
        g.load_state_dict(state)
        g = g.to(dev)
        ParamArena.from_module(g, dev)
        fs = WD.FusedWideDeepStep(g, WD.make_optimizer(g))
        fs.steps_per_execution = 8
        if multi:
            r = fs.run_resident(xs, ys, n)
            assert fs._graphU is not None
        else:
            for _ in range(n):
                r = fs.step_resident(xs, ys)
        torch.cuda.synchronize()
        assert int(fs.cursor.item()) == n % nb
        runs.append((float(r["loss"].reshape(-1)[0]), g._hx_arena.master.clone()))
    assert runs[0][0] == pytest.approx(runs[1][0], rel=1e-5)
    torch.testing.assert_close(runs[0][1], runs[1][1], rtol=1e-5, atol=1e-6)
