"""The persistent flagship step (csrc/ops/mnist_persist.hip, runtime/persist.py) against an fp64
PyTorch reference of the same training steps (same data order, dropout masks, loss, Adadelta), and
its determinism / launch-boundary invariance.

Reference workload: notebooks/ml/Distributed_Training/mirrored_strategy/
mirroredstrategy_mnist_example.ipynb:189-222.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from hops_examples_amd import optim  # noqa: E402
from hops_examples_amd.models.mnist import MirroredMnistCNN  # noqa: E402
from hops_examples_amd.runtime.arena import ParamArena  # noqa: E402
from hops_examples_amd.runtime import persist  # noqa: E402

B = 32


def _setup(seed=0, nb=5, spl=32, stamps=False):
    from hops_examples_amd.ops import functional as HF

    torch.manual_seed(seed)
    dev = torch.device("cuda", 0)
    HF.seed_device_rng(11, dev)  # the device RNG counter advances with every step of every engine
    m = MirroredMnistCNN().to(dev)
    m.pool.salt = 7919  # each MaxPool2d instance draws a new dropout salt from a global counter
    ParamArena.from_module(m, dev)
    opt = optim.Adadelta(m, lr=1.0)
    g = torch.Generator().manual_seed(seed + 7)
    xs = torch.randint(0, 256, (nb, B, 28, 28, 1), dtype=torch.uint8, generator=g).to(dev)
    ys = torch.randint(0, 10, (nb, B), dtype=torch.int64, generator=g).to(dev)
    eng = persist.PersistentMnistStep(m, opt, steps_per_launch=spl, debug_stamps=stamps)
    return m, opt, eng, xs, ys


def _snapshot(m, eng):
    named = dict(m.named_parameters())
    P = {k: named[k].detach().clone() for k in eng.PARAMS}
    a = eng.arena
    S1 = {k: eng.s1[named[k]._hx_off:named[k]._hx_off + named[k].numel()].view_as(named[k]).clone() for k in eng.PARAMS}
    S2 = {k: eng.s2[named[k]._hx_off:named[k]._hx_off + named[k].numel()].view_as(named[k]).clone() for k in eng.PARAMS}
    return P, S1, S2, a.master.clone()


def _run_and_reference(n, seed=0, emulate_bf16=False, margins=None):
    m, opt, eng, xs, ys = _setup(seed)
    P0, S10, S20, _ = _snapshot(m, eng)
    rng0 = eng.rng.clone().cpu()
    eng.run_resident(xs, ys, n)
    torch.cuda.synchronize()
    eng.check()
    losses = eng.losses(n)[:, 0].cpu().double()
    P1, S11, S21, _ = _snapshot(m, eng)
    Pr, S1r, S2r, lr_ = persist.reference_steps(P0, S10, S20, xs, ys, 0, n, int(rng0[0]) & ((1 << 64) - 1),
                                                int(rng0[1]), int(m.pool.salt), float(m.pool.dropout), 1.0, 0.95,
                                                1e-7, emulate_bf16=emulate_bf16, margins=margins)
    return m, opt, eng, P0, P1, Pr, S11, S1r, losses, torch.tensor(lr_, dtype=torch.float64)


def _delta_stats(P0, P1, Pr, k):
    dk = (P1[k] - P0[k]).double().flatten()
    dr = (Pr[k] - P0[k].double()).flatten()
    cos = torch.nn.functional.cosine_similarity(dk, dr, dim=0).item()
    err = (dk - dr).abs()
    return cos, err, dr


def test_persistent_one_step_matches_bf16_emulation():
    """One step against the fp64 reference that rounds exactly the operands the kernel stores as bf16:
    what is left is fp32-vs-fp64 accumulation, so every parameter update must agree to ~1e-6 of the
    Adadelta step (1.41e-3 = sqrt(eps / (1 - rho)) for |g| >> sqrt(eps)).

    The comparison is only this tight away from ReLU ties: with seed 0 one sample's fc1 unit 50 sits
    so close to 0 that fp32-vs-fp64 accumulation flips it, which moves fc1 row 50's gradient and,
    through dh, every conv gradient (tools/persist_diag.py; seeds 1-3 agree to cos 1.000000 on every
    parameter).  The test pins seed 1 (smallest |fc1 pre-activation| 1.8e-5) and checks that it stays
    clear of fp32 accumulation error (~1e-6 over K = 10816), so a change of setup that lands on a tie
    says so instead of failing on the symptom."""
    mg = []
    m, opt, eng, P0, P1, Pr, S1k, S1r, lk, lr_ = _run_and_reference(1, seed=1, emulate_bf16=True, margins=mg)
    assert mg[0]["fc1"] > 5e-6, f"setup sits on an fc1 ReLU tie: {mg[0]}"
    assert abs(float(lk[0]) - float(lr_[0])) < 1e-5 * float(lr_[0]), (lk, lr_)
    for k in eng.PARAMS:
        cos, err, dr = _delta_stats(P0, P1, Pr, k)
        # the conv gradients are sums of ~50k products with cancellation: fp32 vs fp64 order moves an
        # element's update by up to ~5 % of a step (measured max 6.5e-5); more than 7 % of a step (1e-4)
        # is allowed for at most 1 element in 1000 (a gradient within noise of 0), bounded by 2 steps
        nbad = int((err > 1e-4).sum())
        # (the cosine of a 32-element bias update is one element's 6 % error: the element bounds
        # carry those; measured conv1.bias cos 0.99993 with every element within 9.1e-5)
        cmin = 0.99999 if err.numel() >= 1024 else 0.9999
        assert cos > cmin and nbad <= max(0, err.numel() // 1000) and float(err.max()) <= 2 * 1.42e-3, \
            f"{k}: cos {cos:.7f} off {nbad}/{err.numel()} max {float(err.max()):.3e}"
        # E[g^2] = 0.05 g^2: the conv gradients are sums of ~50k terms with cancellation, where fp32
        # vs fp64 order moves the smallest entries by up to ~1 % (measured rel-L2 <= 3.2e-3)
        sk, sr = S1k[k].double().flatten(), S1r[k].flatten()
        srel = float((sk - sr).norm() / sr.norm())
        assert srel < 1e-2, f"{k}: E[g^2] rel {srel:.5f}"
    # bookkeeping advanced on the device; the bf16 shadow the other kernels read is the rounded master
    assert int(eng.cursor.item()) == 1 and float(opt.step_count.item()) == 1
    a = eng.arena
    assert torch.equal(a.shadow, a.master.to(torch.bfloat16))


def test_persistent_trajectory_tracks_references():
    """Six steps: the loss trajectory stays on the bf16-emulating reference (rounding-boundary flips
    decorrelate the updates of near-zero gradients slowly) and within bf16 noise of pure fp64."""
    n = 6
    *_, lk, lemu = _run_and_reference(n, emulate_bf16=True)
    assert torch.allclose(lk, lemu.cpu(), rtol=1e-3, atol=0), (lk, lemu)
    m, opt, eng, P0, P1, Pr, S1k, S1r, lk2, lref = _run_and_reference(n)
    assert torch.equal(lk, lk2)  # deterministic
    assert torch.allclose(lk2, lref.cpu(), rtol=5e-3, atol=0), (lk2, lref)
    assert int(eng.cursor.item()) == n % 5 and float(opt.step_count.item()) == n


def test_persistent_deterministic_and_launch_invariant():
    """Two runs from the same state are bit-identical, and cutting 24 steps into 3 launches of 8
    changes nothing (the state written back between launches is exact)."""
    res = []
    for spl in (24, 24, 8):
        m, opt, eng, xs, ys = _setup(3, spl=spl)
        eng.run_resident(xs, ys, 24)
        torch.cuda.synchronize()
        eng.check()
        res.append((eng.arena.master.clone(), eng.s1.clone(), eng.s2.clone(), float(eng.out[2 * 7].item())))
    (m0, a0, b0, _), (m1, a1, b1, _), (m2, a2, b2, _) = res
    assert torch.equal(m0, m1) and torch.equal(a0, a1) and torch.equal(b0, b1)
    assert torch.equal(m0, m2) and torch.equal(a0, a2) and torch.equal(b0, b2)


def test_persistent_trains():
    m, opt, eng, xs, ys = _setup(5, nb=2)
    eng.run_resident(xs, ys, 60)  # two batches, memorised
    torch.cuda.synchronize()
    eng.check()
    l = eng.losses(28)[:, 0].cpu()  # last launch: steps 32..59
    assert float(l[-1]) < 0.5, l


def test_persistent_phase_stamps():
    m, opt, eng, xs, ys = _setup(1, spl=16, stamps=True)
    eng.run_resident(xs, ys, 16)
    torch.cuda.synchronize()
    eng.check()
    st = eng.phase_stamps(16).cpu()
    pos = st[:169]
    # per step the position workgroups pass their phases in order and every step takes time
    assert bool((pos[:, :, 11] >= pos[:, :, 0]).all())
    steps = (pos[0, 1:, 0] - pos[0, :-1, 0]).double() * 10e-3  # us (100 MHz)
    assert float(steps.median()) > 0.0
