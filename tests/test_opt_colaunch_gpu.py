"""Optimizer co-launch (csrc/ops/optim_slice.h): on one GPU the flagship's last backward launch
(the input-side conv pair) also updates the arena slice whose gradients are final; the optimizer
launch then updates only the prefix.

* kernel level: the slice update of the co-launched conv pair equals the optimizer kernel's on the
  same gradients / states (Adadelta, Adam, SGD momentum; up to FMA-contraction rounding: one rule
  compiled into two kernels), and the conv gradients equal those of the plain pair launch (up to
  fp32 atomic order);
* model level: TrainStep with and without the co-launch trains MirroredMnistCNN to the same weights
  (SGD: a linear update, so atomic-order noise in the gradients stays at noise level — Adadelta's
  normalised step would turn the sign of a ~0 gradient into a full step either way)."""
import math
import os

import pytest
import torch

pytestmark = pytest.mark.gpu
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from hops_examples_amd import optim  # noqa: E402
from hops_examples_amd.models.mnist import MirroredMnistCNN  # noqa: E402
from hops_examples_amd.ops import functional as HF  # noqa: E402
from hops_examples_amd.ops import kernels as K  # noqa: E402
from hops_examples_amd.ops._C import OPTIM  # noqa: E402
from hops_examples_amd.runtime.arena import ParamArena  # noqa: E402
from hops_examples_amd.runtime.step import TrainStep  # noqa: E402

dev = torch.device("cuda", 0)
bf = torch.bfloat16

HP = {"adadelta": [1.0, 1.0, 0.0, 0.95, 1e-7], "adam": [1e-3, 0.5, 0.01, 0.9, 0.999, 1e-8],
      "sgd": [0.05, 1.0, 0.0, 0.5, 0.0, 0.0]}
NS = {"adadelta": 2, "adam": 2, "sgd": 1}


@pytest.mark.parametrize("kind", ["adadelta", "adam", "sgd"])
@pytest.mark.parametrize("first", ["0", "1"])
def test_pair_slice_update_matches_optimizer(kind, first, monkeypatch):
    monkeypatch.setenv("HOPSX_OPT_SLICE_FIRST", first)
    torch.manual_seed(0)
    B = 32
    x0 = torch.randint(0, 256, (B, 28, 28, 1), device=dev, dtype=torch.uint8)
    w1 = (torch.randn(32, 2, 2, 1, device=dev) * 0.3).to(bf)
    b1 = torch.randn(32, device=dev) * 0.1
    g1 = K.conv_geom(x0.shape, w1.shape, (1, 1), (0, 0), (1, 1))
    aff = (1.0 / 255.0, -0.5)
    h1 = K.conv2d_fwd(x0, w1, g1, bias=b1, act="relu", in_affine=aff)
    w2 = (torch.randn(64, 2, 2, 32, device=dev) * 0.1).to(bf)
    g2 = K.conv_geom(h1.shape, w2.shape, (1, 1), (0, 0), (1, 1))
    dy = (torch.randn(B, 26, 26, 64, device=dev) * 0.1).to(bf)

    def grads():
        return [torch.zeros(64, 128, device=dev), torch.zeros(64, device=dev), torch.zeros(32, 4, device=dev),
                torch.zeros(32, device=dev)]

    # an arena slice of 1.38 M parameters (the flagship's fc1 + fc2) with random state
    n = 1_385_216
    p = torch.randn(n, device=dev) * 0.05
    g = torch.randn(n, device=dev) * 1e-3
    st = [torch.rand(n, device=dev) * 1e-4 for _ in range(NS[kind])] + [None] * (3 - NS[kind])
    step = torch.tensor([3.0], device=dev)
    ref = [t.clone() if t is not None else None for t in (p, g, *st)]
    sh_ref = torch.empty(n, device=dev, dtype=bf)
    K.optim_step(OPTIM[kind], ref[0], ref[1], ref[2], ref[3], ref[4], sh_ref, HP[kind], step.clone(),
                 zero_grad=True, arrive=torch.zeros(288, device=dev, dtype=torch.int32))
    sh = torch.empty(n, device=dev, dtype=bf)
    gs_a = grads()
    prev = (x0, g1, gs_a[2], gs_a[3], h1, K.act_id("relu"), aff)
    r = K.conv2d_bwd_pair(dy, w2, g2, h1, gs_a[0], dbias=gs_a[1], prev=prev,
                          opt_slice=(OPTIM[kind], p, g, st[0], st[1], st[2], sh, HP[kind], None, step))
    assert r is None  # launched (the input layer's gradient rides on the dgrad: no dX)
    gs_b = grads()
    prev = (x0, g1, gs_b[2], gs_b[3], h1, K.act_id("relu"), aff)
    K.conv2d_bwd_pair(dy, w2, g2, h1, gs_b[0], dbias=gs_b[1], prev=prev)
    torch.cuda.synchronize()
    # the same update rule compiled into two kernels: equal up to FMA-contraction rounding
    def rel(a, b):  # error relative to the tensor's scale (elements near 0 carry no relative meaning)
        return ((a - b).abs().max() / b.abs().max()).item()

    assert torch.equal(g, torch.zeros_like(g))
    assert rel(p, ref[0]) <= 1e-6, rel(p, ref[0])
    for a, b in zip(st, ref[2:]):
        if a is not None:
            assert rel(a, b) <= 1e-5, rel(a, b)
    assert ((sh.float() - sh_ref.float()).abs() <= 1e-2 * sh_ref.float().abs() + 1e-30).all()
    for a, b in zip(gs_a, gs_b):
        assert (a - b).abs().max().item() <= 1e-4 * b.abs().max().item() + 1e-6


def _train(colaunch: str, graph: bool, steps: int = 6):
    old = os.environ.get("HOPSX_OPT_COLAUNCH")
    os.environ["HOPSX_OPT_COLAUNCH"] = colaunch
    try:
        torch.manual_seed(11)
        m = MirroredMnistCNN().to(dev)
        m.pool.salt = 777
        ParamArena.from_module(m, dev)
        winit = m._hx_arena.master.clone()
        opt = optim.SGD(m, lr=0.05, momentum=0.5)
        step = TrainStep(m, opt, "sparse_ce", graph=graph, warmup=2)
        gen = torch.Generator().manual_seed(5)
        xs = torch.randint(0, 256, (steps, 32, 28, 28, 1), dtype=torch.uint8, generator=gen).to(dev)
        ys = torch.randint(0, 10, (steps, 32), generator=gen).to(dev)
        n0 = HF.COLAUNCH["launched"]
        HF.seed_device_rng(123, dev)
        for i in range(steps):
            r = step(xs[i], ys[i])
        torch.cuda.synchronize()
        return (m._hx_arena.master - winit, float(r["loss"].reshape(-1)[0]), HF.COLAUNCH["launched"] - n0,
                float(opt.step_count.item()))
    finally:
        if old is None:
            os.environ.pop("HOPSX_OPT_COLAUNCH", None)
        else:
            os.environ["HOPSX_OPT_COLAUNCH"] = old


@pytest.mark.parametrize("graph,steps", [(False, 1), (True, 6)])
def test_colaunched_training_matches_unfused(graph, steps):
    """One eager step from the same state: a misplaced or doubled update would show as ~lr * grad,
    the only other difference is fp32 atomic order (tight bound on the weight change).  Six graph-
    replayed steps: bf16 shadow roundings amplify that noise chaotically (two unfused runs drift a few
    % apart), so the weight changes must agree in direction and within 12 % (and the fused path ran)."""
    d1, l1, n1, t1 = _train("1", graph, steps)
    d0, l0, n0, t0 = _train("0", graph, steps)
    assert n0 == 0 and n1 >= 1, (n0, n1)  # the fused path ran (eager steps / captures count launches)
    assert t1 == t0 == float(steps)
    rel = float((d1 - d0).norm()) / float(d0.norm())
    cos = float(torch.nn.functional.cosine_similarity(d1, d0, dim=0))
    if steps == 1:
        assert rel <= 1e-4, rel
    else:
        assert rel <= 0.12 and cos >= 0.99, (rel, cos)
    assert math.isfinite(l1) and abs(l1 - l0) <= 2e-3 * abs(l0) + 1e-4
