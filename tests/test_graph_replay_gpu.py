"""Regression: graph replays of fwd+bwd on fixed weights/inputs must reproduce the first replay
(to fp32 atomic-ordering noise).  hipMemsetAsync blit nodes inside captured graphs were observed
to be intermittently unordered w.r.t. the following split-K kernels (exploding logits after a few
replays at batch 32/256); all in-graph clears now run as kernels (hopsx_zero)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from hops_examples_amd.models.mnist import MirroredMnistCNN  # noqa: E402
from hops_examples_amd.ops import functional as HF  # noqa: E402
from hops_examples_amd.ops import kernels as K  # noqa: E402
from hops_examples_amd.runtime.arena import ParamArena  # noqa: E402


@pytest.mark.parametrize("B", [32, 256])
def test_graph_replays_are_reproducible(B):
    dev = torch.device("cuda", 0)
    torch.manual_seed(1234)
    m = MirroredMnistCNN().to(dev)
    ParamArena.from_module(m, dev)
    a = m._hx_arena
    x = torch.randint(0, 256, (B, 28, 28, 1), dtype=torch.uint8, device=dev)
    y = torch.randint(0, 10, (B,), device=dev)
    box = {}

    def fb():
        out = m(x)
        _, _, _, dl = HF.loss_and_grad(out, y, "sparse_ce")
        out.backward(dl)
        box["out"] = out

    for _ in range(3):
        fb()
        a.grad.zero_()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fb()
    a.grad.zero_()
    g.replay()
    torch.cuda.synchronize()
    ref = a.grad.clone()
    scale = ref.abs().max()
    dev_max = torch.zeros(1500, device=dev)
    with torch.no_grad():
        for i in range(1500):
            a.grad.zero_()
            g.replay()
            dev_max[i] = (a.grad - ref).abs().max()
    torch.cuda.synchronize()
    assert float(dev_max.max()) < 1e-3 * float(scale), float(dev_max.max())


def test_resident_prefetch_walks_the_epoch():
    """TrainStep.step_resident: after capture the optimizer kernel copies batch (cursor+1) into the
    static inputs; the losses of a resident run match explicit per-batch copies step for step."""
    from hops_examples_amd import optim
    from hops_examples_amd.runtime.step import TrainStep

    dev = torch.device("cuda", 0)
    nb, B = 5, 16
    xs = torch.randint(0, 256, (nb, B, 28, 28, 1), dtype=torch.uint8, device=dev)
    ys = torch.randint(0, 10, (nb, B), device=dev)
    losses = []
    for resident in (True, False):
        HF.seed_device_rng(5, dev)
        torch.manual_seed(0)
        m = MirroredMnistCNN().to(dev)
        m.pool.salt = 7919
        ParamArena.from_module(m, dev)
        st = TrainStep(m, optim.Adadelta(m, lr=1.0), "sparse_ce")
        ls = []
        for i in range(12):
            r = st.step_resident(xs, ys) if resident else st(xs[i % nb], ys[i % nb])
            ls.append(float(r["loss"].reshape(-1)[0]))
        losses.append(ls)
        if resident:
            assert int(st._cursor.item()) == 12 % nb
    torch.testing.assert_close(torch.tensor(losses[0]), torch.tensor(losses[1]), rtol=1e-3, atol=1e-3)


@pytest.mark.parametrize("model", ["mirrored", "keras", "resnet20"])
def test_deferred_logits_layer_matches_eager_head(monkeypatch, model):
    """TrainStep defers the logits layer's forward into the fused loss kernel (head_ce forward
    mode) once it has probed that the logits only feed the loss: losses and trained weights match
    the undeferred run (eager warm-up + graph replays)."""
    from hops_examples_amd import optim
    from hops_examples_amd.models import mnist
    from hops_examples_amd.runtime.step import TrainStep

    dev = torch.device("cuda", 0)
    from hops_examples_amd.models.resnet import cifar_resnet

    B = 32
    shape = (32, 32, 3) if model == "resnet20" else (28, 28, 1)
    xs = torch.randint(0, 256, (8, B) + shape, dtype=torch.uint8, device=dev)
    ys = torch.randint(0, 10, (8, B), device=dev)
    make = {"mirrored": mnist.MirroredMnistCNN, "keras": mnist.KerasMnistCNN, "resnet20": lambda: cifar_resnet(20)}
    runs = []
    for defer in ("1", "0"):
        monkeypatch.setenv("HOPSX_DEFER_HEAD", defer)
        HF.seed_device_rng(5, dev)
        torch.manual_seed(0)
        m = make[model]().to(dev)
        for mod in m.modules():
            if hasattr(mod, "salt"):
                mod.salt = 7919
        ParamArena.from_module(m, dev)
        st = TrainStep(m, optim.Adadelta(m, lr=1.0), "sparse_ce")
        ls = [float(st(xs[i], ys[i])["loss"].reshape(-1)[0]) for i in range(8)]
        assert bool(st._head_defer) is (defer == "1")
        runs.append((ls, m._hx_arena.master.float().clone()))
    # ResNet-20: 19 BatchNorm'd bf16 layers under Adadelta(1.0) amplify the head's different fp32
    # summation order step over step (0.2% loss drift after 8 steps); the first step is exact
    tol = 1e-2 if model == "resnet20" else 1e-3
    assert abs(runs[0][0][0] - runs[1][0][0]) <= 1e-3 * abs(runs[1][0][0]) + 1e-4
    torch.testing.assert_close(torch.tensor(runs[0][0]), torch.tensor(runs[1][0]), rtol=tol, atol=tol)
    if model == "resnet20":
        return
    # logits rounded from a different fp32 summation order: bf16 ties flip on a few elements
    torch.testing.assert_close(runs[0][1], runs[1][1], rtol=1e-2, atol=5e-3)


def test_steps_per_execution_matches_single_step_replays():
    """TrainStep.run_resident: U = steps_per_execution steps captured in one graph (each step's
    optimizer prefetches the next batch) trains like U one-step replays: same device cursor, the
    next batch staged in the static inputs, same loss, and a weight trajectory that differs from the
    one-step replays no more than two one-step runs differ from each other (split-K fp32 atomics
    + bf16 shadow rounding make repeated runs diverge by a few %; tools/spe_drift.py measures it)."""
    from hops_examples_amd import optim
    from hops_examples_amd.runtime.step import TrainStep

    dev = torch.device("cuda", 0)
    B, nb, n = 32, 6, 4 + 8 + 3  # eager warm-up + capture, one U-graph replay, a ragged tail
    xs = torch.randint(0, 256, (nb, B, 28, 28, 1), dtype=torch.uint8, device=dev)
    ys = torch.randint(0, 10, (nb, B), device=dev)
    runs = []
    for multi in (True, False, False):
        HF.seed_device_rng(11, dev)
        torch.manual_seed(0)
        m = MirroredMnistCNN().to(dev)
        m.pool.salt = 7919
        ParamArena.from_module(m, dev)
        w0 = m._hx_arena.master.clone()
        st = TrainStep(m, optim.SGD(m, lr=0.05), "sparse_ce", steps_per_execution=8)
        if multi:
            r = st.run_resident(xs, ys, n)
            assert st._gU is not None
        else:
            for _ in range(n):
                r = st.step_resident(xs, ys)
        torch.cuda.synchronize()
        assert int(st._cursor.item()) == n % nb
        assert torch.equal(st._sx, xs[n % nb]) and torch.equal(st._sy, ys[n % nb])
        runs.append((float(r["loss"].reshape(-1)[0]), m._hx_arena.master - w0))
    assert abs(runs[0][0] - runs[1][0]) <= 2e-3 * abs(runs[1][0])

    def rel(a, b):
        return float((a - b).norm()) / float(b.norm())

    noise = rel(runs[2][1], runs[1][1])
    # two one-step runs are sometimes bit-close (noise ~1e-6) and sometimes a few % apart, while the
    # U-graph run has been measured up to 7.7 % from a one-step run in a full-suite session: bound the
    # distance by the larger of the measured noise model and a fixed 12 %, and require the same
    # update direction (a skipped / doubled / wrong-batch step breaks both by far)
    d = rel(runs[0][1], runs[1][1])
    assert d <= max(3 * noise + 0.05, 0.12), (d, noise)
    cos = float(torch.nn.functional.cosine_similarity(runs[0][1], runs[1][1], dim=0))
    assert cos >= 0.99, cos


def _e1_modules(fold: bool):
    """The E1 MNIST CNN (mnist.ipynb:154-164) as keras.Sequential wires it: conv2 -> 4x4 pool (+dropout)
    in one launch, and with ``fold`` the Dense -> Dropout -> logits chain's dropout handed to the logits
    layer (Linear._drop_in), which the deferred head's loss kernel applies."""
    from hops_examples_amd import nn as hnn

    c1 = hnn.Conv2d(1, 32, 4, activation="relu")
    c1.in_affine = (1.0 / 255.0, 0.0)
    c2 = hnn.Conv2d(32, 64, 4, activation="relu")
    pool = hnn.MaxPool2d(4, dropout=0.5)
    c2._pool_next, pool._absorbed = (pool,), True
    d1, drop, d2 = hnn.Linear(1600, 128, activation="relu"), hnn.Dropout(0.5), hnn.Linear(128, 10)
    pool.salt, drop.salt = 7919, 3 * 7919
    if fold:
        d2._drop_in, drop._absorbed = (drop.p, drop.salt), True
    return torch.nn.Sequential(c1, c2, pool, hnn.Flatten(), d1, drop, d2)


def test_dropout_folded_into_deferred_head_matches_unfolded(monkeypatch):
    """E1: the Dropout between the last hidden Dense and the logits layer applied inside the fused loss
    kernel (head_ce_k / mlp_head_k dp: mask on the staged input, the same mask on the input gradient) trains like the
    separate dropout launches — losses and weights after 8 TrainStep steps (eager warm-up + graph replays),
    with no dropout launch left."""
    from hops_examples_amd import optim
    from hops_examples_amd.runtime.step import TrainStep

    dev = torch.device("cuda", 0)
    B = 32
    xs = torch.randint(0, 256, (8, B, 28, 28, 1), dtype=torch.uint8, device=dev)
    ys = torch.randint(0, 10, (8, B), device=dev)
    runs = []
    for fold in (True, False):
        HF.seed_device_rng(5, dev)
        torch.manual_seed(0)
        m = _e1_modules(fold).to(dev)
        ParamArena.from_module(m, dev)
        calls = {"drop": 0, "head": []}
        real_d, real_h, real_m = K.dropout, K.head_ce, K.mlp_head
        monkeypatch.setattr(K, "dropout", lambda *a, **kw: calls.__setitem__("drop", calls["drop"] + 1) or real_d(*a, **kw))
        # the deferred head runs as head_ce_k, or — with the Dense before it deferred too — as mlp_head_k
        monkeypatch.setattr(K, "head_ce", lambda *a, **kw: calls["head"].append(kw.get("drop")) or real_h(*a, **kw))
        monkeypatch.setattr(K, "mlp_head", lambda *a, **kw: calls["head"].append(kw.get("drop")) or real_m(*a, **kw))
        st = TrainStep(m, optim.Adam(m, lr=1e-3), "sparse_ce")
        ls = [float(st(xs[i], ys[i])["loss"].reshape(-1)[0]) for i in range(8)]
        monkeypatch.setattr(K, "dropout", real_d)
        monkeypatch.setattr(K, "head_ce", real_h)
        monkeypatch.setattr(K, "mlp_head", real_m)
        assert st._head_defer
        if fold:
            # (the first, probing step runs the head undeferred: its dropout is the separate kernel, fwd + bwd)
            undeferred = sum(d is None for d in calls["head"])
            assert calls["drop"] == 2 * undeferred and undeferred <= 1, calls
            assert calls["head"] and all(d[0] == 0.5 for d in calls["head"] if d is not None), calls["head"]
            assert calls["head"][-1] is not None
        else:
            assert calls["drop"] > 0 and all(d is None for d in calls["head"])
        runs.append((ls, m._hx_arena.master.float().clone()))
    assert abs(runs[0][0][0] - runs[1][0][0]) <= 1e-3 * abs(runs[1][0][0]) + 1e-4
    torch.testing.assert_close(torch.tensor(runs[0][0]), torch.tensor(runs[1][0]), rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(runs[0][1], runs[1][1], rtol=1e-2, atol=5e-3)
