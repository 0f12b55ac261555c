"""The data-parallel instantiation of the persistent flagship step (csrc/ops/mnist_persist.hip
"data-parallel exchange", runtime/persist.py) in loopback mode: one process plays `world` ranks, so
every exchange (pooled-activation and dh^T fragments, head gradients, conv slice sums, flag epochs
across launches, rank-order sums) runs through the same code as on 8 GPUs, with every "peer" holding
this rank's own batch.  The global-batch mean over `world` identical replicas is the one-replica
mean, so:
  * world 2: every sum is x/2 + x/2 — exact in fp32 — and the run must be BIT-IDENTICAL to world 1;
  * world 8: partial sums k*x/8 can round, so it must track world 1 to fp32 noise.
Two real ranks cannot share one GPU (2 x 201 one-per-CU workgroups are not co-resident), so the
cross-GPU memory path itself is exercised by bench.py's multi-GPU runs (selftest + replica check).

Reference workload: notebooks/ml/Distributed_Training/mirrored_strategy/
mirroredstrategy_mnist_example.ipynb:128-131 (global batch = 32 x replicas), :189-222.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from hops_examples_amd import optim  # noqa: E402
from hops_examples_amd.models.mnist import MirroredMnistCNN  # noqa: E402
from hops_examples_amd.runtime import persist  # noqa: E402
from hops_examples_amd.runtime.arena import ParamArena  # noqa: E402

B = 32


def _run(loopback, n, seed=1, spl=4, nb=5):
    from hops_examples_amd.ops import functional as HF

    dev = torch.device("cuda", 0)
    torch.manual_seed(seed)
    HF.seed_device_rng(11, dev)
    m = MirroredMnistCNN().to(dev)
    m.pool.salt = 7919
    ParamArena.from_module(m, dev)
    opt = optim.Adadelta(m, lr=1.0)
    g = torch.Generator().manual_seed(seed + 7)
    xs = torch.randint(0, 256, (nb, B, 28, 28, 1), dtype=torch.uint8, generator=g).to(dev)
    ys = torch.randint(0, 10, (nb, B), dtype=torch.int64, generator=g).to(dev)
    eng = persist.PersistentMnistStep(m, opt, steps_per_launch=spl, loopback=loopback)
    losses = []
    left = n
    while left > 0:  # several launches: the exchange epochs must carry across launch boundaries
        k = min(left, spl)
        eng.run_resident(xs, ys, k)
        torch.cuda.synchronize()
        eng.check()
        losses += eng.losses(k)[:, 0].cpu().tolist()
        left -= k
    out = (eng.arena.master.clone(), eng.s1.clone(), eng.s2.clone(), torch.tensor(losses), int(eng.cursor.item()))
    eng.close()
    return out


def test_loopback_two_ranks_bit_identical_to_one():
    n = 10
    m1, a1, b1, l1, c1 = _run(0, n)
    m2, a2, b2, l2, c2 = _run(2, n)
    assert c1 == c2 == n % 5
    assert torch.equal(l1, l2), (l1, l2)
    assert torch.equal(m1, m2) and torch.equal(a1, a2) and torch.equal(b1, b2)


def test_loopback_eight_ranks_tracks_one():
    n = 6
    m1, a1, _, l1, _ = _run(0, n)
    m8, a8, _, l8, _ = _run(8, n)
    torch.testing.assert_close(l8, l1, rtol=1e-4, atol=0)
    m0 = _run(0, 0)[0]  # the initial weights (no step)
    d1, d8 = (m1 - m0).double(), (m8 - m0).double()
    cos = float(torch.nn.functional.cosine_similarity(d1, d8, dim=0))
    assert cos > 0.9999, cos


def test_loopback_selftest_and_digest():
    from hops_examples_amd.ops import functional as HF

    dev = torch.device("cuda", 0)
    torch.manual_seed(3)
    HF.seed_device_rng(5, dev)
    m = MirroredMnistCNN().to(dev)
    ParamArena.from_module(m, dev)
    opt = optim.Adadelta(m, lr=1.0)
    eng = persist.PersistentMnistStep(m, opt, steps_per_launch=4, loopback=4)
    before = eng.param_digest()
    rng = eng.rng.clone()
    assert eng.selftest()
    # the pre-flight leaves the real state untouched
    assert eng.param_digest() == before and torch.equal(eng.rng, rng)
    assert eng.verify_replicas()["identical"]
    eng.close()
