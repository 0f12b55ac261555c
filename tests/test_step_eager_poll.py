"""TrainStep's eager path polls the data-parallel engine's failure flag like the replay path
(a sticky P2P error must surface within poll_every steps, not only at close())."""
import torch

from hops_examples_amd import optim
from hops_examples_amd.models.zoo import simulated_mlp
from hops_examples_amd.runtime.arena import ParamArena
from hops_examples_amd.runtime.step import TrainStep


class _FailingEngine:
    """Stands in for DataParallel after a peer timed out: the step tail does nothing, poll raises
    on every ``poll_every``-th call."""

    poll_every = 3

    def __init__(self):
        self.polls = 0

    def grad_scale(self):
        return 1.0

    def finish(self):
        pass

    def allreduce_all(self):
        pass

    def poll(self):
        self.polls += 1
        if self.polls % self.poll_every == 0:
            raise RuntimeError("P2P collective: rank 1 never raised its flag")


def test_eager_step_polls_engine():
    m = simulated_mlp()
    m.build((10,))
    net = m.net
    ParamArena.from_module(net)
    opt = optim.Adam(net, lr=1e-3)
    eng = _FailingEngine()
    st = TrainStep(net, opt, "bce", dp=eng, graph=False)
    x, y = torch.randn(8, 10), torch.randint(0, 2, (8, 1)).float()
    raised_at = None
    for i in range(10):
        try:
            st(x, y)
        except RuntimeError as e:
            assert "never raised" in str(e)
            raised_at = i + 1
            break
    assert raised_at == eng.poll_every
