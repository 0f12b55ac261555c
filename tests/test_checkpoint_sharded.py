"""Checkpoints under the sharded parameter server (gloo, world 2): every optimizer moment is
current only on its shard's owner, so checkpoint.save must gather the shards before rank 0
writes (rank 0 used to serialise its own stale copies of the other shards, which a
restore then spread to every rank).  Round trip: save -> restore into a fresh model + optimizer
-> the same next step as the uninterrupted run."""
import os
import socket
import tempfile

import torch
import torch.multiprocessing as mp


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _build(world):
    from hops_examples_amd import optim
    from hops_examples_amd.parallel import ps as P
    from hops_examples_amd.runtime.arena import ALIGN, ParamArena
    from hops_examples_amd.runtime.step import TrainStep

    torch.manual_seed(0)
    m = torch.nn.Sequential(torch.nn.Linear(8, 32), torch.nn.ReLU(), torch.nn.Linear(32, 4))
    ParamArena.from_module(m, pad_multiple=world * ALIGN)
    opt = optim.Adam(m, lr=0.01)
    dp = P.make(m, opt, "parameter_server")
    return m, opt, dp, TrainStep(m, opt, "sparse_ce", dp=dp, graph=False)


def _worker(rank, world, port, d, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    from hops_examples_amd import checkpoint
    from hops_examples_amd.parallel import dist as hdist

    hdist.init(backend="gloo")
    g = torch.Generator().manual_seed(100 + rank)
    x, y = torch.randn(16, 8, generator=g), torch.randint(0, 4, (16,), generator=g)
    m, opt, dp, st = _build(world)
    for _ in range(4):
        st(x, y)
    # the true moments: every owner's shard
    full = {}
    for k, t in m._hx_arena.states.items():
        parts = [torch.empty_like(t[dp.sl]) for _ in range(world)]
        torch.distributed.all_gather(parts, t[dp.sl].clone())
        full[k] = torch.cat(parts)
    p = checkpoint.save(d, m, opt, step=4)
    if rank == 0:
        sd = torch.load(p, map_location="cpu", weights_only=True)
        for k, t in full.items():
            assert torch.equal(sd["arena"][k], t), k
    # uninterrupted next step vs restored next step
    st(x, y)
    ref = dp.gather_master().clone()
    m2, opt2, dp2, st2 = _build(world)
    checkpoint.load(d, m2, opt2)
    st2(x, y)
    got = dp2.gather_master().clone()
    q.put((rank, float((got - ref).abs().max())))
    hdist.barrier()
    torch.distributed.destroy_process_group()


def test_sharded_ps_checkpoint_round_trip():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    d = tempfile.mkdtemp(prefix="ps_ckpt_")
    procs = [ctx.Process(target=_worker, args=(r, 2, _port_once(), d, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for _, diff in res:
        assert diff == 0.0, res


_PORT = []


def _port_once():
    if not _PORT:
        _PORT.append(_port())
    return _PORT[0]
