"""Failure detection, fault injection and checkpoint/resume on CPU.

* the first failing rank of a gloo gang ends the job at once (the surviving rank would block
  in its next collective forever) and the error names that rank;
* a rank that stops making progress (HOPSX_FAULT ...:hang) is caught by the heartbeat watchdog;
* ``max_restarts`` relaunches the gang and the training function resumes from its latest
  checkpoint (the injected fault fires only on the first attempt);
* checkpoint save/load round-trips the parameter arena, optimizer state, step counter and RNG.
"""
import time
from pathlib import Path

import pytest
import torch


def _gang_train(steps=12, ckpt_every=4):
    def train():
        import os

        import torch
        import torch.distributed as dist

        from hops_examples_amd import checkpoint, optim, tensorboard
        from hops_examples_amd.parallel import dist as hdist
        from hops_examples_amd.runtime import health
        from hops_examples_amd.runtime.arena import ParamArena

        rank, _, world = hdist.init(backend="gloo")
        torch.manual_seed(0)
        m = torch.nn.Sequential(torch.nn.Linear(6, 16), torch.nn.ReLU(), torch.nn.Linear(16, 1))
        ParamArena.from_module(m)
        opt = optim.Adam(m, lr=1e-2)
        ck = os.path.join(tensorboard.logdir(), "ckpt")
        r = checkpoint.load(ck, m, opt)
        start = 0 if r is None else r["step"]
        for step in range(start + 1, steps + 1):
            health.beat(step)
            x = torch.randn(8, 6)
            loss = m(x).float().pow(2).mean()
            loss.backward()
            for p in m.parameters():
                dist.all_reduce(p._hx_grad)
            opt.step()
            if step % ckpt_every == 0:
                checkpoint.save(ck, m, opt, step=step)
        return {"start": start, "world": world, "restart": int(os.environ.get("HOPSX_RESTART", "0"))}

    return train


def test_first_failure_tears_down_gang(project_root, monkeypatch):
    from hops_examples_amd import experiment

    monkeypatch.setenv("HOPSX_NUM_GPUS", "0")
    monkeypatch.setenv("HOPSX_FAULT", "1:3:raise")
    t0 = time.time()
    with pytest.raises(Exception) as ei:
        experiment.mirrored(_gang_train(), name="fault", num_workers=2, timeout=120)
    assert time.time() - t0 < 100  # rank 0 was killed, not left waiting in all_reduce
    msg = str(ei.value)
    assert "rank 1" in msg and "injected failure on rank 1 at step 3" in msg


def test_heartbeat_watchdog_catches_hang(project_root, monkeypatch):
    from hops_examples_amd import experiment

    monkeypatch.setenv("HOPSX_NUM_GPUS", "0")
    monkeypatch.setenv("HOPSX_FAULT", "1:3:hang")
    monkeypatch.setenv("HOPSX_HEARTBEAT_S", "0.1")
    with pytest.raises(Exception) as ei:
        experiment.mirrored(_gang_train(steps=200), name="hang", num_workers=2, timeout=150, heartbeat_timeout=6)
    assert "stalled" in str(ei.value)


def test_restart_resumes_from_checkpoint(project_root, monkeypatch):
    from hops_examples_amd import experiment

    monkeypatch.setenv("HOPSX_NUM_GPUS", "0")
    monkeypatch.setenv("HOPSX_FAULT", "0:7:exit")
    d, res = experiment.mirrored(_gang_train(), name="restart", num_workers=2, timeout=150, max_restarts=1)
    assert res["restart"] == 1 and res["start"] == 4 and res["world"] == 2
    import json

    meta = json.loads((Path(d) / "experiment.json").read_text())
    assert meta["status"] == "FINISHED" and meta["attempts"] == 2


def test_checkpoint_roundtrip(tmp_path):
    from hops_examples_amd import checkpoint, optim
    from hops_examples_amd.models.mnist import TorchMnistNet
    from hops_examples_amd.ops import functional as HF
    from hops_examples_amd.runtime.arena import ParamArena

    def make():
        torch.manual_seed(3)
        m = TorchMnistNet()
        ParamArena.from_module(m)
        return m, optim.Adam(m, lr=1e-3)

    def step(m, opt):
        x = torch.randint(0, 256, (4, 28, 28, 1), dtype=torch.uint8)
        y = torch.randint(0, 10, (4,))
        HF.loss(m(x), y).backward()
        opt.step()

    m, opt = make()
    for _ in range(2):
        step(m, opt)
    p = checkpoint.save(tmp_path, m, opt, step=2, epoch=1)
    assert p is not None and checkpoint.latest(tmp_path) == p
    torch.manual_seed(42)
    step(m, opt)
    ref = m._hx_arena.master.clone()

    m2, opt2 = make()
    r = checkpoint.load(tmp_path, m2, opt2)
    assert r == {"step": 2, "epoch": 1}
    assert torch.equal(opt2.step_count, torch.tensor([2.0]))
    torch.manual_seed(42)
    step(m2, opt2)
    torch.testing.assert_close(m2._hx_arena.master, ref, rtol=0, atol=0)
    for s in range(3, 8):
        checkpoint.save(tmp_path, m2, opt2, step=s, keep=3)
    assert [q.name for q in checkpoint.list_checkpoints(tmp_path)] == ["ckpt-5.pt", "ckpt-6.pt", "ckpt-7.pt"]
