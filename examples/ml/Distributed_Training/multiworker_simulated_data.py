# %% [markdown]
# # Multi-worker collective all-reduce on simulated data (`experiment.collective_allreduce`)
# Mirrors notebooks/ml/Distributed_Training/multiworker_mirrored_strategy/
# multiworkermirroredstrategy_simulated_data_example.ipynb: random (1024, 10) binary task,
# Dense16 relu -> Dense1 sigmoid (193 params), Adam 1e-3, binary cross-entropy, 30 epochs x 5 steps.
# Unlike the reference (autoshard OFF), every worker reads its own shard.
# %%
import os

from hops import experiment

FAST = os.environ.get("HOPSX_FAST") == "1"


def train():
    import torch

    from hops_examples_amd import optim
    from hops_examples_amd.models.zoo import simulated_mlp
    from hops_examples_amd.parallel import dist, ps
    from hops_examples_amd.runtime.arena import ALIGN, ParamArena
    from hops_examples_amd.runtime.step import TrainStep

    rank, _, world = dist.init()
    dev = dist.device()
    torch.manual_seed(0)
    km = simulated_mlp()
    km.build((10,))
    net = km.net.to(dev)
    ParamArena.from_module(net, dev, pad_multiple=world * ALIGN)
    opt = optim.Adam(net, lr=1e-3, eps=1e-7)
    step = TrainStep(net, opt, "bce", dp=ps.make(net, opt), graph=dev.type == "cuda")
    g = torch.Generator().manual_seed(0)
    x = torch.rand(1024, 10, generator=g)
    y = torch.randint(0, 2, (1024, 1), generator=g).float()
    x, y = x[rank::world].to(dev), y[rank::world].to(dev)
    for epoch in range(3 if FAST else 30):
        for s in range(5):
            i = (epoch * 5 + s) * 32 % (len(x) - 32)
            r = step(x[i:i + 32], y[i:i + 32])
    return {"loss": float(r["loss"]), "accuracy": float(r["correct"]) / 32}


# %%
n = None if os.environ.get("HOPSX_NUM_GPUS", "") not in ("", "0") else 2
logdir, result = experiment.collective_allreduce(train, name="multiworker simulated", num_workers=n)
print(result)
