# %% [markdown]
# # Synchronous data-parallel MNIST (`experiment.mirrored`)
# Mirrors notebooks/ml/Distributed_Training/mirrored_strategy/mirroredstrategy_mnist_example.ipynb:
# one worker process per MI355X, RCCL all-reduce of one flat bf16/fp32 gradient bucket per step,
# global batch = 32 x replicas, Conv32 k2 -> Conv64 k2 -> pool2 -> Dropout .01 -> D128 -> D10.
# On a GPU-less host the same code runs 2 gloo ranks on CPU.
# %%
import os

from hops import experiment

FAST = os.environ.get("HOPSX_FAST") == "1"


def mirrored_training():
    import torch

    from hops_examples_amd import optim
    from hops_examples_amd.models.mnist import MirroredMnistCNN
    from hops_examples_amd.ops import functional as F
    from hops_examples_amd.parallel import dist, ps
    from hops_examples_amd.runtime.arena import ALIGN, ParamArena
    from hops_examples_amd.runtime.step import TrainStep

    rank, _, world = dist.init()
    dev = dist.device()
    torch.manual_seed(0)
    model = MirroredMnistCNN().to(dev)
    ParamArena.from_module(model, dev, pad_multiple=world * ALIGN)
    opt = optim.Adadelta(model, lr=1.0)
    step = TrainStep(model, opt, "sparse_ce", dp=ps.make(model, opt), graph=dev.type == "cuda")
    g = torch.Generator().manual_seed(100 + rank)  # each replica reads its own shard
    steps = 10 if FAST else 50
    x = torch.randint(0, 128, (steps, 32, 28, 28, 1), dtype=torch.uint8, generator=g)
    y = torch.randint(0, 10, (steps, 32), generator=g)
    for c in range(10):
        x[y == c, 2 * c:2 * c + 6, 4:10] += 120
    x, y = x.to(dev), y.to(dev)
    for i in range(steps):
        r = step(x[i], y[i])
    st = {}
    with torch.no_grad():
        F.loss(model(x[-1]), y[-1], stats=st)
    acc = dist.all_reduce_scalar(float(st["correct"]) / 32, "sum") / world
    return {"accuracy": acc, "loss": float(r["loss"])}


# %%
n = None if os.environ.get("HOPSX_NUM_GPUS", "") not in ("", "0") else 2
logdir, result = experiment.mirrored(mirrored_training, name="mirrored mnist", metric_key="accuracy",
                                     num_workers=n)
print(result)
