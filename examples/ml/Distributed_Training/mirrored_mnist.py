# %% [markdown]
# # Synchronous data-parallel MNIST (`experiment.mirrored`)
# Mirrors notebooks/ml/Distributed_Training/mirrored_strategy/mirroredstrategy_mnist_example.ipynb:
# one worker process per MI355X, global batch = 32 x replicas, Conv32 k2 -> Conv64 k2 -> pool2 ->
# Dropout .01 -> D128 -> D10, Adadelta(1.0).  `make_step` picks the engine: on MI355X the persistent
# whole-step kernel (32 steps per launch; with N GPUs the replicas exchange activations and gradients
# over xGMI inside the launch), else the hipGraph TrainStep with a bucketed all-reduce.  On a GPU-less
# host the same code runs 2 gloo ranks on CPU.
# %%
import os

from hops import experiment

FAST = os.environ.get("HOPSX_FAST") == "1"


def mirrored_training():
    import torch

    from hops_examples_amd import optim
    from hops_examples_amd.models.mnist import MirroredMnistCNN
    from hops_examples_amd.ops import functional as F
    from hops_examples_amd.parallel import dist
    from hops_examples_amd.runtime.arena import ALIGN, ParamArena
    from hops_examples_amd.runtime.step import make_step

    rank, _, world = dist.init()
    dev = dist.device()
    torch.manual_seed(0)
    model = MirroredMnistCNN().to(dev)
    ParamArena.from_module(model, dev, pad_multiple=world * ALIGN)
    opt = optim.Adadelta(model, lr=1.0)
    step = make_step(model, opt, "sparse_ce", dp="auto", batch=32, graph=dev.type == "cuda")
    g = torch.Generator().manual_seed(100 + rank)  # each replica reads its own shard
    steps = 10 if FAST else 50
    x = torch.randint(0, 128, (steps, 32, 28, 28, 1), dtype=torch.uint8, generator=g)
    y = torch.randint(0, 10, (steps, 32), generator=g)
    for c in range(10):
        x[y == c, 2 * c:2 * c + 6, 4:10] += 120
    x, y = x.to(dev), y.to(dev)  # the epoch stays resident in HBM
    r = step.run_resident(x, y, steps)
    # throughput of the same training loop, timed (no data movement: the batches are resident)
    import time

    n_timed = 64 if FAST or dev.type != "cuda" else 3200
    step.run_resident(x, y, 32)
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    dist.barrier()
    t0 = time.perf_counter()
    r = step.run_resident(x, y, n_timed)
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    el = dist.all_reduce_scalar(time.perf_counter() - t0, "max")
    st = {}
    with torch.no_grad():
        F.loss(model(x[-1]), y[-1], stats=st)
    acc = dist.all_reduce_scalar(float(st["correct"]) / 32, "sum") / world
    return {"accuracy": acc, "loss": float(r["loss"]), "engine": getattr(step, "kind", type(step).__name__),
            "images_per_sec": round(32 * world * n_timed / el, 1)}


# %%
n = None if os.environ.get("HOPSX_NUM_GPUS", "") not in ("", "0") else 2
logdir, result = experiment.mirrored(mirrored_training, name="mirrored mnist", metric_key="accuracy",
                                     num_workers=n)
print(result)
