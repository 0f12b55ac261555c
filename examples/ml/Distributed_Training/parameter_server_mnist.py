# %% [markdown]
# # Parameter-server training (`experiment.parameter_server`)
# The reference names this mode in every experiment notebook's prose ("ParameterServerStrategy,
# CollectiveAllReduceStrategy and MultiworkerMirroredStrategy", notebooks/ml/Experiment/Tensorflow/mnist.ipynb:52)
# and sizes it with `"spark.tensorflow.num.ps": 1` (jobs-client/spark/job_config.json:13).  Here every worker is
# also the parameter server of 1/world of the flat parameter arena (parallel/ps.py ShardedPS): gradients are
# reduce-scattered to the shard owners, each owner runs the fused Adadelta on its shard only, and the new bf16
# weights are all-gathered.  Model: the MirroredStrategy MNIST CNN (E3), 32 images per worker, synthetic data.
# %%
import os

from hops import experiment

FAST = os.environ.get("HOPSX_FAST") == "1"


def train():
    import torch

    from hops_examples_amd import optim
    from hops_examples_amd.models.mnist import MirroredMnistCNN
    from hops_examples_amd.parallel import dist, ps
    from hops_examples_amd.runtime.arena import ALIGN, ParamArena
    from hops_examples_amd.runtime.step import TrainStep

    rank, _, world = dist.init()
    dev = dist.device()
    torch.manual_seed(0)
    net = MirroredMnistCNN().to(dev)
    ParamArena.from_module(net, dev, pad_multiple=world * ALIGN)  # shards of equal size
    opt = optim.Adadelta(net, lr=1.0)
    engine = ps.make(net, opt)  # HOPSX_DP_MODE=parameter_server, set by experiment.parameter_server
    step = TrainStep(net, opt, "sparse_ce", dp=engine, graph=dev.type == "cuda")
    g = torch.Generator().manual_seed(rank)
    x = torch.randint(0, 256, (8, 32, 28, 28, 1), dtype=torch.uint8, generator=g).to(dev)
    y = torch.randint(0, 10, (8, 32), generator=g).to(dev)
    losses = []
    for s in range(12 if FAST else 60):
        r = step(x[s % 8], y[s % 8])
        losses.append(float(r["loss"]))
    ident = engine.verify_replicas()["identical"] if hasattr(engine, "verify_replicas") and engine else True
    return {"loss": losses[-1], "first_loss": losses[0], "accuracy": float(r["correct"]) / 32,
            "engine": type(engine).__name__ if engine else "single", "num_ps": int(os.environ.get("HOPSX_NUM_PS", 0)),
            "replicas_identical": bool(ident)}


# %%
n = None if os.environ.get("HOPSX_NUM_GPUS", "") not in ("", "0") else 2
logdir, result = experiment.parameter_server(train, name="mnist parameter server", num_workers=n, num_ps=1,
                                             metric_key="accuracy")
print(logdir, result)
assert result["loss"] < result["first_loss"]
