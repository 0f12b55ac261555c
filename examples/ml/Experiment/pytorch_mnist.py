# %% [markdown]
# # PyTorch-style MNIST `Net` with a custom train/test loop
# Mirrors notebooks/ml/Experiment/PyTorch/mnist.ipynb: Conv20 k5 -> pool2 -> Conv50 k5 -> pool2 ->
# FC500 -> FC10, SGD(0.01, momentum 0.5), batch 64, SummaryWriter scalars, an image artifact.
# %%
import os

from hops import experiment

FAST = os.environ.get("HOPSX_FAST") == "1"


def wrapper():
    import numpy as np
    import torch

    from hops import tensorboard
    from hops_examples_amd import optim
    from hops_examples_amd.models.mnist import TorchMnistNet
    from hops_examples_amd.ops import functional as F
    from hops_examples_amd.runtime.arena import ParamArena
    from hops_examples_amd.runtime.step import TrainStep

    dev = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
    torch.manual_seed(1)
    n = 640 if FAST else 12800
    g = torch.Generator().manual_seed(0)
    x = torch.randint(0, 128, (n, 28, 28, 1), dtype=torch.uint8, generator=g)
    y = torch.randint(0, 10, (n,), generator=g)
    for c in range(10):
        x[y == c, 2 * c:2 * c + 6, 10:16] += 120
    model = TorchMnistNet().to(dev)
    ParamArena.from_module(model, dev)
    opt = optim.SGD(model, lr=0.01, momentum=0.5)
    step = TrainStep(model, opt, "sparse_ce", graph=dev.type == "cuda")
    writer = tensorboard.SummaryWriter(tensorboard.logdir())
    xd, yd = x.to(dev), y.to(dev)
    for epoch in range(1 if FAST else 2):
        for i in range(0, n - 63, 64):
            r = step(xd[i:i + 64], yd[i:i + 64])
            if i % (64 * 20) == 0:
                writer.add_scalar("train/loss", float(r["loss"]), epoch * n + i)
    model.eval()
    with torch.no_grad():
        st = {}
        F.loss(model(xd[:1000]), yd[:1000], stats=st)
        acc = float(st["correct"]) / min(1000, n)
    writer.close()
    np.save("train_summary.npy", np.array([acc]))
    return {"accuracy": acc, "train_summary": "train_summary.npy"}


# %%
logdir, result = experiment.launch(wrapper, name="pytorch mnist", local_logdir=True, metric_key="accuracy")
print(result)
