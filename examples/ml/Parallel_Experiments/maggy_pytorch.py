# %% [markdown]
# # maggy with a hand-written training loop (regression, direction='min')
# Mirrors notebooks/ml/Parallel_Experiments/Maggy/maggy-pytorch-example.ipynb:
# f(x) = x0 * exp(x0^2 - x1^2), MLP 2 -> l1 -> l2 -> 1, Adam 1e-3, MSE, reporter.broadcast.
# %%
import os

from maggy import Searchspace, experiment

FAST = os.environ.get("HOPSX_FAST") == "1"
sp = Searchspace(l1_size=("INTEGER", [2, 32]), l2_size=("INTEGER", [2, 32]), batch_size=("INTEGER", [2, 16]))


def train_fn(l1_size, l2_size, batch_size, reporter):
    import torch

    from hops_examples_amd import optim
    from hops_examples_amd.models.zoo import maggy_regressor
    from hops_examples_amd.runtime.arena import ParamArena
    from hops_examples_amd.runtime.step import TrainStep

    g = torch.Generator().manual_seed(0)
    x = torch.rand(1000, 2, generator=g) * 4 - 2
    y = (x[:, 0] * torch.exp(-x[:, 0] ** 2 - x[:, 1] ** 2)).unsqueeze(1)
    m = maggy_regressor(l1_size, l2_size)
    m.build((2,))
    ParamArena.from_module(m.net)
    st = TrainStep(m.net, optim.Adam(m.net, lr=1e-3), "mse", graph=False)
    for epoch in range(3 if FAST else 100):
        for i in range(0, 1000 - batch_size + 1, batch_size):
            r = st(x[i:i + batch_size], y[i:i + batch_size])
        reporter.broadcast(metric=float(r["loss"]), step=epoch)
    return float(r["loss"])


# %%
result = experiment.lagom(train_fn, searchspace=sp, optimizer="randomsearch", direction="min",
                          num_trials=2, name="pytorch-regression", hb_interval=1, es_interval=10)
print(result)
