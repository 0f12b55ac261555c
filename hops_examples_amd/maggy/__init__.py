"""maggy-compatible asynchronous hyper-parameter search and ablation studies.

Reference:
  Searchspace(kernel=('INTEGER', [2, 8]), …), .add(...) prints "Hyperparameter added: <name>"
      notebooks/ml/Parallel_Experiments/Maggy/maggy-fashion-mnist-example.ipynb:114-127
  experiment.lagom(train_fn, searchspace, optimizer='randomsearch', direction, num_trials, name,
                   hb_interval, es_interval, es_min)                              :318-327
  reporter.broadcast(metric=…), callbacks.KerasBatchEnd(reporter, metric='accuracy') :265, …/maggy-pytorch-example.ipynb:89
  AblationStudy('titanic_train_dataset', 1, label_name='survived') + LOCO ablator
      …/maggy-ablation-titanic-example.ipynb:135-455

Execution model on MI355X: the driver runs in the notebook process; every trial
is a worker process pinned to one GPU (8 concurrent trials per node); workers
heartbeat their latest metric to the driver over a local TCP socket every
``hb_interval`` seconds and the driver applies the median early-stopping rule
(stop a trial whose metric at step s is worse than the median of finished
trials at s, once ``es_min`` trials have finished; checked every
``es_interval`` seconds).
"""
from . import callbacks, tensorboard  # noqa: F401
from .ablation import AblationStudy  # noqa: F401
from .experiment import lagom  # noqa: F401
from .reporter import EarlyStopException, Reporter  # noqa: F401
from .searchspace import Searchspace  # noqa: F401

__all__ = ["Searchspace", "lagom", "Reporter", "EarlyStopException", "AblationStudy", "callbacks", "tensorboard"]
