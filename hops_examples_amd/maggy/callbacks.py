"""Training-loop callbacks that feed the lagom reporter (maggy.callbacks.KerasBatchEnd /
KerasEpochEnd, maggy-fashion-mnist-example.ipynb:265).  hopsx training loops call
``on_batch_end(batch, logs)`` / ``on_epoch_end(epoch, logs)`` with a dict of
host-side metric values."""
from __future__ import annotations


class _Base:
    def __init__(self, reporter, metric: str = "loss"):
        self.reporter, self.metric = reporter, metric

    def _report(self, logs, step):
        v = (logs or {}).get(self.metric)
        if v is not None:
            self.reporter.broadcast(v, step)


class KerasBatchEnd(_Base):
    def __init__(self, reporter, metric: str = "loss"):
        super().__init__(reporter, metric)
        self._step = 0

    def on_batch_end(self, batch, logs=None):
        self._report(logs, self._step)
        self._step += 1

    on_train_batch_end = on_batch_end


class KerasEpochEnd(_Base):
    def on_epoch_end(self, epoch, logs=None):
        self._report(logs, epoch)


BatchEnd = KerasBatchEnd
EpochEnd = KerasEpochEnd
