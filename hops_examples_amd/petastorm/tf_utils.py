"""tf.data-shaped helpers without TensorFlow: ``make_petastorm_dataset(reader)`` returns an
iterable dataset object (``.batch``, ``.take``, iteration) and ``tf_tensors(reader)`` the next
sample, so notebook code that only iterates keeps working."""
from __future__ import annotations

import itertools

import numpy as np


class PetastormDataset:
    def __init__(self, reader, batch: int | None = None, n: int | None = None):
        self.reader, self._batch, self._n = reader, batch, n

    def batch(self, b: int) -> "PetastormDataset":
        return PetastormDataset(self.reader, b, self._n)

    def take(self, n: int) -> "PetastormDataset":
        return PetastormDataset(self.reader, self._batch, n)

    def __iter__(self):
        it = iter(self.reader)
        if self._batch:
            def gen():
                while True:
                    rows = list(itertools.islice(it, self._batch))
                    if not rows:
                        return
                    yield type(rows[0])(*[np.stack([getattr(r, f) for r in rows]) for f in rows[0]._fields])
            it = gen()
        return itertools.islice(it, self._n) if self._n is not None else it

    def make_one_shot_iterator(self):
        return iter(self)


def make_petastorm_dataset(reader) -> PetastormDataset:
    return PetastormDataset(reader)


def tf_tensors(reader):
    return next(iter(reader))
