"""Searchspace: typed hyper-parameter domains (INTEGER / DOUBLE / DISCRETE / CATEGORICAL)."""
from __future__ import annotations

import itertools
import random


class Searchspace:
    INTEGER, DOUBLE, DISCRETE, CATEGORICAL = "INTEGER", "DOUBLE", "DISCRETE", "CATEGORICAL"

    def __init__(self, **kwargs):
        self._hparams: dict[str, tuple[str, list]] = {}
        for name, value in kwargs.items():
            self.add(name, value)

    def add(self, name: str, value) -> None:
        if not isinstance(value, (tuple, list)) or len(value) != 2:
            raise ValueError(f"hyperparameter {name}: expected (type, feasible region)")
        t, region = value
        t = str(t).upper()
        if t not in (self.INTEGER, self.DOUBLE, self.DISCRETE, self.CATEGORICAL):
            raise ValueError(f"hyperparameter {name}: unknown type {value[0]!r}")
        region = list(region)
        if t in (self.INTEGER, self.DOUBLE):
            if len(region) != 2 or region[0] > region[1]:
                raise ValueError(f"hyperparameter {name}: region must be [low, high]")
            if t == self.INTEGER and not all(float(x).is_integer() for x in region):
                raise ValueError(f"hyperparameter {name}: INTEGER bounds must be integers")
        if name in self._hparams:
            raise ValueError(f"hyperparameter {name} already defined")
        self._hparams[name] = (t, region)
        print(f"Hyperparameter added: {name}")

    def names(self) -> dict:
        return {k: v[0] for k, v in self._hparams.items()}

    def get(self, name, default=None):
        return self._hparams.get(name, default)

    def items(self):
        return self._hparams.items()

    def to_dict(self) -> dict:
        return {k: {"type": v[0], "values": v[1]} for k, v in self._hparams.items()}

    def __iter__(self):
        return iter(self._hparams)

    def __len__(self):
        return len(self._hparams)

    def sample(self, rng: random.Random) -> dict:
        out = {}
        for k, (t, r) in self._hparams.items():
            if t == self.INTEGER:
                out[k] = rng.randint(int(r[0]), int(r[1]))
            elif t == self.DOUBLE:
                out[k] = rng.uniform(float(r[0]), float(r[1]))
            else:
                out[k] = rng.choice(r)
        return out

    def get_random_parameter_values(self, num: int, seed: int | None = None) -> list[dict]:
        rng = random.Random(seed)
        return [self.sample(rng) for _ in range(num)]

    def grid(self, points_per_axis: int = 3) -> list[dict]:
        axes = []
        for k, (t, r) in self._hparams.items():
            if t == self.INTEGER:
                lo, hi = int(r[0]), int(r[1])
                vals = sorted({round(lo + (hi - lo) * i / max(1, points_per_axis - 1)) for i in range(points_per_axis)})
            elif t == self.DOUBLE:
                vals = [r[0] + (r[1] - r[0]) * i / max(1, points_per_axis - 1) for i in range(points_per_axis)]
            else:
                vals = list(r)
            axes.append([(k, v) for v in vals])
        return [dict(c) for c in itertools.product(*axes)]

    def __repr__(self):
        return f"Searchspace({self.to_dict()})"
