"""Import aliases so reference notebooks run unchanged: ``from hops import experiment``,
``import hsfs``, ``from maggy import experiment``, ``from petastorm import make_reader`` resolve to
hops_examples_amd modules (the same module objects, not copies)."""
from __future__ import annotations

import importlib
import importlib.abc
import importlib.util
import sys


class AliasFinder(importlib.abc.MetaPathFinder, importlib.abc.Loader):
    def __init__(self, prefix: str, target: str, mapping: dict | None = None):
        self.prefix, self.target, self.mapping = prefix, target, mapping or {}

    def resolve(self, sub: str) -> str:
        head, _, rest = sub.partition(".")
        if head in self.mapping:
            return self.mapping[head] + ("." + rest if rest else "")
        return f"{self.target}.{sub}"

    def find_spec(self, fullname, path=None, target=None):
        if not fullname.startswith(self.prefix + "."):
            return None
        tgt = self.resolve(fullname[len(self.prefix) + 1:])
        if importlib.util.find_spec(tgt) is None:
            return None
        return importlib.util.spec_from_loader(fullname, self, origin=tgt)

    def create_module(self, spec):
        return importlib.import_module(spec.origin)

    def exec_module(self, module):
        pass


def install(prefix: str, target: str, mapping: dict | None = None) -> AliasFinder:
    for f in sys.meta_path:
        if isinstance(f, AliasFinder) and f.prefix == prefix:
            return f
    f = AliasFinder(prefix, target, mapping)
    sys.meta_path.insert(0, f)
    return f


def module_getattr(prefix: str, name: str):
    try:
        return importlib.import_module(f"{prefix}.{name}")
    except ModuleNotFoundError as e:
        raise AttributeError(f"module {prefix!r} has no attribute {name!r}") from e
