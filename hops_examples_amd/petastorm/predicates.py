"""Row predicates for ``make_reader(predicate=...)``."""
from __future__ import annotations


class PredicateBase:
    def get_fields(self) -> set:
        raise NotImplementedError

    def do_include(self, values: dict) -> bool:
        raise NotImplementedError


class in_lambda(PredicateBase):  # noqa: N801 (petastorm name)
    def __init__(self, fields, fn, state_arg=None):
        self.fields, self.fn, self.state = list(fields), fn, state_arg

    def get_fields(self):
        return set(self.fields)

    def do_include(self, values):
        args = [values[f] for f in self.fields]
        return self.fn(*args, self.state) if self.state is not None else self.fn(*args)


class in_set(PredicateBase):  # noqa: N801
    def __init__(self, values, field):
        self.values, self.field = set(values), field

    def get_fields(self):
        return {self.field}

    def do_include(self, values):
        return values[self.field] in self.values


class in_negate(PredicateBase):  # noqa: N801
    def __init__(self, p):
        self.p = p

    def get_fields(self):
        return self.p.get_fields()

    def do_include(self, values):
        return not self.p.do_include(values)
