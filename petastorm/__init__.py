"""``petastorm`` API surface backed by hops_examples_amd.petastorm."""
from hops_examples_amd import _alias
from hops_examples_amd.petastorm import *  # noqa: F401,F403
from hops_examples_amd.petastorm import make_batch_reader, make_reader  # noqa: F401

_alias.install("petastorm", "hops_examples_amd.petastorm")


def __getattr__(name):
    return _alias.module_getattr("petastorm", name)
