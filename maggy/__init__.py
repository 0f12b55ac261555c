"""``maggy`` API surface backed by hops_examples_amd.maggy."""
from hops_examples_amd import _alias
from hops_examples_amd.maggy import *  # noqa: F401,F403
from hops_examples_amd.maggy import Searchspace, experiment  # noqa: F401

_alias.install("maggy", "hops_examples_amd.maggy")


def __getattr__(name):
    return _alias.module_getattr("maggy", name)
