"""``hsfs`` API surface (connection, feature groups, queries, training datasets, rules)
backed by hops_examples_amd.featurestore."""
from hops_examples_amd import _alias
from hops_examples_amd.featurestore import *  # noqa: F401,F403
from hops_examples_amd.featurestore import connection  # noqa: F401

_alias.install("hsfs", "hops_examples_amd.featurestore",
               {"rule": "hops_examples_amd.featurestore.rules", "feature": "hops_examples_amd.featurestore.core",
                "feature_group": "hops_examples_amd.featurestore.core", "constructor": "hops_examples_amd.featurestore.core",
                "training_dataset": "hops_examples_amd.featurestore.training_dataset",
                "expectation": "hops_examples_amd.featurestore.rules",
                "storage_connector": "hops_examples_amd.featurestore.store",
                "client": "hops_examples_amd.featurestore.store"})


def __getattr__(name):
    return _alias.module_getattr("hsfs", name)
