"""``hops`` API surface (experiment, hdfs, tensorboard, model, serving, kafka, tls, featurestore,
jobs, project, dataset, hive, elasticsearch, …) backed by hops_examples_amd."""
from hops_examples_amd import _alias

_alias.install("hops", "hops_examples_amd", {"featurestore": "hops_examples_amd.featurestore.legacy"})


def __getattr__(name):
    return _alias.module_getattr("hops", name)
