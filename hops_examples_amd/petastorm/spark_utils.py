"""``dataset_as_rdd`` without Spark: the decoded rows as a list (RDD stand-in)."""
from __future__ import annotations

from .reader import make_reader


class _LocalRDD(list):
    def first(self):
        return self[0]

    def count(self):
        return len(self)

    def map(self, fn):
        return _LocalRDD(fn(r) for r in self)


def dataset_as_rdd(dataset_url, spark_session=None, schema_fields=None, hdfs_driver=None):
    with make_reader(dataset_url, schema_fields=schema_fields, shuffle_row_groups=False) as r:
        return _LocalRDD(r)
