"""Petastorm-compatible datasets on Parquet (notebooks/featurestore/petastorm/PetastormHelloWorld.ipynb).

Unischema + codecs (scalar / PNG-JPEG image / ndarray), ``materialize_dataset`` +
``write_rows``, ``make_reader`` / ``make_batch_reader`` with sharding, predicates,
row-group shuffling and a decode thread pool, and a torch ``DataLoader`` that can
stage batches straight into HBM.  Python-only (no Spark / TF in the image).
"""
from . import codecs, predicates, pytorch, spark_utils, tf_utils, types, unischema  # noqa: F401
from .etl.dataset_metadata import materialize_dataset, write_rows  # noqa: F401
from .reader import make_batch_reader, make_reader  # noqa: F401
from .unischema import Unischema, UnischemaField, dict_to_spark_row  # noqa: F401
