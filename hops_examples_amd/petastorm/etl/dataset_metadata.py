"""Dataset materialisation: Parquet row groups + ``_common_metadata`` holding the Unischema.

``materialize_dataset(spark, url, schema, rowgroup_size_mb)`` is a context manager
(PetastormHelloWorld.ipynb: ``with materialize_dataset(...)``); without Spark, rows are
written inside it with :func:`write_rows` (or any Parquet writer), and on exit the
schema metadata is stored so readers can decode the binary columns.
"""
from __future__ import annotations

import contextlib
import json
from pathlib import Path

import pyarrow as pa
import pyarrow.parquet as pq

from ..unischema import Unischema, dict_to_spark_row

META = "_common_metadata"


def _local(url: str) -> Path:
    from ... import hdfs

    return Path(hdfs._resolve(url))


@contextlib.contextmanager
def materialize_dataset(spark, dataset_url: str, schema: Unischema, row_group_size_mb: int | None = None,
                        filesystem_factory=None, use_summary_metadata: bool = False):
    path = _local(dataset_url)
    path.mkdir(parents=True, exist_ok=True)
    yield path
    (path / META).write_text(json.dumps({"unischema": schema.to_json(), "row_group_size_mb": row_group_size_mb}))


def write_rows(dataset_url: str, schema: Unischema, rows, rows_per_group: int | None = None,
               row_group_size_mb: int = 256, files: int = 1, mode: str = "overwrite") -> Path:
    """Encode dict rows with the schema codecs and write them as Parquet row groups."""
    path = _local(dataset_url)
    if mode == "overwrite" and path.exists():
        for p in path.glob("*.parquet"):
            p.unlink()
    path.mkdir(parents=True, exist_ok=True)
    enc = [dict_to_spark_row(schema, r) for r in rows]
    if rows_per_group is None:
        est = max(1, sum(len(v) if isinstance(v, (bytes, str)) else 8 for v in enc[0].values())) if enc else 1
        rows_per_group = max(1, int(row_group_size_mb * 2 ** 20 // est))
    sch = schema.as_spark_schema()
    per_file = -(-len(enc) // files) if enc else 0
    for fi in range(files):
        chunk = enc[fi * per_file:(fi + 1) * per_file]
        if not chunk and fi:
            continue
        tbl = pa.Table.from_pylist(chunk, schema=sch)
        pq.write_table(tbl, str(path / f"part-{fi:05d}.parquet"), row_group_size=rows_per_group)
    (path / META).write_text(json.dumps({"unischema": schema.to_json(), "row_group_size_mb": row_group_size_mb}))
    return path


def get_schema_from_dataset_url(dataset_url: str) -> Unischema | None:
    p = _local(dataset_url) / META
    if not p.exists():
        return None
    return Unischema.from_json(json.loads(p.read_text())["unischema"])
