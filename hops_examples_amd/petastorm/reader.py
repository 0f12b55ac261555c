"""Readers: ``make_reader`` (Unischema datasets, one decoded row at a time) and
``make_batch_reader`` (any Parquet store, one column batch per row group).

Work unit = Parquet row group.  Sharding assigns row group i to shard
``i % shard_count`` (each DP rank passes ``cur_shard=rank``), ``shuffle_row_groups``
permutes the work list per epoch, and decoding (PNG / ndarray codecs) runs in a
thread pool of ``workers_count`` — the codec work releases the GIL inside zlib/PIL.
"""
from __future__ import annotations

import collections
import concurrent.futures as cf
import random
from pathlib import Path

import numpy as np
import pyarrow.parquet as pq

from .etl.dataset_metadata import _local, get_schema_from_dataset_url


def _row_groups(path: Path):
    files = sorted(p for p in path.rglob("*.parquet")) if path.is_dir() else [path]
    out = []
    for f in files:
        md = pq.ParquetFile(str(f)).metadata
        out += [(f, i) for i in range(md.num_row_groups)]
    return out


class Reader:
    def __init__(self, dataset_url, schema_fields=None, reader_pool_type="thread", workers_count=10,
                 shard_count=None, cur_shard=None, predicate=None, num_epochs=1, shuffle_row_groups=True,
                 shuffle_row_drop_partitions=1, seed=None, batched=False, **_):
        self.path = _local(dataset_url)
        self.schema = get_schema_from_dataset_url(dataset_url)
        if self.schema is None and not batched:
            raise ValueError(f"{dataset_url} is not a petastorm dataset (no {'_common_metadata'}); "
                             "use make_batch_reader for plain Parquet")
        self.batched = batched
        groups = _row_groups(self.path)
        if shard_count is not None:
            if cur_shard is None or not 0 <= cur_shard < shard_count:
                raise ValueError("cur_shard must be in [0, shard_count)")
            groups = [g for i, g in enumerate(groups) if i % shard_count == cur_shard]
        self.groups = groups
        if schema_fields is not None:
            names = [f if isinstance(f, str) else f.name for f in schema_fields]
        elif self.schema is not None:
            names = list(self.schema.fields)
        else:
            names = pq.ParquetFile(str(groups[0][0])).schema_arrow.names if groups else []
        self.fields = names
        self.predicate = predicate
        self.num_epochs = num_epochs
        self.shuffle = shuffle_row_groups
        self.drop_parts = max(1, int(shuffle_row_drop_partitions))
        self.rng = random.Random(seed)
        self.pool = cf.ThreadPoolExecutor(max(1, workers_count)) if reader_pool_type in ("thread", "process") else None
        self._nt = collections.namedtuple("schema_view", self.fields)
        self._it = None
        self.last_row_consumed = False

    # -- decoding
    def _decode_group(self, item):
        f, g, part = item
        read_cols = list(dict.fromkeys(self.fields + (sorted(self.predicate.get_fields()) if self.predicate else [])))
        tbl = pq.ParquetFile(str(f)).read_row_group(g, columns=read_cols)
        cols = {c: tbl.column(c).to_pylist() for c in read_cols}
        n = tbl.num_rows
        idx = range(part, n, self.drop_parts)
        if self.batched:
            out = {c: np.asarray([cols[c][i] for i in idx]) for c in self.fields}
            return [self._nt(**out)]
        rows = []
        for i in idx:
            vals = {}
            for c in read_cols:
                v = cols[c][i]
                fld = self.schema.fields.get(c) if self.schema else None
                vals[c] = fld.codec.decode(fld, v) if (fld is not None and fld.codec is not None and v is not None) \
                    else v
            if self.predicate is not None and not self.predicate.do_include(vals):
                continue
            rows.append(self._nt(**{c: vals[c] for c in self.fields}))
        return rows

    def _work(self):
        epoch = 0
        while self.num_epochs is None or epoch < self.num_epochs:
            items = [(f, g, p) for f, g in self.groups for p in range(self.drop_parts)]
            if self.shuffle:
                self.rng.shuffle(items)
            yield from items
            epoch += 1

    def _iter(self):
        work = self._work()
        if self.pool is None:
            for it in work:
                yield from self._decode_group(it)
            return
        pending = collections.deque()
        depth = 8
        for it in work:
            pending.append(self.pool.submit(self._decode_group, it))
            if len(pending) >= depth:
                yield from pending.popleft().result()
        while pending:
            yield from pending.popleft().result()

    def __iter__(self):
        return self

    def __next__(self):
        if self._it is None:
            self._it = self._iter()
        try:
            return next(self._it)
        except StopIteration:
            self.last_row_consumed = True
            raise

    def reset(self):
        self._it = None
        self.last_row_consumed = False

    def stop(self):
        if self.pool is not None:
            self.pool.shutdown(wait=False, cancel_futures=True)

    def join(self):
        pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.stop()
        self.join()


def make_reader(dataset_url, schema_fields=None, reader_pool_type="thread", workers_count=10, pyarrow_serialize=False,
                results_queue_size=50, shuffle_row_groups=True, shuffle_row_drop_partitions=1, predicate=None,
                rowgroup_selector=None, num_epochs=1, cur_shard=None, shard_count=None, cache_type="null",
                seed=None, hdfs_driver=None, **kw) -> Reader:
    return Reader(dataset_url, schema_fields, reader_pool_type, workers_count, shard_count, cur_shard, predicate,
                  num_epochs, shuffle_row_groups, shuffle_row_drop_partitions, seed)


def make_batch_reader(dataset_url, schema_fields=None, reader_pool_type="thread", workers_count=10,
                      shuffle_row_groups=True, shuffle_row_drop_partitions=1, predicate=None, num_epochs=1,
                      cur_shard=None, shard_count=None, seed=None, hdfs_driver=None, **kw) -> Reader:
    return Reader(dataset_url, schema_fields, reader_pool_type, workers_count, shard_count, cur_shard, None,
                  num_epochs, shuffle_row_groups, shuffle_row_drop_partitions, seed, batched=True)
