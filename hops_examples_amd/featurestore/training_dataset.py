"""Training datasets: materialised, split, versioned feature sets + model input pipelines.

Reference: hsfs/basics/training_datasets.ipynb (formats :125-340, splits :187-193,
query replay :375-376, read split :395-401, ``tf_data(...).tf_record_dataset(process=True,
batch_size=32)`` -> ((32, 14), (32,)) float32 batches :429-447), coalesce
(hsfs/training/training-data-coalesced.ipynb:58-64), online serving vectors
(hsfs/serving/feature_vector_model_serving.ipynb:151-254).

Formats: csv, tsv, parquet, tfrecord (tf.train.Example rows encoded by the C++ IO library from
whole columns), npy, orc (pyarrow.orc), avro (object container files, avro.py), petastorm (Parquet
+ the inferred Unischema in ``_common_metadata``, readable by the petastorm readers); hdf5 needs
h5py, which this image lacks, and is refused at creation rather than silently written as Parquet.  Model input: ``tf_data``
yields numpy batches with the TF API's shapes; ``torch_data`` streams batches
into HBM through pinned host buffers on a side stream (DeviceLoader).
"""
from __future__ import annotations

import json
import random
import shutil
from pathlib import Path

import numpy as np
import torch
import pandas as pd

from .builders import CamelCaseAPI
from .. import io as hio
from . import statistics as ST

FORMATS = {"csv", "tsv", "parquet", "tfrecord", "tfrecords", "npy", "hdf5", "avro", "orc", "petastorm"}
SUPPORTED_TF_TYPES = ("string", "short", "int", "long", "float", "double", "bigint", "boolean")


class TrainingDatasetFeature:
    def __init__(self, name, type, index, label=False):
        self.name, self.type, self.index, self.label = name, type, index, label

    def __repr__(self):
        return f"TrainingDatasetFeature({self.name!r}, {self.type!r})"


class TrainingDataset(CamelCaseAPI):
    row_group_rows = 65536  # Parquet row-group size: the data-parallel shard unit of to_device
    ENTITY_TYPE = "trainingdatasets"

    def __init__(self, fs, name, version, description="", data_format="tfrecords", coalesce=False,
                 storage_connector=None, splits=None, location="", seed=None, statistics_config=None, label=None,
                 meta=None):
        self._fs = fs
        self.name, self.version = name, int(version)
        self.description = description or ""
        fmt = (data_format or "tfrecords").lower()
        if fmt not in FORMATS:
            raise ValueError(f"unsupported data format {data_format}")
        if fmt == "hdf5":
            try:
                import h5py  # noqa: F401
            except ImportError as e:
                raise ValueError("hdf5 training datasets need h5py, which is not installed") from e
            raise ValueError("hdf5 training datasets are not supported by this feature store")
        self.data_format = "tfrecord" if fmt == "tfrecords" else fmt
        self.coalesce = coalesce
        self.storage_connector = storage_connector
        self.splits = dict(splits or {})
        self.seed = seed
        self.label = [label] if isinstance(label, str) else list(label or [])
        self.statistics_config = ST.StatisticsConfig.parse(statistics_config)
        self._meta = meta or {"tags": {}}
        self._query_sql = self._meta.get("query")
        self._query_obj = None
        self._schema = [TrainingDatasetFeature(**f) for f in self._meta.get("schema", [])]
        self.id = self._meta.get("id")
        self._prepared = None
        if location:
            self._location = Path(location)
        elif storage_connector is not None and getattr(storage_connector, "path", None):
            self._location = Path(storage_connector.path) / f"{name}_{self.version}"
        else:
            self._location = fs._td_root / f"{name}_{self.version}"

    # --------------------------------------------------------------- metadata
    @property
    def location(self):
        return str(self._location)

    @property
    def schema(self):
        return self._schema

    @property
    def query(self):
        return self._query_sql

    @property
    def label_features(self):
        return self.label

    def _persist(self):
        self._meta.update({"name": self.name, "version": self.version, "description": self.description,
                           "data_format": self.data_format, "coalesce": self.coalesce, "splits": self.splits,
                           "seed": self.seed, "label": self.label, "location": str(self._location),
                           "statistics_config": self.statistics_config.to_dict(), "query": self._query_sql,
                           "schema": [f.__dict__ for f in self._schema],
                           "storage_connector": getattr(self.storage_connector, "name", None)})
        self._fs._write_meta(self.ENTITY_TYPE, f"{self.name}_{self.version}", self._meta)

    # --------------------------------------------------------------- write
    def save(self, features, write_options: dict | None = None):
        from .core import Query, _hsfs_type, _to_pandas

        if isinstance(features, Query):
            self._query_obj = features
            self._query_sql = features.to_string()
            self._meta["query_fgs"] = [[fg.name, fg.version] for fg in features._fgs()]
            df = features.read()
        else:
            df = _to_pandas(features)
        if self.id is None:
            self.id = self._fs._next_id()
            self._meta["id"] = self.id
        self._schema = [TrainingDatasetFeature(c, _hsfs_type(df[c].dtype), i, c in self.label)
                        for i, c in enumerate(df.columns)]
        if self._location.exists():
            shutil.rmtree(self._location)
        self._location.mkdir(parents=True)
        parts = self._split(df)
        self._wopts = dict(write_options or {})
        for split, part in parts.items():
            self._write_split(part.reset_index(drop=True), split)
        if self.data_format == "petastorm":
            self._write_unischema(df)
        if self.statistics_config.enabled:
            try:
                (self._location / "statistics.json").write_text(
                    json.dumps(ST.compute(df, self.statistics_config), default=float))
            except Exception:
                pass
        self._persist()
        return self

    def insert(self, features, overwrite: bool = True, write_options=None):
        return self.save(features, write_options)

    def _split(self, df: pd.DataFrame) -> dict:
        if not self.splits:
            return {"": df}
        names = list(self.splits)
        w = np.asarray([float(self.splits[n]) for n in names])
        w = w / w.sum()
        rng = np.random.default_rng(self.seed if self.seed is not None else random.randrange(1 << 30))
        u = rng.random(len(df))
        edges = np.cumsum(w)
        which = np.searchsorted(edges, u, side="right").clip(0, len(names) - 1)
        return {n: df[which == i] for i, n in enumerate(names)}

    def _split_dir(self, split: str) -> Path:
        return self._location / split if split else self._location

    def _write_split(self, df: pd.DataFrame, split: str):
        d = self._split_dir(split)
        d.mkdir(parents=True, exist_ok=True)
        fmt = self.data_format
        wo = getattr(self, "_wopts", {})
        part_rows = int(wo.get("part_rows", 200_000))
        nparts = 1 if self.coalesce or len(df) < part_rows else max(1, len(df) // part_rows)
        chunks = np.array_split(np.arange(len(df)), nparts) if len(df) else [np.arange(0)]
        for i, idx in enumerate(chunks):
            part = df.iloc[idx]
            base = d / f"part-{i:05d}"
            if fmt in ("csv", "tsv"):
                part.to_csv(f"{base}.{fmt}", index=False, sep="," if fmt == "csv" else "\t")
            elif fmt == "tfrecord":
                # whole columns to the native writer: rows encoded + framed by C++ threads
                cols = []
                for c in part.columns:
                    k = part[c].dtype.kind
                    if k in "iub":
                        cols.append((c, "int64", part[c].to_numpy(np.int64)))
                    elif k == "f":
                        cols.append((c, "float", part[c].to_numpy(np.float32)))
                    else:
                        cols.append((c, "bytes", [str(v).encode() for v in part[c].tolist()]))
                hio.write_tfrecord_columns(f"{base}.tfrecord", cols, len(part))
            elif fmt == "npy":
                np.save(f"{base}.npy", part.to_records(index=False), allow_pickle=False)
            elif fmt == "orc":
                import pyarrow as pa
                import pyarrow.orc as paorc

                paorc.write_table(pa.Table.from_pandas(part, preserve_index=False), f"{base}.orc")
            elif fmt == "avro":
                from .. import avro

                avro.write_container(f"{base}.avro", avro.schema_of_frame(part, self.name),
                                     part.to_dict(orient="records"))
            elif fmt in ("parquet", "petastorm"):
                # petastorm datasets ARE Parquet (+ the Unischema in _common_metadata, written in save());
                # 64k-row row groups: the unit data-parallel readers shard by (to_device(shard=...))
                # write_options: row_group_size / compression / use_dictionary (a PLAIN, uncompressed
                # TD is one memcpy per column chunk for the native reader: io/parquet.py)
                part.to_parquet(f"{base}.parquet", index=False,
                                row_group_size=int(wo.get("row_group_size", self.row_group_rows)),
                                compression=wo.get("compression", "snappy"),
                                use_dictionary=bool(wo.get("use_dictionary", True)))
            else:
                raise ValueError(f"training dataset format {fmt!r} is not supported here")

    def _write_unischema(self, df: pd.DataFrame) -> None:
        """petastorm metadata: a Unischema of scalar fields (dtype from the frame) in every split's
        ``_common_metadata``, so ``petastorm.make_reader(td.location)`` can open the dataset."""
        from ..petastorm.codecs import ScalarCodec
        from ..petastorm.etl.dataset_metadata import META
        from ..petastorm.unischema import Unischema, UnischemaField

        fields = []
        for c in df.columns:
            k = df[c].dtype.kind
            dt = (np.int64 if k in "iu" else np.float64 if k == "f" else np.bool_ if k == "b" else np.str_)
            fields.append(UnischemaField(str(c), dt, (), ScalarCodec(), bool(df[c].isna().any())))
        js = json.dumps({"unischema": Unischema(self.name, fields).to_json(), "row_group_size_mb": None})
        for split in (self.splits or {"": None}):
            (self._split_dir(split) / META).write_text(js)

    # --------------------------------------------------------------- read
    def _files(self, split: str | None):
        d = self._split_dir(split or "")
        if split is None and self.splits:
            return sorted(p for s in self.splits for p in self._split_dir(s).glob("part-*"))
        return sorted(d.glob("part-*"))

    def read(self, split: str | None = None, read_options=None) -> pd.DataFrame:
        if split is not None and split not in self.splits:
            raise ValueError(f"split {split!r} not in {list(self.splits)}")
        frames = []
        cols = [f.name for f in self._schema]
        for p in self._files(split):
            if p.suffix in (".csv", ".tsv"):
                frames.append(pd.read_csv(p, sep="," if p.suffix == ".csv" else "\t"))
            elif p.suffix == ".parquet":
                frames.append(pd.read_parquet(p))
            elif p.suffix == ".npy":
                frames.append(pd.DataFrame(np.load(p, allow_pickle=False)))
            elif p.suffix == ".tfrecord":
                frames.append(self._read_tfrecord(p))
            elif p.suffix == ".orc":
                import pyarrow.orc as paorc

                frames.append(paorc.read_table(str(p)).to_pandas())
            elif p.suffix == ".avro":
                from .. import avro

                frames.append(pd.DataFrame(avro.read_container(str(p))[1]))
        if not frames:
            return pd.DataFrame(columns=cols)
        return pd.concat(frames, ignore_index=True)

    def _read_tfrecord(self, p: Path) -> pd.DataFrame:
        recs = hio.read_tfrecords(str(p))
        num = [(f.name, "float" if f.type in ("float", "double") else "int64", 1) for f in self._schema
               if f.type not in ("string", "timestamp")]
        cols = hio.decode_batch(recs, num) if num else {}
        out = {}
        for f in self._schema:
            if f.name in cols:
                a = cols[f.name][:, 0]
                out[f.name] = a.astype(np.float64) if f.type == "double" else a
            else:
                out[f.name] = [hio.decode_example(r)[f.name][0].decode() for r in recs]
        return pd.DataFrame(out)

    def show(self, n: int = 20, split: str | None = None):
        from .core import _spark_show

        _spark_show(self.read(split), n)

    # --------------------------------------------------------------- model input
    def tf_data(self, target_name: str, split: str | None = None, feature_names=None, var_len_features=None,
                is_training: bool = True, cycle_length: int = 2):
        return TFDataEngine(self, target_name, split, feature_names, is_training)

    def torch_data(self, target_name: str, split: str | None = None, batch_size: int = 32, shuffle: bool = True,
                   drop_last: bool = True, device=None, feature_names=None, shard=None):
        from ..io.loader import DeviceLoader

        if self._parquet_parts(split) and (device is None or torch.device(device).type == "cuda") \
                and torch.cuda.is_available():
            x, y = self.to_device(target_name, split, feature_names=feature_names, device=device, shard=shard)
            return DeviceLoader.from_tensors(x, y, batch_size, shuffle=shuffle, drop_last=drop_last, seed=self.seed)
        x, y = _xy(self.read(split), target_name, feature_names)
        return DeviceLoader(x, y, batch_size, shuffle=shuffle, drop_last=drop_last, device=device, shard=shard,
                            seed=self.seed)

    def _parquet_parts(self, split):
        files = self._files(split)
        return files if files and all(p.suffix == ".parquet" for p in files) else None

    def to_device(self, target_name: str, split: str | None = None, feature_names=None, device=None, shard=None):
        """(features fp32 [n, k], target fp32 [n]) resident in HBM.  Parquet parts stream through
        io.parquet.ParquetDeviceReader (Arrow decode -> pinned staging -> side-stream H2D -> fp32
        conversion on the GPU); other formats go through ``read()``.

        ``shard=(n, i)``: rank i of n gets an EQUAL number of rows (data-parallel ranks must run the
        same number of steps).  Row-group sharding (petastorm's ``shard_count`` / ``cur_shard``: every
        n-th row group of the whole dataset, only those are read) when every shard gets at least half
        the rows of the largest; else — e.g. a small dataset written as ONE row group — every rank reads all rows
        and keeps rows i, i+n, ... (the DeviceLoader rule).  Either way each shard is truncated to
        the smallest shard's row count, computed from the Parquet metadata on every rank alike."""
        from ..io.parquet import ParquetDeviceReader

        targets = [target_name] if isinstance(target_name, str) else list(target_name)
        names = [f.name for f in self._schema]
        feats = feature_names or [c for c in names if c not in targets]
        parts = self._parquet_parts(split)
        if parts is None:
            x, y = _xy(self.read(split), target_name, feature_names)
            dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
            x, y = torch.from_numpy(x).to(dev), torch.from_numpy(y).to(dev)
            if shard is not None:
                n, i = shard
                m = x.shape[0] // n
                x, y = x[i::n][:m].contiguous(), y[i::n][:m].contiguous()
            return x, y
        row_sharded = False
        picks = None  # per part: the row groups this rank reads
        keep = None
        if shard is not None:
            import pyarrow.parquet as pq

            n, i = shard
            # dataset-wide row-group sharding: global row group j (over all parts in order) goes to
            # rank j % n, so parts with few row groups still spread over every rank
            sizes = []
            for p in parts:  # the footer of each part is read once
                md = pq.ParquetFile(str(p)).metadata
                sizes.append([md.row_group(g).num_rows for g in range(md.num_row_groups)])
            per, mine, j = [0] * n, [[] for _ in parts], 0
            for pi, rgs in enumerate(sizes):
                for g, rows in enumerate(rgs):
                    per[j % n] += rows
                    if j % n == i:
                        mine[pi].append(g)
                    j += 1
            # equal shards by truncation must not silently drop data: with more than one row group's
            # worth of rows lost (e.g. 3 groups over 2 ranks), shard by rows instead (petastorm's
            # cur_shard reads every row group and never truncates)
            biggest = max((r for rgs in sizes for r in rgs), default=0)
            if min(per) == 0 or sum(per) - n * min(per) > biggest:
                row_sharded = True
            else:
                picks, keep = mine, min(per)
        self.last_shard_dropped = 0 if shard is None or row_sharded else sum(per) - n * keep
        self.last_shard_mode = None if shard is None else ("rows" if row_sharded else "row_groups")
        # every part through ONE reader pipeline (decode pool, pinned ring, one convert per row group)
        rd = ParquetDeviceReader([str(p) for p in parts], feats + targets, device=device, row_groups=picks)
        total = rd.rows
        out = torch.empty(total, len(feats) + len(targets), dtype=torch.float32, device=rd.device)
        rd.read(out)
        self.last_read_bytes = rd.bytes_read
        if row_sharded:
            n, i = shard
            out = out[i::n][:total // n]
        elif keep is not None:
            out = out[:keep]
        y = out[:, len(feats):]
        return out[:, :len(feats)].contiguous(), (y[:, 0].contiguous() if len(targets) == 1 else y.contiguous())

    # --------------------------------------------------------------- online serving
    def init_prepared_statement(self, batch: bool | None = None, external: bool | None = None):
        q = self._query_obj
        if q is None:
            q = self._fs._rebuild_query(self)
        self._prepared = self._fs._online.prepare(q, exclude=set(self.label))

    @property
    def serving_keys(self) -> set:
        if self._prepared is None:
            self.init_prepared_statement()
        return set(self._prepared["keys"])

    def get_serving_vector(self, entry: dict, external=None) -> list:
        if self._prepared is None:
            self.init_prepared_statement()
        return self._fs._online.vector(self._prepared, entry)

    def get_serving_vectors(self, entry: dict) -> list:
        keys = list(entry)
        n = len(entry[keys[0]])
        return [self.get_serving_vector({k: entry[k][i] for k in keys}) for i in range(n)]

    # --------------------------------------------------------------- tags/statistics
    def add_tag(self, name, value):
        self._fs._tags.check(name, value)
        self._meta.setdefault("tags", {})[name] = value
        self._persist()

    def get_tag(self, name):
        return self._meta.get("tags", {}).get(name)

    def get_tags(self):
        return dict(self._meta.get("tags", {}))

    def delete_tag(self, name):
        self._meta.get("tags", {}).pop(name, None)
        self._persist()

    def get_statistics(self):
        p = self._location / "statistics.json"
        return json.loads(p.read_text()) if p.exists() else ST.compute(self.read(), self.statistics_config)

    def delete(self):
        shutil.rmtree(self._location, ignore_errors=True)
        self._fs._delete_meta(self.ENTITY_TYPE, f"{self.name}_{self.version}")

    def __repr__(self):
        return f"TrainingDataset({self.name!r}, {self.version}, format={self.data_format!r}, splits={self.splits})"


def _xy(df: pd.DataFrame, target_name, feature_names=None):
    targets = [target_name] if isinstance(target_name, str) else list(target_name)
    feats = feature_names or [c for c in df.columns if c not in targets]
    for c in feats:
        if not pd.api.types.is_numeric_dtype(df[c]):
            raise TypeError(f"feature {c!r} is not numeric (supported: {SUPPORTED_TF_TYPES})")
    x = df[feats].to_numpy(np.float32)
    y = df[targets].to_numpy(np.float32)
    return x, (y[:, 0] if len(targets) == 1 else y)


class TFDataEngine:
    """``td.tf_data(target_name, split)`` — numpy batch pipelines with the TF API's shapes."""

    def __init__(self, td, target_name, split, feature_names, is_training):
        self.td, self.target, self.split, self.feature_names, self.is_training = td, target_name, split, \
            feature_names, is_training

    def _batches(self, batch_size, num_epochs, process):
        x, y = _xy(self.td.read(self.split), self.target, self.feature_names)
        rng = np.random.default_rng(self.td.seed)
        epochs = num_epochs if num_epochs is not None else (None if self.is_training else 1)
        e = 0
        while epochs is None or e < epochs:
            idx = rng.permutation(len(x)) if self.is_training else np.arange(len(x))
            bs = batch_size or len(x)
            stop = len(x) - (len(x) % bs if self.is_training else 0)
            for s in range(0, stop, bs):
                b = idx[s:s + bs]
                yield (x[b], y[b]) if process else ({n: x[b, i] for i, n in enumerate(self._names(x))}, y[b])
            e += 1

    def _names(self, x):
        df_cols = [f.name for f in self.td.schema if f.name != self.target]
        return self.feature_names or df_cols

    def tf_record_dataset(self, batch_size: int | None = None, num_epochs: int | None = None,
                          one_hot_encode_labels: bool = False, num_classes: int | None = None,
                          process: bool = False, serialized_ndarray_fname=None):
        return _Dataset(lambda: self._batches(batch_size, num_epochs if num_epochs is not None else 1, process))

    def tf_csv_dataset(self, batch_size: int | None = None, num_epochs: int | None = None,
                       one_hot_encode_labels: bool = False, num_classes: int | None = None, process: bool = False):
        return self.tf_record_dataset(batch_size, num_epochs, one_hot_encode_labels, num_classes, process)


class _Dataset:
    def __init__(self, gen):
        self._gen = gen

    def __iter__(self):
        return self._gen()

    def take(self, n):
        def g():
            for i, b in enumerate(self._gen()):
                if i >= n:
                    return
                yield b

        return _Dataset(g)

    @property
    def element_spec(self):
        x, y = next(iter(self._gen()))
        return ((x.shape, x.dtype), (y.shape, y.dtype))
