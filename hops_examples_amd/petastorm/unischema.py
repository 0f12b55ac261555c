"""Unischema: a dataset schema whose fields carry numpy dtype, shape and storage codec."""
from __future__ import annotations

import collections
import json

import numpy as np

from . import codecs as C

UnischemaField = collections.namedtuple("UnischemaField", ["name", "numpy_dtype", "shape", "codec", "nullable"])
UnischemaField.__new__.__defaults__ = (None, False)


def _shape_ok(field, a) -> bool:
    if field.shape is None or not isinstance(a, np.ndarray):
        return True
    return a.ndim == len(field.shape) and all(d is None or d == s for d, s in zip(field.shape, a.shape))


class Unischema:
    def __init__(self, name: str, fields):
        self._name = name
        self._fields = collections.OrderedDict((f.name, f) for f in fields)
        for f in fields:
            setattr(self, f.name, f)
        self._nt = collections.namedtuple(f"{name}_view", list(self._fields))

    @property
    def fields(self):
        return self._fields

    def create_schema_view(self, fields) -> "Unischema":
        names = [f if isinstance(f, str) else f.name for f in fields]
        return Unischema(f"{self._name}_view", [self._fields[n] for n in names])

    def make_namedtuple(self, **kw):
        return self._nt(**kw)

    def as_spark_schema(self):
        """Storage schema (pyarrow): scalar codecs -> native columns, others -> binary."""
        import pyarrow as pa

        cols = []
        for f in self._fields.values():
            t = (f.codec or C.ScalarCodec()).arrow_type(f)
            cols.append(pa.field(f.name, pa.type_for_alias(t), nullable=f.nullable))
        return pa.schema(cols)

    as_arrow_schema = as_spark_schema

    def to_json(self) -> str:
        return json.dumps({"name": self._name, "fields": [
            {"name": f.name, "dtype": np.dtype(f.numpy_dtype).str if f.numpy_dtype not in (np.str_, str) else "str",
             "shape": list(f.shape) if f.shape is not None else None, "codec": repr(f.codec),
             "codec_args": _codec_args(f.codec), "nullable": f.nullable} for f in self._fields.values()]})

    @staticmethod
    def from_json(s: str) -> "Unischema":
        d = json.loads(s)
        fields = []
        for f in d["fields"]:
            dt = np.str_ if f["dtype"] == "str" else np.dtype(f["dtype"]).type
            fields.append(UnischemaField(f["name"], dt, tuple(f["shape"]) if f["shape"] is not None else None,
                                         _codec_from(f["codec"], f["codec_args"]), f["nullable"]))
        return Unischema(d["name"], fields)

    def __repr__(self):
        return f"Unischema({self._name}, [{', '.join(self._fields)}])"


def _codec_args(c):
    if isinstance(c, C.CompressedImageCodec):
        return {"image_codec": c.image_codec, "quality": c.quality}
    if isinstance(c, C.ScalarCodec) and c.spark_type is not None:
        return {"type": type(c.spark_type).__name__}
    return {}


def _codec_from(r: str, args: dict):
    from . import types as T

    if r.startswith("CompressedImageCodec"):
        return C.CompressedImageCodec(args["image_codec"], args["quality"])
    if r.startswith("CompressedNdarrayCodec"):
        return C.CompressedNdarrayCodec()
    if r.startswith("NdarrayCodec"):
        return C.NdarrayCodec()
    return C.ScalarCodec(getattr(T, args["type"])() if args.get("type") else None)


def dict_to_spark_row(schema: Unischema, row: dict) -> dict:
    """Validate and encode one row (dict of field -> value) into its storage form."""
    if set(row) != set(schema.fields):
        raise ValueError(f"row fields {sorted(row)} do not match schema fields {sorted(schema.fields)}")
    out = {}
    for name, f in schema.fields.items():
        v = row[name]
        if v is None:
            if not f.nullable:
                raise ValueError(f"field {name} is not nullable")
            out[name] = None
            continue
        if isinstance(v, np.ndarray) and not _shape_ok(f, v):
            raise ValueError(f"field {name}: shape {v.shape} does not match {f.shape}")
        out[name] = (f.codec or C.ScalarCodec()).encode(f, v)
    return out


def encode_row(schema: Unischema, row: dict) -> dict:
    return dict_to_spark_row(schema, row)
