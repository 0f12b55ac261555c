"""Avro binary encoding for record schemas (the Kafka payload format of the reference:
``to_avro`` / ``from_avro(Hops.getSchema(topic))`` in
spark/src/main/scala/io/hops/examples/spark/kafka/StructuredStreamingKafka.scala:22-41 and
``parse_avro_msg`` in notebooks/kafka/KafkaPython.ipynb).

Supports null, boolean, int, long, float, double, bytes, string, enum, fixed, array, map,
record and unions — zig-zag varints, IEEE little-endian floats, length-prefixed bytes/strings,
block-encoded arrays/maps — i.e. the Avro 1.x binary spec, no code generation.
"""
from __future__ import annotations

import io
import json
import struct


def _schema(s):
    return json.loads(s) if isinstance(s, str) and s.strip().startswith(("{", "[", '"')) else s


def _zz(n: int) -> int:
    return (n << 1) ^ (n >> 63)


def _write_long(out, n: int):
    n = _zz(n) & ((1 << 64) - 1)
    while n & ~0x7F:
        out.write(bytes(((n & 0x7F) | 0x80,)))
        n >>= 7
    out.write(bytes((n,)))


def _read_long(inp) -> int:
    shift, acc = 0, 0
    while True:
        b = inp.read(1)[0]
        acc |= (b & 0x7F) << shift
        if not b & 0x80:
            break
        shift += 7
    return (acc >> 1) ^ -(acc & 1)


def _matches(s, v) -> bool:
    t = s if isinstance(s, str) else (s.get("type") if isinstance(s, dict) else "union")
    return {"null": v is None, "boolean": isinstance(v, bool), "int": isinstance(v, int) and not isinstance(v, bool),
            "long": isinstance(v, int) and not isinstance(v, bool), "float": isinstance(v, (int, float)),
            "double": isinstance(v, (int, float)), "string": isinstance(v, str),
            "bytes": isinstance(v, (bytes, bytearray)), "record": isinstance(v, dict), "map": isinstance(v, dict),
            "array": isinstance(v, (list, tuple)), "enum": isinstance(v, str),
            "fixed": isinstance(v, (bytes, bytearray))}.get(t, False)


def _enc(s, v, out):
    if isinstance(s, list):  # union
        for i, b in enumerate(s):
            if _matches(b, v):
                _write_long(out, i)
                return _enc(b, v, out)
        raise ValueError(f"value {v!r} matches no branch of union {s}")
    t = s if isinstance(s, str) else s["type"]
    if isinstance(t, (dict, list)):
        return _enc(t, v, out)
    if t == "null":
        return
    if t == "boolean":
        out.write(b"\x01" if v else b"\x00")
    elif t in ("int", "long"):
        _write_long(out, int(v))
    elif t == "float":
        out.write(struct.pack("<f", float(v)))
    elif t == "double":
        out.write(struct.pack("<d", float(v)))
    elif t in ("bytes", "string"):
        b = v.encode() if isinstance(v, str) else bytes(v)
        _write_long(out, len(b))
        out.write(b)
    elif t == "fixed":
        out.write(bytes(v))
    elif t == "enum":
        _write_long(out, s["symbols"].index(v))
    elif t == "array":
        if v:
            _write_long(out, len(v))
            for x in v:
                _enc(s["items"], x, out)
        _write_long(out, 0)
    elif t == "map":
        if v:
            _write_long(out, len(v))
            for k, x in v.items():
                _enc("string", k, out)
                _enc(s["values"], x, out)
        _write_long(out, 0)
    elif t == "record":
        for f in s["fields"]:
            val = v.get(f["name"], f.get("default"))
            _enc(f["type"], val, out)
    else:
        raise ValueError(f"unsupported avro type {t!r}")


def _dec(s, inp):
    if isinstance(s, list):
        return _dec(s[_read_long(inp)], inp)
    t = s if isinstance(s, str) else s["type"]
    if isinstance(t, (dict, list)):
        return _dec(t, inp)
    if t == "null":
        return None
    if t == "boolean":
        return inp.read(1) == b"\x01"
    if t in ("int", "long"):
        return _read_long(inp)
    if t == "float":
        return struct.unpack("<f", inp.read(4))[0]
    if t == "double":
        return struct.unpack("<d", inp.read(8))[0]
    if t in ("bytes", "string"):
        b = inp.read(_read_long(inp))
        return b.decode() if t == "string" else b
    if t == "fixed":
        return inp.read(s["size"])
    if t == "enum":
        return s["symbols"][_read_long(inp)]
    if t in ("array", "map"):
        out = [] if t == "array" else {}
        while True:
            n = _read_long(inp)
            if n == 0:
                return out
            if n < 0:
                n = -n
                _read_long(inp)  # block byte size
            for _ in range(n):
                if t == "array":
                    out.append(_dec(s["items"], inp))
                else:
                    k = _dec("string", inp)
                    out[k] = _dec(s["values"], inp)
    if t == "record":
        return {f["name"]: _dec(f["type"], inp) for f in s["fields"]}
    raise ValueError(f"unsupported avro type {t!r}")


def encode(schema, record) -> bytes:
    out = io.BytesIO()
    _enc(_schema(schema), record, out)
    return out.getvalue()


def decode(schema, data: bytes):
    return _dec(_schema(schema), io.BytesIO(data))


# ------------------------------------------------------------------ object container files
# Avro 1.x Object Container File: magic "Obj\x01", file metadata map {avro.schema, avro.codec},
# a 16-byte sync marker, then blocks of (record count, byte size, records, sync).  Used by the
# "avro" training-dataset format (notebooks/featurestore/hsfs/basics/training_datasets.ipynb:125-340).
_MAGIC = b"Obj\x01"


def _write_bytes(out, b: bytes):
    _write_long(out, len(b))
    out.write(b)


def _read_bytes(inp) -> bytes:
    return inp.read(_read_long(inp))


def schema_of_frame(df, name: str = "record") -> dict:
    """A record schema for a pandas frame: every field nullable (["null", type])."""
    fields = []
    for c in df.columns:
        k = df[c].dtype.kind
        t = "boolean" if k == "b" else ("long" if k in "iu" else ("double" if k == "f" else "string"))
        fields.append({"name": str(c), "type": ["null", t]})
    safe = "".join(ch if ch.isalnum() or ch == "_" else "_" for ch in str(name)) or "record"
    return {"type": "record", "name": safe, "fields": fields}


def _py(v):
    """numpy scalars -> Python values the encoder matches (NaT / None -> null)."""
    if v is None:
        return None
    if hasattr(v, "item"):
        v = v.item()
    if isinstance(v, float) and v != v:
        return v  # NaN is a valid double
    return v


def write_container(path, schema, records, block_records: int = 4096, sync: bytes | None = None) -> int:
    """Write ``records`` (dicts) as an Avro object container file; returns the record count."""
    import os

    sch = _schema(schema)
    sync = sync or os.urandom(16)
    kinds = {f["name"]: f["type"] for f in sch["fields"]}
    n = 0
    with open(path, "wb") as f:
        f.write(_MAGIC)
        meta = {"avro.schema": json.dumps(sch).encode(), "avro.codec": b"null"}
        _write_long(f, len(meta))
        for k, v in meta.items():
            _write_bytes(f, k.encode())
            _write_bytes(f, v)
        _write_long(f, 0)
        f.write(sync)
        block, cnt = io.BytesIO(), 0
        for rec in records:
            r = {k: _py(rec.get(k)) for k in kinds}
            for k, t in kinds.items():  # ints stored in a double column, strings for object values
                if isinstance(t, list) and "string" in t and r[k] is not None and not isinstance(r[k], str):
                    r[k] = str(r[k])
            _enc(sch, r, block)
            cnt += 1
            if cnt == block_records:
                _write_long(f, cnt)
                _write_bytes(f, block.getvalue())
                f.write(sync)
                n += cnt
                block, cnt = io.BytesIO(), 0
        if cnt:
            _write_long(f, cnt)
            _write_bytes(f, block.getvalue())
            f.write(sync)
            n += cnt
    return n


def read_container(path):
    """(schema, [records]) of an Avro object container file (null codec)."""
    with open(path, "rb") as f:
        buf = f.read()
    inp = io.BytesIO(buf)
    if inp.read(4) != _MAGIC:
        raise ValueError(f"{path}: not an Avro object container file")
    meta = {}
    while True:
        cnt = _read_long(inp)
        if cnt == 0:
            break
        if cnt < 0:
            _read_long(inp)
            cnt = -cnt
        for _ in range(cnt):
            k = _read_bytes(inp).decode()
            meta[k] = _read_bytes(inp)
    if meta.get("avro.codec", b"null") not in (b"null", b""):
        raise ValueError(f"{path}: codec {meta['avro.codec']!r} not supported")
    sch = json.loads(meta["avro.schema"])
    sync = inp.read(16)
    out = []
    while inp.tell() < len(buf):
        cnt = _read_long(inp)
        size = _read_long(inp)
        blk = io.BytesIO(inp.read(size))
        for _ in range(cnt):
            out.append(_dec(sch, blk))
        if inp.read(16) != sync:
            raise ValueError(f"{path}: sync marker mismatch")
    return sch, out
