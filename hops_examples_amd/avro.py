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
