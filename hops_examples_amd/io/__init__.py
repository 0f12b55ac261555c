"""Data path: TFRecord / tf.train.Example / CSV codecs (C++ ``_hopsx_io`` with a
pure-Python fallback), sharded readers and the pinned-memory -> HBM loader.

The reference feeds models through ``tf.data.TFRecordDataset`` + Example parsing
(mirroredstrategy_mnist_example.ipynb:153-186), CSV datasets and petastorm
(PetastormHelloWorld.ipynb).  Here a dataset is decoded columnar on the host by
C++ threads and streamed to HBM by :class:`DeviceLoader`.
"""
from __future__ import annotations

import importlib
import struct

import numpy as np

try:
    _io = importlib.import_module("hops_examples_amd._hopsx_io")
except Exception:  # pragma: no cover - fallback when the extension is not built
    _io = None

NATIVE = _io is not None


# ------------------------------------------------------------------ crc32c
def _crc_table():
    t = []
    for i in range(256):
        c = i
        for _ in range(8):
            c = (c >> 1) ^ 0x82F63B78 if c & 1 else c >> 1
        t.append(c)
    return t


_TABLE = None


def crc32c(data: bytes) -> int:
    if _io is not None:
        return _io.crc32c(data)
    global _TABLE
    if _TABLE is None:
        _TABLE = _crc_table()
    c = 0xFFFFFFFF
    for b in data:
        c = _TABLE[(c ^ b) & 0xFF] ^ (c >> 8)
    return c ^ 0xFFFFFFFF


def masked_crc32c(data: bytes) -> int:
    c = crc32c(data)
    return (((c >> 15) | (c << 17)) + 0xA282EAD8) & 0xFFFFFFFF


# ---------------------------------------------------------------- TFRecord
class TFRecordWriter:
    def __init__(self, path: str, append: bool = False):
        self._native = _io.TFRecordWriter(str(path), append) if _io is not None else None
        self._f = None if self._native else open(path, "ab" if append else "wb")

    def write(self, record: bytes) -> None:
        if self._native is not None:
            self._native.write(record)
            return
        hdr = struct.pack("<Q", len(record))
        self._f.write(hdr + struct.pack("<I", masked_crc32c(hdr)) + record + struct.pack("<I", masked_crc32c(record)))

    def flush(self):
        (self._native or self._f).flush()

    def close(self):
        (self._native or self._f).close()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


def write_tfrecord_columns(path: str, columns: list, n: int, nthreads: int = 8) -> int:
    """One tf.train.Example per row from whole columns: ``columns`` = [(name, 'float'|'int64'|'bytes',
    values)], every column with ``n`` values.  Native (multi-threaded encode, one write) when the IO
    extension is built; returns the bytes written."""
    if _io is not None:
        return int(_io.write_tfrecord_columnar(str(path), [(c, k, v) for c, k, v in columns], int(n), nthreads))
    total = 0
    with TFRecordWriter(path) as w:
        for r in range(n):
            rec = encode_example({c: (k, [v[r]] if k == "bytes" else np.asarray([v[r]])) for c, k, v in columns})
            w.write(rec)
            total += len(rec) + 16
    return total


def read_tfrecords(path: str, verify: bool = True) -> list[bytes]:
    if _io is not None:
        return _io.read_tfrecords(str(path), verify)
    out = []
    with open(path, "rb") as f:
        buf = f.read()
    pos = 0
    while pos + 12 <= len(buf):
        (n,) = struct.unpack_from("<Q", buf, pos)
        if verify and struct.unpack_from("<I", buf, pos + 8)[0] != masked_crc32c(buf[pos:pos + 8]):
            raise IOError("TFRecord length crc mismatch")
        rec = buf[pos + 12:pos + 12 + n]
        if verify and struct.unpack_from("<I", buf, pos + 12 + n)[0] != masked_crc32c(rec):
            raise IOError("TFRecord data crc mismatch")
        out.append(bytes(rec))
        pos += 12 + n + 4
    return out


# -------------------------------------------------------- tf.train.Example
def _varint(v: int) -> bytes:
    out = bytearray()
    v &= (1 << 64) - 1
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def _ld(field: int, payload: bytes) -> bytes:
    return _varint((field << 3) | 2) + _varint(len(payload)) + payload


def _infer(v):
    if isinstance(v, (bytes, str)):
        return "bytes", [v]
    a = np.asarray(v)
    if a.dtype.kind in "SUO":
        return "bytes", [x if isinstance(x, bytes) else str(x).encode() for x in a.reshape(-1)]
    if a.dtype.kind in "iub":
        return "int64", a.reshape(-1).astype(np.int64)
    return "float", a.reshape(-1).astype(np.float32)


def encode_example(features: dict) -> bytes:
    """features: {name: value | (kind, values)} -> serialized tf.train.Example."""
    norm = {}
    for k, v in features.items():
        norm[k] = v if (isinstance(v, tuple) and len(v) == 2 and v[0] in ("float", "int64", "bytes")) else _infer(v)
    if _io is not None:
        return _io.encode_example(norm)
    fs = b""
    for name, (kind, vals) in norm.items():
        if kind == "float":
            lst = _ld(1, np.asarray(vals, dtype="<f4").tobytes())
            feat = _ld(2, lst)
        elif kind == "int64":
            lst = _ld(1, b"".join(_varint(int(x)) for x in np.asarray(vals).reshape(-1)))
            feat = _ld(3, lst)
        else:
            lst = b"".join(_ld(1, x if isinstance(x, bytes) else str(x).encode()) for x in vals)
            feat = _ld(1, lst)
        fs += _ld(1, _ld(1, name.encode()) + _ld(2, feat))
    return _ld(1, fs)


def decode_example(rec: bytes) -> dict:
    if _io is None:
        raise RuntimeError("decode_example requires the native _hopsx_io extension")
    return {k: v[1] for k, v in _io.decode_example(rec).items()}


def decode_batch(records: list[bytes], schema: list[tuple[str, str, int]], nthreads: int = 8) -> dict:
    """Columnar decode of many Examples: schema [(name, 'float'|'int64'|'bytes', length)] ->
    {name: ndarray[n, length]} ('bytes': the first value of the feature, exactly ``length`` bytes, as
    uint8 — a raw image)."""
    if _io is not None:
        return _io.decode_examples_columnar(records, schema, nthreads)
    out = {n: np.zeros((len(records), L), np.float32 if k == "float" else np.int64) for n, k, L in schema}
    for i, r in enumerate(records):
        d = decode_example(r)
        for n, k, L in schema:
            v = np.asarray(d.get(n, []))[:L]
            out[n][i, :len(v)] = v
    return out


# --------------------------------------------------------------------- CSV
def read_csv_numeric(path: str, delimiter: str = ",", header: bool = True):
    """(column_names, float32 matrix); empty / non-numeric cells are NaN."""
    if _io is not None:
        names, arr = _io.parse_csv_numeric(str(path), delimiter, header)
        return list(names), arr
    import pandas as pd

    df = pd.read_csv(path, sep=delimiter, header=0 if header else None)
    return [str(c) for c in df.columns], df.apply(pd.to_numeric, errors="coerce").to_numpy(np.float32)


def gather_rows(src: np.ndarray, idx: np.ndarray, dst: np.ndarray, nthreads: int = 8) -> np.ndarray:
    """dst[i] = src[idx[i]] (C++ thread pool; used to assemble shuffled batches into pinned buffers)."""
    if _io is not None and src.flags.c_contiguous and dst.flags.c_contiguous:
        _io.gather_rows(src, np.ascontiguousarray(idx, dtype=np.int64), dst, nthreads)
    else:
        np.take(src, idx, axis=0, out=dst[: len(idx)])
    return dst
