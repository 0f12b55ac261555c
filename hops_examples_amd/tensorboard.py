"""TensorBoard integration (``hops.tensorboard``): per-run log directory and a
dependency-free event-file writer.

Reference: ``tensorboard.logdir()`` is the directory every experiment writes its
summaries / checkpoints into (notebooks/ml/Experiment/Tensorflow/mnist.ipynb:116,172;
…/Parallel_Experiments/TensorFlow/evolutionary_search/evolutionary_search_mnist.ipynb:265-266),
and PyTorch runs use ``SummaryWriter.add_scalar('Loss/train', …)``
(notebooks/ml/Experiment/PyTorch/mnist.ipynb:153,184).  Event files are standard
``events.out.tfevents.*`` TFRecord files readable by TensorBoard.
"""
from __future__ import annotations

import os
import socket
import struct
import time
from pathlib import Path

from . import config
from . import io as hio


def logdir() -> str:
    """The current experiment run's log directory (local if ``local_logdir=True``)."""
    d = os.environ.get("HOPSX_TB_LOGDIR") or os.environ.get("HOPSX_LOGDIR")
    if not d:
        d = str(config.get().project_root / "Logs" / "TensorBoard" / time.strftime("%Y%m%d-%H%M%S"))
    Path(d).mkdir(parents=True, exist_ok=True)
    return d


def interactive_debugger():  # pragma: no cover - API parity (tfdbg has no MI355X analogue)
    return logdir()


def non_interactive_debugger():  # pragma: no cover
    return logdir()


# --------------------------------------------------------- protobuf encoding
def _varint(v):
    return hio._varint(v)


def _field(num, wire):
    return _varint((num << 3) | wire)


def _double(num, v):
    return _field(num, 1) + struct.pack("<d", v)


def _float(num, v):
    return _field(num, 5) + struct.pack("<f", v)


def _int(num, v):
    return _field(num, 0) + _varint(int(v))


def _bytes(num, b):
    return hio._ld(num, b)


def _event(wall, step=None, file_version=None, summary=None) -> bytes:
    e = _double(1, wall)
    if step is not None:
        e += _int(2, step)
    if file_version is not None:
        e += _bytes(3, file_version.encode())
    if summary is not None:
        e += _bytes(5, summary)
    return e


def _scalar_value(tag: str, v: float) -> bytes:
    return _bytes(1, _bytes(1, tag.encode()) + _float(2, float(v)))


def _histo_value(tag: str, values) -> bytes:
    import numpy as np

    a = np.asarray(values, dtype=np.float64).reshape(-1)
    if a.size == 0:
        a = np.zeros(1)
    counts, edges = np.histogram(a, bins=30)
    h = (_double(1, float(a.min())) + _double(2, float(a.max())) + _double(3, float(a.size)) +
         _double(4, float(a.sum())) + _double(5, float((a * a).sum())))
    h += _bytes(6, b"".join(struct.pack("<d", float(x)) for x in edges[1:]))
    h += _bytes(7, b"".join(struct.pack("<d", float(x)) for x in counts))
    return _bytes(1, _bytes(1, tag.encode()) + _bytes(5, h))


def _text_value(tag: str, text: str) -> bytes:
    # TensorProto{dtype=DT_STRING(7), string_val(8)} + plugin metadata "text"
    tensor = _int(1, 7) + _bytes(8, text.encode())
    meta = _bytes(1, _bytes(1, b"text"))
    return _bytes(1, _bytes(1, tag.encode()) + _bytes(9, meta) + _bytes(8, tensor))


class SummaryWriter:
    """Minimal ``torch.utils.tensorboard.SummaryWriter``-compatible event writer."""

    def __init__(self, log_dir: str | None = None, comment: str = "", filename_suffix: str = ""):
        self.log_dir = log_dir or logdir()
        Path(self.log_dir).mkdir(parents=True, exist_ok=True)
        name = f"events.out.tfevents.{int(time.time())}.{socket.gethostname()}.{os.getpid()}{filename_suffix}"
        self.path = os.path.join(self.log_dir, name)
        self._w = hio.TFRecordWriter(self.path)
        self._w.write(_event(time.time(), file_version="brain.Event:2"))

    def add_scalar(self, tag, scalar_value, global_step=None, walltime=None):
        if hasattr(scalar_value, "item"):
            scalar_value = scalar_value.item()
        self._w.write(_event(walltime or time.time(), global_step or 0, summary=_scalar_value(tag, scalar_value)))

    def add_scalars(self, main_tag, tag_scalar_dict, global_step=None, walltime=None):
        for k, v in tag_scalar_dict.items():
            self.add_scalar(f"{main_tag}/{k}", v, global_step, walltime)

    def add_histogram(self, tag, values, global_step=None, walltime=None):
        if hasattr(values, "detach"):
            values = values.detach().float().cpu().numpy()
        self._w.write(_event(walltime or time.time(), global_step or 0, summary=_histo_value(tag, values)))

    def add_text(self, tag, text_string, global_step=None, walltime=None):
        self._w.write(_event(walltime or time.time(), global_step or 0, summary=_text_value(tag, text_string)))

    def flush(self):
        self._w.flush()

    def close(self):
        self._w.close()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


def read_scalars(path_or_dir: str) -> dict:
    """Parse scalar summaries back from event files: {tag: [(step, value)]} (used by tests/UI)."""
    p = Path(path_or_dir)
    files = sorted(p.glob("events.out.tfevents.*")) if p.is_dir() else [p]
    out: dict = {}
    for f in files:
        for rec in hio.read_tfrecords(str(f)):
            step, i = 0, 0
            summ = None
            while i < len(rec):
                key, i = _read_varint(rec, i)
                num, wire = key >> 3, key & 7
                if wire == 0:
                    v, i = _read_varint(rec, i)
                    if num == 2:
                        step = v
                elif wire == 1:
                    i += 8
                elif wire == 5:
                    i += 4
                else:
                    n, i = _read_varint(rec, i)
                    if num == 5:
                        summ = rec[i:i + n]
                    i += n
            if summ is None:
                continue
            for tag, val in _parse_summary(summ):
                out.setdefault(tag, []).append((step, val))
    return out


def _read_varint(b, i):
    v, sh = 0, 0
    while True:
        x = b[i]
        i += 1
        v |= (x & 0x7F) << sh
        if not x & 0x80:
            return v, i
        sh += 7


def _parse_summary(b):
    i = 0
    while i < len(b):
        key, i = _read_varint(b, i)
        n, i = _read_varint(b, i)
        val = b[i:i + n]
        i += n
        j, tag, sv = 0, None, None
        while j < len(val):
            k2, j = _read_varint(val, j)
            num, wire = k2 >> 3, k2 & 7
            if wire == 2:
                m, j = _read_varint(val, j)
                if num == 1:
                    tag = val[j:j + m].decode()
                j += m
            elif wire == 5:
                if num == 2:
                    sv = struct.unpack_from("<f", val, j)[0]
                j += 4
            elif wire == 1:
                j += 8
            else:
                _, j = _read_varint(val, j)
        if tag is not None and sv is not None:
            yield tag, sv
