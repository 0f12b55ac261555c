"""DeviceLoader: host arrays -> shuffled mini-batches -> HBM, overlapped with compute.

The path the SURVEY asks for (§1.2 DATA, BASELINE north star "Parquet on
HopsFS -> tensor streams into 288 GB HBM via pinned hipMemcpyAsync on a side
stream"):

  * batch assembly: rows gathered by index into a PINNED host slot by the C++
    thread pool (``_hopsx_io.gather_rows``; no Python per row);
  * transfer: ``copy_`` with ``non_blocking=True`` on a dedicated copy stream
    (hipMemcpyAsync from pinned memory, DMA engine, no SM time);
  * hand-off: the consumer stream waits on a per-slot event, and the slot is
    recycled only after the transfer that read it has completed;
  * ``resident=True`` (default when it fits) keeps the WHOLE dataset in HBM —
    with 288 GB per MI355X every reference dataset fits — and batches are then
    device-side index gathers with no host traffic at all;
  * sharding (petastorm's ``shard_count``/``cur_shard``) splits rows per rank.
"""
from __future__ import annotations

import numpy as np
import torch

from . import gather_rows


class DeviceLoader:
    def __init__(self, x: np.ndarray, y: np.ndarray | None, batch_size: int, shuffle: bool = True,
                 drop_last: bool = True, device=None, shard: tuple[int, int] | None = None, seed: int | None = None,
                 resident: bool | None = None, depth: int = 3, x_dtype=None):
        if shard is not None:
            n, i = shard
            sel = np.arange(len(x))[i::n]
            x = x[sel]
            y = y[sel] if y is not None else None
        self.x = np.ascontiguousarray(x)
        self.y = None if y is None else np.ascontiguousarray(y)
        self.batch_size, self.shuffle, self.drop_last = batch_size, shuffle, drop_last
        self.device = torch.device(device) if device is not None else (
            torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu"))
        self.rng = np.random.default_rng(seed)
        self.depth = depth
        nbytes = self.x.nbytes + (0 if self.y is None else self.y.nbytes)
        if resident is None:
            resident = self.device.type == "cuda" and nbytes < (8 << 30)
        self.resident = resident and self.device.type == "cuda"
        self._x_dev = self._y_dev = None
        if self.resident:
            self._x_dev = torch.from_numpy(self.x).to(self.device, non_blocking=False)
            if x_dtype is not None:
                self._x_dev = self._x_dev.to(x_dtype)
            if self.y is not None:
                self._y_dev = torch.from_numpy(self.y).to(self.device)
        elif self.device.type == "cuda":
            self._stream = torch.cuda.Stream(self.device)
            self._slots = []
            for _ in range(depth):
                hx = torch.empty((batch_size,) + self.x.shape[1:], dtype=torch.from_numpy(self.x[:1]).dtype).pin_memory()
                hy = None if self.y is None else torch.empty((batch_size,) + self.y.shape[1:],
                                                             dtype=torch.from_numpy(self.y[:1]).dtype).pin_memory()
                self._slots.append([hx, hy, None])

    @classmethod
    def from_tensors(cls, x: torch.Tensor, y: torch.Tensor | None, batch_size: int, shuffle: bool = True,
                     drop_last: bool = True, seed: int | None = None) -> "DeviceLoader":
        """A resident loader over tensors already in HBM (e.g. io.parquet.ParquetDeviceReader output)."""
        self = cls.__new__(cls)
        self.x, self.y = x, y
        self.batch_size, self.shuffle, self.drop_last = batch_size, shuffle, drop_last
        self.device = x.device
        self.rng = np.random.default_rng(seed)
        self.depth = 0
        self.resident = True
        self._x_dev, self._y_dev = x, y
        return self

    def __len__(self):
        n = len(self.x)
        return n // self.batch_size if self.drop_last else -(-n // self.batch_size)

    def _order(self):
        return self.rng.permutation(len(self.x)) if self.shuffle else np.arange(len(self.x))

    def __iter__(self):
        order = self._order()
        nb = len(self)
        if self.resident:
            perm = torch.from_numpy(order).to(self.device)
            for b in range(nb):
                idx = perm[b * self.batch_size:(b + 1) * self.batch_size]
                yield (self._x_dev.index_select(0, idx),
                       None if self._y_dev is None else self._y_dev.index_select(0, idx))
            return
        if self.device.type != "cuda":
            for b in range(nb):
                idx = order[b * self.batch_size:(b + 1) * self.batch_size]
                yield torch.from_numpy(self.x[idx]), (None if self.y is None else torch.from_numpy(self.y[idx]))
            return
        cur = torch.cuda.current_stream(self.device)
        pending = []
        for b in range(nb):
            slot = self._slots[b % self.depth]
            if slot[2] is not None:
                slot[2].synchronize()  # the H2D that last read this pinned slot is done
            idx = order[b * self.batch_size:(b + 1) * self.batch_size]
            k = len(idx)
            gather_rows(self.x, idx, slot[0].numpy())
            if self.y is not None:
                gather_rows(self.y, idx, slot[1].numpy())
            with torch.cuda.stream(self._stream):
                dx = slot[0][:k].to(self.device, non_blocking=True)
                dy = None if self.y is None else slot[1][:k].to(self.device, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(self._stream)
            slot[2] = ev
            pending.append((dx, dy, ev))
            if len(pending) >= 2 or b == nb - 1:
                while pending:
                    px, py, pev = pending.pop(0)
                    cur.wait_event(pev)
                    px.record_stream(cur)
                    if py is not None:
                        py.record_stream(cur)
                    yield px, py


# ------------------------------------------------------------------ TFRecord image datasets
def write_image_tfrecords(path, images: np.ndarray, labels: np.ndarray, image_key: str = "image_raw",
                          label_key: str = "label") -> int:
    """Write uint8 images + int labels as tf.train.Examples {image_raw: bytes, label: int64} — the
    layout of the reference's MNIST TFRecords (mirroredstrategy_mnist_example.ipynb:153-186)."""
    from . import write_tfrecord_columns

    imgs = np.ascontiguousarray(images, dtype=np.uint8)
    n = len(imgs)
    flat = imgs.reshape(n, -1)
    return write_tfrecord_columns(str(path), [(image_key, "bytes", [r.tobytes() for r in flat]),
                                              (label_key, "int64", np.asarray(labels, np.int64))], n)


class TFRecordImageDataset:
    """``tf.data.TFRecordDataset(files).map(parser).batch(B, drop_remainder=True).repeat()`` with the
    parse done by the C++ IO library (framing CRCs checked, Examples decoded columnar by a thread
    pool) and the decoded uint8 images + labels kept resident in HBM.

    ``shard=None`` is ``AutoShardPolicy.OFF`` (the reference's multi-worker setting,
    multiworkermirroredstrategy_mnist_example.ipynb:183-185): every worker reads every record.
    ``shard=(n, i)`` keeps records i, i+n, ... (``AutoShardPolicy.DATA``)."""

    def __init__(self, files, image_shape=(28, 28, 1), image_key: str = "image_raw", label_key: str = "label",
                 shard: tuple[int, int] | None = None, device=None):
        from . import decode_batch, read_tfrecords

        files = [files] if isinstance(files, (str, bytes)) or hasattr(files, "__fspath__") else list(files)
        recs = [r for f in files for r in read_tfrecords(str(f))]
        if shard is not None:
            n, i = shard
            recs = recs[i::n]
        size = int(np.prod(image_shape))
        cols = decode_batch(recs, [(image_key, "bytes", size), (label_key, "int64", 1)]) if recs else {
            image_key: np.zeros((0, size), np.uint8), label_key: np.zeros((0, 1), np.int64)}
        self.device = torch.device(device) if device is not None else (
            torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu"))
        pin = self.device.type == "cuda"
        x = torch.from_numpy(cols[image_key].reshape((-1,) + tuple(image_shape)))
        y = torch.from_numpy(cols[label_key][:, 0])
        self.images = (x.pin_memory() if pin else x).to(self.device, non_blocking=True)
        self.labels = (y.pin_memory() if pin else y).to(self.device, non_blocking=True)

    def __len__(self) -> int:
        return int(self.labels.shape[0])

    def batches(self, batch_size: int):
        """[nb, B, ...] views of the resident epoch (drop_remainder=True), ready for
        TrainStep.step_resident / run_resident (the repeat is the cursor wrapping around)."""
        nb = len(self) // batch_size
        if nb < 1:
            raise ValueError(f"{len(self)} records < one batch of {batch_size}")
        return (self.images[:nb * batch_size].view((nb, batch_size) + tuple(self.images.shape[1:])),
                self.labels[:nb * batch_size].view(nb, batch_size))
