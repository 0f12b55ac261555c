"""torch adapter: batches reader rows into dicts of tensors; with ``device='cuda'`` the
batches land in HBM through pinned staging + a non-blocking copy."""
from __future__ import annotations

import numpy as np
import torch


def _collate(rows):
    out = {}
    for k in rows[0]._fields:
        vals = [getattr(r, k) for r in rows]
        if isinstance(vals[0], np.ndarray):
            if vals[0].ndim >= 1 and len(rows) == 1:  # batch reader: already a column batch
                out[k] = torch.from_numpy(np.ascontiguousarray(vals[0]))
            else:
                out[k] = torch.from_numpy(np.stack(vals))
        elif isinstance(vals[0], (int, float, np.integer, np.floating, bool)):
            out[k] = torch.as_tensor(np.asarray(vals))
        else:
            out[k] = vals
    return out


class DataLoader:
    def __init__(self, reader, batch_size: int = 1, collate_fn=None, device=None, drop_last: bool = False):
        self.reader, self.batch_size, self.collate = reader, batch_size, collate_fn or _collate
        self.device = torch.device(device) if device is not None else None
        self.drop_last = drop_last

    def _move(self, b):
        if self.device is None or self.device.type != "cuda":
            return b
        return {k: (v.pin_memory().to(self.device, non_blocking=True) if isinstance(v, torch.Tensor) else v)
                for k, v in b.items()}

    def __iter__(self):
        buf = []
        for row in self.reader:
            if getattr(self.reader, "batched", False):
                yield self._move(self.collate([row]))
                continue
            buf.append(row)
            if len(buf) == self.batch_size:
                yield self._move(self.collate(buf))
                buf = []
        if buf and not self.drop_last:
            yield self._move(self.collate(buf))

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.reader.stop()


BatchedDataLoader = DataLoader
