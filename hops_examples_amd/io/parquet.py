"""Parquet -> HBM streaming reader (BASELINE config 4's ingest; north star: "the featurestore read
path (Parquet on HopsFS -> tensor) streams into 288 GB HBM via pinned hipMemcpyAsync on a side
stream").

Row groups are decoded by Arrow's C++ reader on a pool of worker threads (one ParquetFile handle
per thread; Arrow and torch's copy release the GIL); each worker packs its row group's RAW column
buffers (int64, float64, float32, int32, bool — whatever the file stores) into a slot of a reusable
pinned staging ring, and the main thread sends every slot host->device on a side stream as ONE
copy and converts + interleaves all its columns into the row-major fp32 destination with ONE
hopsx kernel (columns.hip).  The host never converts, stacks or re-pins anything; decodes of the
next row groups overlap the transfer and conversion of the current one.

Reference parity: the training-dataset readers the notebooks use (``td.read()``,
``tf_data(...).tf_record_dataset``; notebooks/featurestore/hsfs/basics/training_datasets.ipynb:
463-526) and petastorm's Parquet readers (PetastormHelloWorld.ipynb:864-899, sharding by row group).
"""
from __future__ import annotations

import os

import numpy as np
import torch

_ALIGN = 256  # byte alignment of each column inside a staging chunk


class ParquetDeviceReader:
    """``ParquetDeviceReader(path, columns).read()`` -> fp32 tensor [rows, len(columns)] in HBM.

    ``shard=(n, i)`` keeps every n-th row group starting at i (petastorm's ``shard_count`` /
    ``cur_shard``), ``row_groups`` an explicit list; ``depth`` pinned staging slots (double buffering
    by default)."""

    def __init__(self, path, columns, device=None, shard: tuple[int, int] | None = None, depth: int = 2,
                 threads: bool = True, row_groups=None, workers: int | None = None):
        import pyarrow.parquet as pq

        self._path = str(path)
        self.pf = pq.ParquetFile(self._path)
        self.columns = list(columns)
        self.device = torch.device(device) if device is not None else (
            torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu"))
        md = self.pf.metadata
        groups = list(range(md.num_row_groups))
        if row_groups is not None:  # an explicit subset (a dataset-wide row-group shard, see to_device)
            groups = [g for g in row_groups if 0 <= g < md.num_row_groups]
        elif shard is not None:
            n, i = shard
            groups = groups[i::n]
        self.groups = groups
        self.rows = sum(md.row_group(g).num_rows for g in groups)
        self.depth = max(1, depth)
        self.threads = threads
        # row groups decoded + packed in parallel (Arrow and torch's copy release the GIL)
        self.workers = workers or int(os.environ.get("HOPSX_PARQUET_WORKERS", min(8, os.cpu_count() or 4)))
        self._slots = None
        self._stream = None
        self.bytes_read = 0  # raw column bytes moved host -> device by the last read()

    # ---------------------------------------------------------------- host side
    def _decode(self, g: int, pf=None):
        """One row group -> list of numpy views of the raw column buffers (zero-copy where Arrow allows)."""
        tbl = (pf or self.pf).read_row_group(g, columns=self.columns, use_threads=self.threads)
        cols = []
        for c in self.columns:
            a = tbl.column(c)
            if a.num_chunks != 1:
                a = a.combine_chunks()
            else:
                a = a.chunk(0)
            if a.null_count:
                # missing values: NaN in float columns (what td.read() gives), 0 elsewhere
                import pyarrow as pa

                a = a.fill_null(float("nan") if pa.types.is_floating(a.type) else 0)
            try:
                v = a.to_numpy(zero_copy_only=True)
            except Exception:  # bools / dictionary columns: one conversion on the host
                v = a.to_numpy(zero_copy_only=False)
            if v.dtype == np.bool_:
                v = v.view(np.uint8)
            cols.append(v)
        return cols

    def _slot(self, nbytes: int):
        if self._slots is not None and self._slots[0][0].numel() < nbytes:
            raise RuntimeError("row group larger than the staging bound")  # (sized from the metadata)
        if self._slots is None:
            md = self.pf.metadata
            # upper bound of one row group's raw column bytes: 8 bytes per value + alignment
            rows = max((md.row_group(g).num_rows for g in self.groups), default=0)
            cap = max(nbytes, rows * len(self.columns) * 8 + len(self.columns) * _ALIGN, 1 << 20)
            self._slots = []
            for _ in range(self.depth):
                host = torch.empty(cap, dtype=torch.uint8, pin_memory=self.device.type == "cuda")
                dev = torch.empty(cap, dtype=torch.uint8, device=self.device)
                self._slots.append([host, dev, None])
        return self._slots

    # ---------------------------------------------------------------- read
    def read(self, out: torch.Tensor | None = None) -> torch.Tensor:
        n, k = self.rows, len(self.columns)
        if out is None:
            out = torch.empty(n, k, dtype=torch.float32, device=self.device)
        if self.device.type != "cuda":
            r0 = 0
            for g in self.groups:
                cols = self._decode(g)
                m = len(cols[0])
                for j, v in enumerate(cols):
                    out[r0:r0 + m, j] = torch.from_numpy(np.array(v, dtype=np.float32))
                r0 += m
            return out
        if self._stream is None:
            self._stream = torch.cuda.Stream(self.device)
        from ..ops import kernels as K

        cur = torch.cuda.current_stream(self.device)
        self._stream.wait_stream(cur)  # out may have been allocated / used on the current stream
        n_g = len(self.groups)
        nthreads = max(1, min(self.workers, n_g))
        depth = max(self.depth, nthreads + 1)
        if self._slots is not None and len(self._slots) < depth:
            self._slots = None
        self.depth = depth
        import threading
        from concurrent.futures import ThreadPoolExecutor

        local = threading.local()

        def decode_pack(i: int, g: int, wait_ev):
            """Worker: decode row group g (its own ParquetFile handle: Arrow readers are not shared
            across threads), then pack the raw column buffers into pinned slot i % depth once the
            H2D copy that last read that slot has completed (wait_ev)."""
            if not hasattr(local, "pf"):
                import pyarrow.parquet as pq

                local.pf = pq.ParquetFile(self._path)
            cols = self._decode(g, local.pf)
            offs, nb = [], 0
            for v in cols:
                offs.append(nb)
                nb += -(-v.nbytes // _ALIGN) * _ALIGN
            if wait_ev is not None:
                wait_ev.synchronize()
            host = self._slots[i % depth][0]
            for v, o in zip(cols, offs):
                # torch's copy_ releases the GIL (the workers' packs run in parallel)
                host[o:o + v.nbytes].copy_(torch.from_numpy(v.view(np.uint8).reshape(-1)))
            return cols, offs, nb

        # size the ring from the metadata before any worker writes into it
        self._slot(0)
        r0 = 0
        moved = 0
        events = [None] * depth
        with ThreadPoolExecutor(max_workers=nthreads) as ex:
            futs = {}
            for i in range(min(depth, n_g)):
                futs[i] = ex.submit(decode_pack, i, self.groups[i], None)
            for i in range(n_g):
                cols, offs, nb = futs.pop(i).result()
                m = len(cols[0])
                host, dev, _ = self._slots[i % depth]
                with torch.cuda.stream(self._stream):
                    dev[:nb].copy_(host[:nb], non_blocking=True)  # one hipMemcpyAsync per row group
                    srcs = [dev[o:o + v.nbytes].view(_torch_dtype(v.dtype)) for v, o in zip(cols, offs)]
                    K.cols_to_f32(srcs, out[r0:r0 + m])  # convert + interleave: one launch per row group
                    e = torch.cuda.Event()
                    e.record(self._stream)
                events[i % depth] = e
                nxt = i + depth
                if nxt < n_g:
                    futs[nxt] = ex.submit(decode_pack, nxt, self.groups[nxt], e)
                r0 += m
                moved += nb
        cur.wait_stream(self._stream)
        out.record_stream(cur)
        self.bytes_read = moved
        return out


def _torch_dtype(dt: np.dtype):
    m = {np.dtype(np.float32): torch.float32, np.dtype(np.float64): torch.float64,
         np.dtype(np.int64): torch.int64, np.dtype(np.int32): torch.int32, np.dtype(np.int16): torch.int16,
         np.dtype(np.int8): torch.int8, np.dtype(np.uint8): torch.uint8, np.dtype(np.float16): torch.float16}
    if np.dtype(dt) not in m:
        raise TypeError(f"unsupported Parquet column dtype {dt}")
    return m[np.dtype(dt)]


def read_parquet_to_device(path, columns, device=None, shard=None) -> torch.Tensor:
    """One-call form: fp32 [rows, len(columns)] in HBM."""
    return ParquetDeviceReader(path, columns, device=device, shard=shard).read()
