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
import threading
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import torch

_ALIGN = 256  # byte alignment of each column inside a staging chunk


class _Staging:
    """Per-device resources shared by every reader of the process: the pinned + device staging ring
    (pinned allocation costs milliseconds — a training-dataset read opens one reader per Parquet
    part, so per-reader rings were allocated inside every read), the side stream, the decode pool.
    Slot i carries the event of the last H2D copy that read it; a worker packs into a slot only
    after that copy completed."""

    def __init__(self, device: torch.device):
        self.device = device
        self.slots: list = []  # [host pinned, device buffer, last H2D event]
        self.cap = 0
        self.stream = torch.cuda.Stream(device)
        self.pool = None
        self.workers = 0
        self.lock = threading.Lock()

    def ring(self, depth: int, cap: int) -> list:
        if cap > self.cap or len(self.slots) < depth:
            for s in self.slots:  # a grown ring replaces the old one once its copies are done
                if s[2] is not None:
                    s[2].synchronize()
            self.cap = max(cap, self.cap, 1 << 20)
            n = max(depth, len(self.slots))
            self.slots = [[torch.empty(self.cap, dtype=torch.uint8, pin_memory=True),
                           torch.empty(self.cap, dtype=torch.uint8, device=self.device), None] for _ in range(n)]
        return self.slots

    def executor(self, workers: int):
        if self.pool is None or self.workers < workers:
            if self.pool is not None:
                self.pool.shutdown(wait=True)
            self.pool = ThreadPoolExecutor(max_workers=workers, thread_name_prefix="hopsx-parquet")
            self.workers = workers
        return self.pool


_STAGING: dict = {}
_TLS = threading.local()  # per worker thread: {path: ParquetFile} (Arrow readers are not shared)


def _staging(device: torch.device) -> _Staging:
    st = _STAGING.get(device)
    if st is None:
        st = _STAGING[device] = _Staging(device)
    return st


def _thread_file(path: str):
    files = getattr(_TLS, "files", None)
    if files is None:
        files = _TLS.files = {}
    pf = files.get(path)
    if pf is None:
        import pyarrow.parquet as pq

        pf = files[path] = pq.ParquetFile(path)
    return pf


class ParquetDeviceReader:
    """``ParquetDeviceReader(path, columns).read()`` -> fp32 tensor [rows, len(columns)] in HBM.

    ``shard=(n, i)`` keeps every n-th row group starting at i (petastorm's ``shard_count`` /
    ``cur_shard``), ``row_groups`` an explicit list; ``depth`` pinned staging slots (double buffering
    by default)."""

    def __init__(self, path, columns, device=None, shard: tuple[int, int] | None = None, depth: int = 2,
                 threads: bool = True, row_groups=None, workers: int | None = None):
        """``path``: one Parquet file, or a list of files read as one table (a training dataset's
        parts) through ONE pipeline; ``row_groups``: the row groups to read (a list per file when
        ``path`` is a list)."""
        import pyarrow.parquet as pq

        multi = isinstance(path, (list, tuple))
        paths = [str(p) for p in path] if multi else [str(path)]
        per_file = list(row_groups) if (multi and row_groups is not None) else [row_groups] * len(paths)
        self.columns = list(columns)
        self.device = torch.device(device) if device is not None else (
            torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu"))
        self.sources = []  # (path, row group, rows), in output order
        for p, rg in zip(paths, per_file):
            md = pq.ParquetFile(p).metadata
            groups = list(range(md.num_row_groups))
            if rg is not None:  # an explicit subset (a dataset-wide row-group shard, see to_device)
                groups = [g for g in rg if 0 <= g < md.num_row_groups]
            elif shard is not None:
                n, i = shard
                groups = groups[i::n]
            self.sources += [(p, g, md.row_group(g).num_rows) for g in groups]
        self._path = paths[0]
        self.pf = pq.ParquetFile(self._path)
        self.groups = [g for _, g, _ in self.sources]
        self.rows = sum(r for _, _, r in self.sources)
        self.depth = max(1, depth)
        self.threads = threads
        # row groups decoded + packed in parallel (Arrow and torch's copy release the GIL)
        self.workers = workers or int(os.environ.get("HOPSX_PARQUET_WORKERS", min(8, os.cpu_count() or 4)))
        self.bytes_read = 0  # raw column bytes moved host -> device by the last read()

    # ---------------------------------------------------------------- host side
    def _decode(self, src, threads: bool | None = None):
        """One (path, row group) -> list of numpy views of the raw column buffers (zero-copy where
        Arrow allows); the calling thread's own ParquetFile handle."""
        tbl = _thread_file(src[0]).read_row_group(src[1], columns=self.columns,
                                                  use_threads=self.threads if threads is None else threads)
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

    def _cap(self) -> int:
        """Upper bound of one row group's raw column bytes (8 bytes a value + alignment)."""
        rows = max((r for _, _, r in self.sources), default=0)
        return rows * len(self.columns) * 8 + len(self.columns) * _ALIGN

    # ---------------------------------------------------------------- read
    def read(self, out: torch.Tensor | None = None) -> torch.Tensor:
        n, k = self.rows, len(self.columns)
        if out is None:
            out = torch.empty(n, k, dtype=torch.float32, device=self.device)
        if self.device.type != "cuda":
            r0 = 0
            for src in self.sources:
                cols = self._decode(src)
                m = len(cols[0])
                for j, v in enumerate(cols):
                    out[r0:r0 + m, j] = torch.from_numpy(np.array(v, dtype=np.float32))
                r0 += m
            return out
        from ..ops import kernels as K

        st = _staging(self.device)
        n_g = len(self.sources)
        nthreads = max(1, min(self.workers, n_g))
        with st.lock:  # one read at a time per device: the ring and the side stream are shared
            depth = max(self.depth, nthreads + 1)
            slots = st.ring(depth, self._cap())
            depth = len(slots)
            pool = st.executor(nthreads)
            cur = torch.cuda.current_stream(self.device)
            st.stream.wait_stream(cur)  # out may have been allocated / used on the current stream
            threads = self.threads and nthreads == 1  # Arrow's own column threads only without the pool

            def decode_pack(i: int, src):
                """Worker: decode one row group, then pack its raw column buffers into ring slot
                i % depth once the H2D copy that last read that slot has completed."""
                cols = self._decode(src, threads)
                offs, nb = [], 0
                for v in cols:
                    offs.append(nb)
                    nb += -(-v.nbytes // _ALIGN) * _ALIGN
                host, _, ev = slots[i % depth]
                if ev is not None:
                    ev.synchronize()
                for v, o in zip(cols, offs):
                    # torch's copy releases the GIL: the workers' packs run in parallel
                    host[o:o + v.nbytes].copy_(torch.from_numpy(v.view(np.uint8).reshape(-1)))
                return cols, offs, nb

            r0 = 0
            moved = 0
            futs = {i: pool.submit(decode_pack, i, self.sources[i]) for i in range(min(depth, n_g))}
            for i in range(n_g):
                cols, offs, nb = futs.pop(i).result()
                m = len(cols[0])
                slot = slots[i % depth]
                host, dev = slot[0], slot[1]
                with torch.cuda.stream(st.stream):
                    dev[:nb].copy_(host[:nb], non_blocking=True)  # one hipMemcpyAsync per row group
                    srcs = [dev[o:o + v.nbytes].view(_torch_dtype(v.dtype)) for v, o in zip(cols, offs)]
                    K.cols_to_f32(srcs, out[r0:r0 + m])  # convert + interleave: one launch per row group
                    e = torch.cuda.Event()
                    e.record(st.stream)
                slot[2] = e
                if i + depth < n_g:
                    futs[i + depth] = pool.submit(decode_pack, i + depth, self.sources[i + depth])
                r0 += m
                moved += nb
            cur.wait_stream(st.stream)
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
