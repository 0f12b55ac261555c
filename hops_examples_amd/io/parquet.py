"""Parquet -> HBM streaming reader (BASELINE config 4's ingest; north star: "the featurestore read
path (Parquet on HopsFS -> tensor) streams into 288 GB HBM via pinned hipMemcpyAsync on a side
stream").

Row groups are decoded on a pool of worker threads straight into a slot of a reusable pinned
staging ring: by the native decoder of ``_hopsx_io`` (csrc/io/parquet_core.h: mmapped file, Thrift
footer, PLAIN / dictionary / RLE pages, snappy; the GIL released, no Arrow objects and no
intermediate copy — a PLAIN page is one memcpy from the page cache into pinned memory), or, for
files it does not cover (nested or string columns, other codecs), by Arrow's reader plus one pack
copy.  The slot holds each column's RAW values (int64, float64, float32, int32, bool — whatever the
file stores); the main thread sends every slot host->device on a side stream as ONE copy and
converts + interleaves all its columns into the row-major fp32 destination with ONE hopsx kernel
(columns.hip).  Decodes of the next row groups overlap the transfer and conversion of the current
one.

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


def close_staging() -> None:
    """Join the decode pools and free the pinned / device staging rings (parallel.dist teardown order:
    after the comm handles, before the process group)."""
    for st in list(_STAGING.values()):
        for s in st.slots:
            if s[2] is not None:
                s[2].synchronize()
        if st.pool is not None:
            st.pool.shutdown(wait=True)
            st.pool = None
        st.slots = []
    _STAGING.clear()


_TLS = threading.local()  # per worker thread: {path: ParquetFile} (Arrow readers are not shared)


def _staging(device: torch.device) -> _Staging:
    st = _STAGING.get(device)
    if st is None:
        st = _STAGING[device] = _Staging(device)
    return st


_NATIVE: dict = {}  # (path, size, mtime_ns) -> _hopsx_io.ParquetFile (footer parsed once, mmapped; LRU)
_NATIVE_MAX = 256  # mapped files kept (each holds its mapping, not a descriptor)
_NP = {0: np.dtype(np.uint8), 1: np.dtype(np.int32), 2: np.dtype(np.int64), 4: np.dtype(np.float32),
       5: np.dtype(np.float64)}  # Parquet physical type -> raw value dtype in the staging slot


def _native_file(path: str):
    """The native decoder's handle of ``path`` (cached per file version), or None when the native
    library is unavailable or the file is outside its scope."""
    if os.environ.get("HOPSX_PARQUET_NATIVE", "1") != "1":
        return None
    try:
        st = os.stat(path)
    except OSError:
        return None
    key = (path, st.st_size, st.st_mtime_ns)
    f = _NATIVE.pop(key, False)
    if f is False:
        for k in [k for k in _NATIVE if k[0] == path]:  # an older version of this file: drop its mapping
            del _NATIVE[k]
        try:
            from .. import _hopsx_io as io

            f = io.ParquetFile(path)
        except Exception:  # noqa: BLE001 - not built, not Parquet, or unsupported layout: Arrow reads it
            f = None
    _NATIVE[key] = f  # (re)inserted last: the dict is in LRU order
    while len(_NATIVE) > _NATIVE_MAX:
        del _NATIVE[next(iter(_NATIVE))]
    return f


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
        self.native = {}   # path -> (native handle, column indices, raw dtypes) when natively decodable
        for p, rg in zip(paths, per_file):
            nf = _native_file(p)
            plan = self._native_plan(nf) if nf is not None else None
            if plan is not None:
                self.native[p] = plan
                rows_of = [r for r, _ in nf.meta()["row_groups"]]
            else:
                md = pq.ParquetFile(p).metadata
                rows_of = [md.row_group(g).num_rows for g in range(md.num_row_groups)]
            groups = list(range(len(rows_of)))
            if rg is not None:  # an explicit subset (a dataset-wide row-group shard, see to_device)
                groups = [g for g in rg if 0 <= g < len(rows_of)]
            elif shard is not None:
                n, i = shard
                groups = groups[i::n]
            self.sources += [(p, g, rows_of[g]) for g in groups]
        self._path = paths[0]
        self.groups = [g for _, g, _ in self.sources]
        self.rows = sum(r for _, _, r in self.sources)
        self.depth = max(1, depth)
        self.threads = threads
        # row groups decoded + packed in parallel (Arrow and torch's copy release the GIL)
        self.workers = workers or int(os.environ.get("HOPSX_PARQUET_WORKERS", min(8, os.cpu_count() or 4)))
        self.bytes_read = 0  # raw column bytes moved host -> device by the last read()

    # ---------------------------------------------------------------- host side
    def _native_plan(self, nf):
        """(handle, leaf indices, raw dtypes) of the requested columns, or None if any is outside
        the native decoder's scope (missing, nested, string / INT96 / fixed-length, repeated, or a
        converted / logical type that changes the meaning of the raw values: DECIMAL, unsigned,
        DATE / TIME / TIMESTAMP — Arrow converts those)."""
        md = nf.meta()
        by_name = {col[0]: (i, *col[1:]) for i, col in enumerate(md["columns"])}
        idx, dts = [], []
        for c in self.columns:
            e = by_name.get(c)
            if e is None or e[1] not in _NP or e[2] == 2 or (len(e) > 3 and not e[3]):
                return None
            idx.append(e[0])
            dts.append(_NP[e[1]])
        return nf, idx, dts

    def _layout(self, src):
        """Byte offsets of each column's raw values in a staging slot (native sources)."""
        _, _, dts = self.native[src[0]]
        offs, nb = [], 0
        for dt in dts:
            offs.append(nb)
            nb += -(-src[2] * dt.itemsize // _ALIGN) * _ALIGN
        return offs, nb

    def _decode_native_into(self, src, host_ptr: int):
        """Decode row group ``src`` straight into pinned memory at ``host_ptr``; returns
        (per-column (dtype, nbytes), offsets, total bytes), or None when the native decoder refuses a
        page (the caller falls back to Arrow for this row group)."""
        nf, idx, dts = self.native[src[0]]
        offs, nb = self._layout(src)
        try:
            nf.decode(src[1], idx, host_ptr, offs)  # releases the GIL
        except Exception as e:  # noqa: BLE001
            from .. import _hopsx_io as io

            if isinstance(e, io.ParquetUnsupported):
                return None
            raise
        return [(dt, src[2] * dt.itemsize) for dt in dts], offs, nb

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
            r0, moved = 0, 0
            for src in self.sources:
                m = src[2]
                got = None
                if src[0] in self.native:
                    _, nb = self._layout(src)
                    buf = torch.empty(nb, dtype=torch.uint8)
                    got = self._decode_native_into(src, buf.data_ptr())
                if got is not None:
                    cols = [buf[o:o + n].numpy().view(dt) for (dt, n), o in zip(got[0], got[1])]
                    moved += got[2]
                else:
                    cols = self._decode(src)
                for j, v in enumerate(cols):
                    out[r0:r0 + m, j] = torch.from_numpy(np.asarray(v, dtype=np.float32))
                r0 += m
            self.bytes_read = moved
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
                """Worker: decode one row group into ring slot i % depth once the H2D copy that last
                read that slot has completed — natively straight into the pinned slot, else Arrow
                decode + one pack copy.  Returns ([(dtype, nbytes)], offsets, slot bytes)."""
                host, _, ev = slots[i % depth]
                if src[0] in self.native:
                    if ev is not None:
                        ev.synchronize()
                    got = self._decode_native_into(src, host.data_ptr())
                    if got is not None:
                        return got
                cols = self._decode(src, threads)
                offs, nb = [], 0
                for v in cols:
                    offs.append(nb)
                    nb += -(-v.nbytes // _ALIGN) * _ALIGN
                if ev is not None:
                    ev.synchronize()
                for v, o in zip(cols, offs):
                    # torch's copy releases the GIL: the workers' packs run in parallel
                    host[o:o + v.nbytes].copy_(torch.from_numpy(v.view(np.uint8).reshape(-1)))
                return [(v.dtype, v.nbytes) for v in cols], offs, nb

            r0 = 0
            moved = 0
            futs = {i: pool.submit(decode_pack, i, self.sources[i]) for i in range(min(depth, n_g))}
            for i in range(n_g):
                cols, offs, nb = futs.pop(i).result()
                m = self.sources[i][2]
                slot = slots[i % depth]
                host, dev = slot[0], slot[1]
                with torch.cuda.stream(st.stream):
                    dev[:nb].copy_(host[:nb], non_blocking=True)  # one hipMemcpyAsync per row group
                    srcs = [dev[o:o + n].view(_torch_dtype(dt)) for (dt, n), o in zip(cols, offs)]
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
