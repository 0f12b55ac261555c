"""Spark-style range windows for feature engineering:
``F.sum(col).over(Window.partitionBy(keys).orderBy(ts).rangeBetween(lo, hi))``.

Reference: notebooks/featurestore/hsfs/basics/feature_engineering.ipynb:229-249 — weekly sales
summed over the last 30/90/180/365 days (``rangeBetween(days(-N), days(-1))``) per (store, dept)
and per store, then ``fillna(0)``.

The host sorts the rows by (partition, order key) and finds the partition boundaries; the sums run
on the GPU (``window.hip``: fp64 prefix sum + two binary searches per row and window, every window
in one launch) when a GPU is present and the frame is large enough to pay for the copies, else
through the same algorithm in numpy.  An empty range gives NaN (Spark's null) — fill as the
reference does.  Result order is the input frame's order.
"""
from __future__ import annotations

import numpy as np
import pandas as pd

GPU_MIN_ROWS = 50_000
DAY = 86_400


def days(i: int) -> int:
    """Seconds in ``i`` days (the reference's ``days = lambda i: i * 86400``)."""
    return int(i) * DAY


def _sorted_layout(df: pd.DataFrame, partition_by, order_by: str):
    keys = [partition_by] if isinstance(partition_by, str) else list(partition_by)
    ts = pd.to_numeric(df[order_by], errors="coerce")
    if ts.isna().any():
        raise ValueError(f"order column {order_by!r} has missing values")
    codes = [pd.factorize(df[k], sort=True)[0] for k in keys]
    order = np.lexsort([ts.to_numpy()] + codes[::-1])
    newseg = np.ones(len(order), bool)
    if len(order) > 1:
        newseg[1:] = False
        for c in codes:
            cs = c[order]
            newseg[1:] |= cs[1:] != cs[:-1]
    seg = np.cumsum(newseg) - 1
    seg_off = np.concatenate([np.flatnonzero(newseg), [len(order)]]).astype(np.int64)
    return order, ts.to_numpy(np.int64)[order], seg.astype(np.int32), seg_off


def _sums_sorted(ts, seg_off, v, lo, hi, with_count, device):
    """Window sums/counts of rows already sorted by (partition, order key); sorted order out."""
    n, nw = len(ts), len(lo)
    use_gpu = False
    if n:
        import torch

        use_gpu = torch.cuda.is_available() and (device is not None and torch.device(device).type == "cuda"
                                                 or (device is None and n >= GPU_MIN_ROWS))
    if use_gpu:
        import torch

        from ..ops import kernels as K

        dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
        seg = np.repeat(np.arange(len(seg_off) - 1, dtype=np.int32), np.diff(seg_off))
        r = K.range_window(t(ts), t(seg), t(seg_off), t(v), t(lo), t(hi), want_count=with_count)
        if with_count:
            return r[0].cpu().numpy(), r[1].cpu().numpy()
        return r.cpu().numpy(), None
    P = np.concatenate([[0.0], np.cumsum(v)])
    sums = np.full((n, nw), np.nan)
    cnts = np.zeros((n, nw), np.int64)
    for s in range(len(seg_off) - 1):
        a, b = seg_off[s], seg_off[s + 1]
        tt = ts[a:b]
        for w in range(nw):
            f = a + np.searchsorted(tt, tt + lo[w], side="left")
            e = a + np.searchsorted(tt, tt + hi[w], side="right")
            c = np.maximum(e - f, 0)
            cnts[a:b, w] = c
            sums[a:b, w] = np.where(c > 0, P[np.maximum(e, f)] - P[f], np.nan)
    return sums, cnts


def _world(process_group):
    import torch.distributed as dist

    if process_group is False or not dist.is_available() or not dist.is_initialized():
        return 1, 0
    return dist.get_world_size(process_group), dist.get_rank(process_group)


def range_sums(df: pd.DataFrame, partition_by, order_by: str, value: str, windows, device=None,
               with_count: bool = False, process_group=None):
    """Sums of ``value`` over each ``(lo, hi)`` range of the order key (inclusive, relative to the
    row's own key) within its partition.  Returns a float64 array [len(df), len(windows)] in the
    frame's row order (NaN: empty range), plus int counts with ``with_count``.

    Data-parallel (``torch.distributed`` initialised with world > 1, or an explicit
    ``process_group``; ``False`` turns it off): every rank computes the windows of the partitions it
    owns (partition i -> rank i % world, like a Spark shuffle by the partition keys) on its own
    device, then the per-rank results are all-gathered, so each rank returns the full frame's
    result — the reference runs this ``Window.partitionBy`` aggregation on Spark executors
    (feature_engineering.ipynb:229-249)."""
    windows = [(int(lo), int(hi)) for lo, hi in windows]
    n = len(df)
    order, ts, seg, seg_off = _sorted_layout(df, partition_by, order_by)
    v = pd.to_numeric(df[value], errors="coerce").fillna(0).to_numpy(np.float64)[order]
    lo = np.array([w[0] for w in windows], np.int64)
    hi = np.array([w[1] for w in windows], np.int64)
    world, rank = _world(process_group)
    if world > 1 and n:
        import torch.distributed as dist

        own = (seg % world) == rank  # this rank's partitions (whole partitions, rows contiguous)
        sizes = np.diff(seg_off)
        mine = np.arange(len(sizes)) % world == rank
        sub_off = np.concatenate([[0], np.cumsum(sizes[mine])]).astype(np.int64)
        s_sub, c_sub = _sums_sorted(ts[own], sub_off, v[own], lo, hi, with_count, device)
        parts = [None] * world
        dist.all_gather_object(parts, (order[own], s_sub, c_sub), group=process_group)
        sums = np.empty((n, len(windows)))
        cnts = np.zeros((n, len(windows)), np.int64)
        for idx, s_, c_ in parts:
            sums[idx] = s_
            if with_count:
                cnts[idx] = c_
        return (sums, cnts) if with_count else sums
    sums, cnts = _sums_sorted(ts, seg_off, v, lo, hi, with_count, device)
    out = np.empty_like(sums)
    out[order] = sums
    if not with_count:
        return out
    oc = np.empty_like(cnts)
    oc[order] = cnts
    return out, oc


def with_range_sums(df: pd.DataFrame, specs: dict, partition_by, order_by: str, value: str, device=None,
                    fill=0.0, process_group=None) -> pd.DataFrame:
    """``df`` plus one column per ``{name: (lo, hi)}`` — the reference's chain of ``withColumn(name,
    F.sum(value).over(window))`` followed by ``fillna(fill)``."""
    names = list(specs)
    sums = range_sums(df, partition_by, order_by, value, [specs[k] for k in names], device=device,
                      process_group=process_group)
    out = df.copy()
    for j, k in enumerate(names):
        col = sums[:, j]
        out[k] = np.where(np.isnan(col), fill, col) if fill is not None else col
    return out
