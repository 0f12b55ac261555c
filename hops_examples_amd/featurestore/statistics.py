"""Feature statistics (descriptive, histograms, correlations) for feature groups
and training datasets — ``statistics_config={"enabled", "histograms", "correlations"}``
(hsfs/basics/feature_engineering.ipynb:182).

Numeric columns are reduced on the GPU by the hopsx column-statistics kernels
(one pass for count/sum/sum^2/min/max, one for histograms, one centred Gram
matrix for Pearson correlations) when a GPU is present and the frame is large
enough to amortise the transfer; otherwise numpy computes the same values.
"""
from __future__ import annotations

import math

import numpy as np
import pandas as pd

GPU_MIN_ROWS = 1 << 16


class StatisticsConfig:
    def __init__(self, enabled=True, histograms=False, correlations=False, columns=None):
        self.enabled, self.histograms, self.correlations, self.columns = enabled, histograms, correlations, columns

    @classmethod
    def parse(cls, cfg):
        if cfg is None:
            return cls(True, False, False)
        if isinstance(cfg, bool):
            return cls(cfg, False, False)
        if isinstance(cfg, StatisticsConfig):
            return cfg
        return cls(cfg.get("enabled", True), cfg.get("histograms", False), cfg.get("correlations", False),
                   cfg.get("columns"))

    def to_dict(self):
        return {"enabled": self.enabled, "histograms": self.histograms, "correlations": self.correlations,
                "columns": self.columns}


def _numeric_matrix(df: pd.DataFrame):
    cols = [c for c in df.columns if pd.api.types.is_numeric_dtype(df[c]) and not pd.api.types.is_bool_dtype(df[c])]
    if not cols:
        return cols, np.zeros((len(df), 0), np.float32)
    return cols, df[cols].apply(pd.to_numeric, errors="coerce").to_numpy(np.float32)


def _gpu_ok(rows: int) -> bool:
    try:
        import torch

        return torch.cuda.is_available() and rows >= GPU_MIN_ROWS
    except Exception:  # pragma: no cover
        return False


def column_stats(x: np.ndarray, bins: int = 20, correlations: bool = False, histograms: bool = False):
    """x [rows, cols] float32 (NaN = missing) -> dict of per-column arrays (+hist, +corr)."""
    rows, cols = x.shape
    out = {}
    if _gpu_ok(rows) and cols:
        import torch

        from ..ops import kernels as K

        xt = torch.from_numpy(np.ascontiguousarray(x)).pin_memory().cuda(non_blocking=True)
        st = K.column_stats(xt)
        cnt, s, sq, mn, mx = (st[:, i] for i in range(5))
        mean = s / cnt.clamp_min(1)
        var = (sq / cnt.clamp_min(1) - mean * mean).clamp_min(0)
        out.update(count=cnt.cpu().numpy(), sum=s.cpu().numpy(), mean=mean.cpu().numpy(),
                   stddev=var.sqrt().cpu().numpy(), min=mn.cpu().numpy(), max=mx.cpu().numpy())
        if histograms:
            out["hist"] = K.column_hist(xt, mn.contiguous(), mx.contiguous(), bins).cpu().numpy()
        if correlations:
            g = K.gram(xt, mean.contiguous()).double()
            d = g.diagonal().clamp_min(1e-30).sqrt()
            out["corr"] = (g / d[:, None] / d[None, :]).cpu().numpy()
        out["device"] = "gpu"
        return out
    valid = ~np.isnan(x)
    cnt = valid.sum(0).astype(np.float64)
    xz = np.where(valid, x, 0).astype(np.float64)
    s = xz.sum(0)
    mean = s / np.maximum(cnt, 1)
    var = np.maximum((xz * xz).sum(0) / np.maximum(cnt, 1) - mean * mean, 0)
    mn = np.where(valid, x, np.inf).min(0) if rows else np.full(cols, np.inf)
    mx = np.where(valid, x, -np.inf).max(0) if rows else np.full(cols, -np.inf)
    out.update(count=cnt, sum=s, mean=mean, stddev=np.sqrt(var), min=mn, max=mx)
    if histograms:
        h = np.zeros((cols, bins), np.int64)
        for c in range(cols):
            v = x[valid[:, c], c]
            if len(v):
                lo, hi = mn[c], mx[c]
                idx = np.zeros(len(v), np.int64) if hi <= lo else np.clip(((v - lo) / (hi - lo) * bins).astype(
                    np.int64), 0, bins - 1)
                h[c] = np.bincount(idx, minlength=bins)
        out["hist"] = h
    if correlations:
        xc = np.where(valid, x - mean, 0)
        g = xc.T @ xc
        d = np.sqrt(np.maximum(np.diag(g), 1e-30))
        out["corr"] = g / d[:, None] / d[None, :]
    out["device"] = "cpu"
    return out


def compute(df: pd.DataFrame, cfg: StatisticsConfig | None = None, bins: int = 20) -> dict:
    """hsfs-style statistics JSON: {'columns': [{column, dataType, count, completeness, mean, …}], …}."""
    cfg = cfg or StatisticsConfig()
    if cfg.columns:
        df = df[[c for c in cfg.columns if c in df.columns]]
    cols, x = _numeric_matrix(df)
    st = column_stats(x, bins, cfg.correlations, cfg.histograms) if cols else {}
    n = len(df)
    columns = []
    for i, c in enumerate(cols):
        e = {"column": c, "dataType": "Fractional", "count": int(st["count"][i]),
             "completeness": float(st["count"][i] / n) if n else 1.0, "mean": float(st["mean"][i]),
             "stdDev": float(st["stddev"][i]), "minimum": float(st["min"][i]), "maximum": float(st["max"][i]),
             "sum": float(st["sum"][i]), "approximateNumDistinctValues": int(df[c].nunique(dropna=True))}
        if cfg.histograms and "hist" in st:
            lo, hi = float(st["min"][i]), float(st["max"][i])
            edges = np.linspace(lo, hi if hi > lo else lo + 1, bins + 1)
            e["histogram"] = [{"bin": f"{edges[b]:.6g}-{edges[b + 1]:.6g}", "value": int(st["hist"][i][b])}
                              for b in range(bins)]
        if cfg.correlations and "corr" in st:
            e["correlations"] = [{"column": cols[j], "correlation": float(st["corr"][i][j])}
                                 for j in range(len(cols)) if not math.isnan(st["corr"][i][j])]
        columns.append(e)
    for c in df.columns:
        if c in cols:
            continue
        s = df[c]
        columns.append({"column": c, "dataType": "String", "count": int(s.notna().sum()),
                        "completeness": float(s.notna().mean()) if n else 1.0,
                        "approximateNumDistinctValues": int(s.nunique(dropna=True))})
    return {"columns": columns, "rows": n, "device": st.get("device", "cpu") if cols else "cpu"}
