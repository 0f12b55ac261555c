"""Chicago-taxi Transform: analyze on the full training split, apply to every split.

tf.Transform's two halves (the public TFX taxi ``preprocessing_fn`` the reference README points to,
README.md:99-112):

* **analyze** (one pass over the training data, GPU when present):
  * z-score statistics of the dense columns — count / sum / sum of squares from the ``stats.hip``
    column-statistics kernel over the missing-filled values (``tft.scale_to_z_score``: population
    variance, unit scale when the variance is 0);
  * 10-quantile bucket boundaries of the lat/long columns — a 4096-bin ``stats.hip`` histogram per
    column between its min and max, inverted on the host (boundaries exact to 1/4096 of the range;
    ``tft.bucketize`` also uses an approximate quantile sketch);
  * vocabularies of the string columns — top 1000 by frequency (ties by value), missing values
    filled with '' first as tft does; a value outside the vocabulary maps to one of 10 OOV buckets
    by a stable CRC32 hash (tft: farmhash fingerprint) at ids 1000..1009, so the wide model's
    one-hot layout is fixed.
* **apply** (``transform.hip`` ``taxi_transform_k``: one launch for every numeric column of every
  row): z-scored dense block, the 13 wide ids already offset into the wide&deep model's
  concatenated one-hot space (``models.widedeep.wide_offsets``), and the big-tipper label.

``TaxiTransform`` is the transform_fn: JSON-serialisable (``save`` / ``load``), applied identically
at training and serving time.  ``apply_numpy`` is the fp32 host reference the tests hold the GPU
path to.
"""
from __future__ import annotations

import json
import zlib
from pathlib import Path

import numpy as np
import pandas as pd

from ..models.widedeep import (BUCKET_FEATURE_KEYS, CATEGORICAL_FEATURE_KEYS, DENSE_FLOAT_FEATURE_KEYS,
                               FEATURE_BUCKET_COUNT, LABEL_KEY, MAX_CATEGORICAL_FEATURE_VALUES, OOV_SIZE,
                               VOCAB_FEATURE_KEYS, VOCAB_SIZE, wide_offsets)
from .taxi import FARE_KEY, TIP_FRACTION

NUMERIC = DENSE_FLOAT_FEATURE_KEYS + BUCKET_FEATURE_KEYS + CATEGORICAL_FEATURE_KEYS + [FARE_KEY, LABEL_KEY]
MAX_BOUNDS = 31  # transform.hip kMaxBounds
HIST_BINS = 4096


def _col(name: str) -> int:
    return NUMERIC.index(name)


def raw_matrix(df: pd.DataFrame) -> np.ndarray:
    """The raw numeric columns as fp32 [n, len(NUMERIC)] (NaN = missing); a column absent from a
    serving request (e.g. the label) reads as missing."""
    out = np.full((len(df), len(NUMERIC)), np.nan, np.float32)
    for j, c in enumerate(NUMERIC):
        if c in df.columns:
            out[:, j] = pd.to_numeric(df[c], errors="coerce").to_numpy(np.float32)
    return out


def _oov(value: str) -> int:
    return VOCAB_SIZE + zlib.crc32(value.encode()) % OOV_SIZE


class TaxiTransform:
    """The analyzed transform (tf.Transform's transform_fn)."""

    def __init__(self, mean, std, boundaries, vocabs, rows: int = 0):
        self.mean = [float(v) for v in mean]
        self.std = [float(v) for v in std]
        self.boundaries = [[float(b) for b in bs] for bs in boundaries]
        self.vocabs = [list(v) for v in vocabs]
        self.rows = int(rows)
        self._index = [{s: i for i, s in enumerate(v)} for v in self.vocabs]

    # ------------------------------------------------------------ persistence
    def to_dict(self) -> dict:
        return {"dense_keys": DENSE_FLOAT_FEATURE_KEYS, "mean": self.mean, "std": self.std,
                "bucket_keys": BUCKET_FEATURE_KEYS, "boundaries": self.boundaries, "vocab_keys": VOCAB_FEATURE_KEYS,
                "vocabularies": self.vocabs, "vocab_size": VOCAB_SIZE, "num_oov_buckets": OOV_SIZE,
                "categorical_keys": CATEGORICAL_FEATURE_KEYS, "categorical_cardinality": MAX_CATEGORICAL_FEATURE_VALUES,
                "wide_offsets": [int(v) for v in wide_offsets()], "label": f"{LABEL_KEY} > {TIP_FRACTION} * {FARE_KEY}",
                "analyzed_rows": self.rows}

    def save(self, path) -> str:
        p = Path(path)
        p.parent.mkdir(parents=True, exist_ok=True)
        p.write_text(json.dumps(self.to_dict()))
        return str(p)

    @classmethod
    def load(cls, path) -> "TaxiTransform":
        d = json.loads(Path(path).read_text())
        return cls(d["mean"], d["std"], d["boundaries"], d["vocabularies"], d.get("analyzed_rows", 0))

    # ------------------------------------------------------------ apply
    def vocab_ids(self, df: pd.DataFrame) -> np.ndarray:
        """Host vocabulary lookup: int32 [n, len(VOCAB_FEATURE_KEYS)]."""
        out = np.empty((len(df), len(VOCAB_FEATURE_KEYS)), np.int32)
        for j, c in enumerate(VOCAB_FEATURE_KEYS):
            idx = self._index[j]
            vals = df[c].fillna("").astype(str) if c in df.columns else pd.Series([""] * len(df))
            uniq = pd.unique(vals)
            m = {u: idx.get(u, _oov(u)) for u in uniq}
            out[:, j] = vals.map(m).to_numpy(np.int32)
        return out

    def _spec(self):
        nd, nb, ni, nv = (len(DENSE_FLOAT_FEATURE_KEYS), len(BUCKET_FEATURE_KEYS), len(CATEGORICAL_FEATURE_KEYS),
                          len(VOCAB_FEATURE_KEYS))
        ints = [len(NUMERIC), nd, nb, ni, nv, _col(FARE_KEY), _col(LABEL_KEY)]
        ints += [_col(c) for c in DENSE_FLOAT_FEATURE_KEYS]
        ints += [_col(c) for c in BUCKET_FEATURE_KEYS]
        ints += [len(b) for b in self.boundaries]
        ints += [_col(c) for c in CATEGORICAL_FEATURE_KEYS]
        ints += list(MAX_CATEGORICAL_FEATURE_VALUES)
        ints += [VOCAB_SIZE + OOV_SIZE] * nv
        inv = [1.0 / s if s > 0 else 1.0 for s in self.std]
        flts = [TIP_FRACTION] + self.mean + inv
        for b in self.boundaries:
            flts += b + [0.0] * (MAX_BOUNDS - len(b))
        return ints, flts, [int(v) for v in wide_offsets()]

    def apply(self, df: pd.DataFrame, device=None, with_label: bool = True):
        """(dense fp32 [n, 3], cat int64 [n, 13] global wide ids, label fp32 [n, 1] | None) as torch
        tensors on ``device`` — the GPU kernel on a CUDA device, the numpy reference otherwise."""
        import torch

        dev = torch.device(device) if device is not None else (
            torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu"))
        if dev.type != "cuda":
            d, c, y = apply_numpy(self, df, with_label)
            return torch.from_numpy(d), torch.from_numpy(c), (torch.from_numpy(y) if y is not None else None)
        from ..ops import kernels as K

        raw = torch.from_numpy(raw_matrix(df)).pin_memory().to(dev, non_blocking=True)
        vids = torch.from_numpy(self.vocab_ids(df)).pin_memory().to(dev, non_blocking=True)
        ints, flts, offs = self._spec()
        if not with_label:
            ints[5] = ints[6] = -1
        return K.taxi_transform(raw, vids, ints, flts, offs, len(DENSE_FLOAT_FEATURE_KEYS), len(offs), with_label)


def apply_numpy(t: TaxiTransform, df: pd.DataFrame, with_label: bool = True):
    """Host fp32 reference of transform.hip (same fill / bucket / identity / label rules)."""
    raw = raw_matrix(df)
    filled = np.nan_to_num(raw, nan=0.0)
    dense = np.stack([(filled[:, _col(c)] - np.float32(m)) * np.float32(1.0 / s if s > 0 else 1.0)
                      for c, m, s in zip(DENSE_FLOAT_FEATURE_KEYS, t.mean, t.std)], 1).astype(np.float32)
    offs = wide_offsets()
    cols = []
    for c, b in zip(BUCKET_FEATURE_KEYS, t.boundaries):
        v = filled[:, _col(c)]
        cols.append((np.asarray(b, np.float32)[None, :] <= v[:, None]).sum(1))
    vids = t.vocab_ids(df)
    for j in range(len(VOCAB_FEATURE_KEYS)):
        v = vids[:, j].astype(np.int64)
        cols.append(np.where((v < 0) | (v >= VOCAB_SIZE + OOV_SIZE), 0, v))
    for c, card in zip(CATEGORICAL_FEATURE_KEYS, MAX_CATEGORICAL_FEATURE_VALUES):
        v = raw[:, _col(c)]
        iv = np.where(np.isnan(v), 0, v).astype(np.int64)
        cols.append(np.where((iv < 0) | (iv >= card), 0, iv))
    cat = np.stack(cols, 1).astype(np.int64) + offs[None, :]
    label = None
    if with_label:
        fare, tips = raw[:, _col(FARE_KEY)], raw[:, _col(LABEL_KEY)]
        label = np.where(np.isnan(fare), 0.0, (np.nan_to_num(tips) > np.float32(TIP_FRACTION) * fare)).astype(
            np.float32)[:, None]
    return dense, cat, label


def _quantile_bounds_from_hist(hist: np.ndarray, lo: float, hi: float, n: int, k: int) -> list[float]:
    """k-1 interior quantile boundaries from a histogram over [lo, hi] (linear within a bin)."""
    if n <= 0 or hi <= lo:
        return [float(lo)] * (k - 1)
    bins = len(hist)
    cdf = np.cumsum(hist, dtype=np.float64)
    out = []
    for q in range(1, k):
        target = q * n / k
        b = int(np.searchsorted(cdf, target, side="left"))
        b = min(b, bins - 1)
        prev = cdf[b - 1] if b > 0 else 0.0
        frac = 0.0 if hist[b] == 0 else (target - prev) / hist[b]
        out.append(float(lo + (hi - lo) * (b + frac) / bins))
    return out


def analyze(df: pd.DataFrame, device=None, bins: int = HIST_BINS) -> TaxiTransform:
    """One analysis pass over the training split (see the module docstring)."""
    import torch

    raw = raw_matrix(df)
    filled = np.nan_to_num(raw, nan=0.0)
    dcols = [_col(c) for c in DENSE_FLOAT_FEATURE_KEYS]
    bcols = [_col(c) for c in BUCKET_FEATURE_KEYS]
    n = len(df)
    use_gpu = (device is None or torch.device(device).type == "cuda") and torch.cuda.is_available() and n > 0
    if use_gpu:
        from ..ops import kernels as K

        dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        x = torch.from_numpy(np.ascontiguousarray(filled[:, dcols + bcols])).pin_memory().to(dev, non_blocking=True)
        st = K.column_stats(x).double()
        cnt, s, sq, mn, mx = (st[:, i] for i in range(5))
        mean = s / cnt.clamp_min(1)
        var = (sq / cnt.clamp_min(1) - mean * mean).clamp_min(0)
        nd = len(dcols)
        xb = x[:, nd:].contiguous()
        hist = K.column_hist(xb, mn[nd:].float().contiguous(), mx[nd:].float().contiguous(), bins).cpu().numpy()
        mean_h, std_h = mean[:nd].cpu().numpy(), var[:nd].sqrt().cpu().numpy()
        lo, hi = mn[nd:].cpu().numpy(), mx[nd:].cpu().numpy()
    else:
        xd = filled[:, dcols].astype(np.float64)
        mean_h = xd.mean(0) if n else np.zeros(len(dcols))
        std_h = xd.std(0) if n else np.ones(len(dcols))
        xb = filled[:, bcols]
        lo, hi = (xb.min(0), xb.max(0)) if n else (np.zeros(len(bcols)), np.zeros(len(bcols)))
        hist = np.zeros((len(bcols), bins), np.int64)
        for j in range(len(bcols)):
            if hi[j] > lo[j]:
                idx = np.clip(((xb[:, j] - lo[j]) / (hi[j] - lo[j]) * bins).astype(np.int64), 0, bins - 1)
                hist[j] = np.bincount(idx, minlength=bins)
            else:
                hist[j, 0] = n
    bounds = [_quantile_bounds_from_hist(hist[j], float(lo[j]), float(hi[j]), n, FEATURE_BUCKET_COUNT)
              for j in range(len(bcols))]
    vocabs = []
    for c in VOCAB_FEATURE_KEYS:
        vc = df[c].fillna("").astype(str).value_counts()
        order = sorted(vc.items(), key=lambda kv: (-kv[1], kv[0]))[:VOCAB_SIZE]
        vocabs.append([k for k, _ in order])
    return TaxiTransform(mean_h, std_h, bounds, vocabs, rows=n)


def transformed_frame(dense, cat, label) -> pd.DataFrame:
    """Transformed examples as a flat frame (dense_0.., wide_0.., label) for a Parquet training dataset."""
    d = dense.cpu().numpy() if hasattr(dense, "cpu") else dense
    c = cat.cpu().numpy() if hasattr(cat, "cpu") else cat
    cols = {f"dense_{j}": d[:, j] for j in range(d.shape[1])}
    cols.update({f"wide_{j}": c[:, j].astype(np.int64) for j in range(c.shape[1])})
    if label is not None:
        y = label.cpu().numpy() if hasattr(label, "cpu") else label
        cols["label"] = y[:, 0].astype(np.float32)
    return pd.DataFrame(cols)
