"""What-If probing without the widget.

The reference's What-If Tool notebooks (notebooks/ml/Plotting/What_If_Tool_Notebook.ipynb:43-651,
notebooks/featurestore/feature-bias/feature-bias-whatif.ipynb:661-663) hand a trained census
classifier to the interactive WIT widget, whose views are: edit one datapoint and re-infer, the
nearest counterfactual (closest example with the other prediction), partial dependence of the score
on one feature, and per-slice performance / fairness with a movable threshold.  :class:`WhatIfProbe`
computes the same views programmatically from any ``predict(df) -> scores`` function; every view
returns plain data, and ``*_svg`` helpers draw them with :mod:`hops_examples_amd.plotting`.
"""
from __future__ import annotations

import numpy as np
import pandas as pd

from . import plotting


class WhatIfProbe:
    def __init__(self, predict, examples: pd.DataFrame, label: str | None = None, threshold: float = 0.5):
        """``predict(df) -> np.ndarray`` of scores (positive-class probabilities); ``examples`` the
        datapoints under study (the label column, if given, is never passed to ``predict``)."""
        self._predict = predict
        self.examples = examples.reset_index(drop=True)
        self.label = label
        self.threshold = float(threshold)
        self.features = [c for c in self.examples.columns if c != label]
        self.scores = self.predict(self.examples)

    def predict(self, df: pd.DataFrame) -> np.ndarray:
        return np.asarray(self._predict(df[self.features]), dtype=np.float64).reshape(-1)

    # ------------------------------------------------------------ datapoint editor
    def edit(self, index: int, **changes) -> dict:
        """Re-infer one datapoint with feature values changed: {'before', 'after', 'delta', 'row'}."""
        row = self.examples.iloc[[index]].copy()
        for k, v in changes.items():
            if k not in self.features:
                raise KeyError(f"unknown feature {k!r}")
            row[k] = v
        after = float(self.predict(row)[0])
        before = float(self.scores[index])
        return {"before": before, "after": after, "delta": after - before, "row": row.iloc[0].to_dict()}

    # ------------------------------------------------------------ counterfactuals
    def _distance(self, index: int) -> np.ndarray:
        """WIT's L1 distance: numeric features scaled by their std, categorical mismatch = 1."""
        ref = self.examples.iloc[index]
        d = np.zeros(len(self.examples))
        for f in self.features:
            col = self.examples[f]
            if pd.api.types.is_numeric_dtype(col):
                sd = float(col.std()) or 1.0
                d += np.abs(col.to_numpy(np.float64) - float(ref[f])) / sd
            else:
                d += (col.to_numpy() != ref[f]).astype(np.float64)
        return d

    def nearest_counterfactual(self, index: int) -> dict | None:
        """The closest example whose thresholded prediction differs from datapoint ``index``'s."""
        pos = self.scores >= self.threshold
        other = np.flatnonzero(pos != pos[index])
        if not len(other):
            return None
        d = self._distance(index)
        j = int(other[np.argmin(d[other])])
        diff = {f: (self.examples.iloc[index][f], self.examples.iloc[j][f]) for f in self.features
                if self.examples.iloc[index][f] != self.examples.iloc[j][f]}
        return {"index": j, "distance": float(d[j]), "score": float(self.scores[j]), "differs_in": diff}

    # ------------------------------------------------------------ partial dependence
    def partial_dependence(self, feature: str, values=None, num: int = 20) -> pd.DataFrame:
        """Mean score over all examples with ``feature`` set to each value (all categories of a
        categorical feature; ``num`` points over the observed range of a numeric one)."""
        col = self.examples[feature]
        if values is None:
            values = (np.linspace(float(col.min()), float(col.max()), num) if pd.api.types.is_numeric_dtype(col)
                      else sorted(col.unique()))
        rows = []
        for v in values:
            s = self.predict(self.examples.assign(**{feature: v}))
            rows.append({feature: v, "mean_score": float(s.mean()), "positive_rate": float((s >= self.threshold).mean())})
        return pd.DataFrame(rows)

    # ------------------------------------------------------------ performance & fairness
    def slice_metrics(self, feature: str, threshold: float | None = None) -> pd.DataFrame:
        """Per-value count, positive rate, and (with a label) accuracy / TPR / FPR — WIT's
        'Performance & Fairness' table for one slicing feature."""
        t = self.threshold if threshold is None else float(threshold)
        pred = self.scores >= t
        rows = []
        for v, idx in self.examples.groupby(feature).indices.items():
            r = {feature: v, "count": int(len(idx)), "positive_rate": float(pred[idx].mean())}
            if self.label is not None:
                y = self.examples[self.label].to_numpy()[idx] > 0.5
                p = pred[idx]
                r["accuracy"] = float((p == y).mean())
                r["tpr"] = float(p[y].mean()) if y.any() else float("nan")
                r["fpr"] = float(p[~y].mean()) if (~y).any() else float("nan")
            rows.append(r)
        return pd.DataFrame(rows)

    def equal_opportunity_thresholds(self, feature: str, target_tpr: float = 0.8) -> dict:
        """Per-slice threshold that reaches ``target_tpr`` (WIT's 'equal opportunity' optimisation)."""
        if self.label is None:
            raise ValueError("needs a label column")
        out = {}
        for v, idx in self.examples.groupby(feature).indices.items():
            y = self.examples[self.label].to_numpy()[idx] > 0.5
            s = np.sort(self.scores[idx][y])[::-1]
            out[v] = float(s[min(len(s) - 1, int(np.ceil(target_tpr * len(s))) - 1)]) if len(s) else self.threshold
        return out

    # ------------------------------------------------------------ drawings
    def partial_dependence_svg(self, feature: str, **kw) -> str:
        pd_ = self.partial_dependence(feature, **kw)
        if pd.api.types.is_numeric_dtype(pd_[feature]):
            return plotting.line(pd_[feature].to_numpy(), {"mean score": pd_["mean_score"].to_numpy()},
                                 title=f"partial dependence on {feature}", xlabel=feature, ylabel="score")
        return plotting.bar([str(v) for v in pd_[feature]], pd_["mean_score"].to_numpy(),
                            title=f"partial dependence on {feature}", ylabel="mean score")

    def slice_svg(self, feature: str, metric: str = "positive_rate") -> str:
        m = self.slice_metrics(feature)
        return plotting.bar([str(v) for v in m[feature]], m[metric].to_numpy(), title=f"{metric} by {feature}",
                            ylabel=metric)
