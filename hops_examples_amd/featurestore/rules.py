"""Data-validation rules, expectations and the rule evaluator (hsfs + Deequ surface).

Rule catalogue and its printed form: notebooks/featurestore/hsfs/data_validation/feature_validation_python.ipynb:218-242.
Validation result JSON (``validationId``, ``validationTime``, ``expectationResults`` …): same notebook :498-566.
Failure message "Value: 2022.0 does not meet the constraint requirement! HAS_MAX": :655.
Validation types STRICT / WARNING / ALL / NONE: :686-691.

Numeric aggregates (count / min / max / mean / sum / stddev and the IS_NON_NEGATIVE / IS_POSITIVE
fractions) come from ONE fp64 GPU column-statistics launch over every numeric feature the rules
touch (stats.hip ``colstats64_k``; Deequ computes in double too) when the frame has at least
``GPU_MIN_ROWS`` rows and a GPU is present, otherwise from numpy.  ``validate`` reports which.
"""
from __future__ import annotations

import math
import re
import time

import numpy as np
import pandas as pd

RULE_DEFINITIONS = [
    ("HAS_SIZE", "VALUE", "Integral", "A rule that asserts the number of rows of the dataframe"),
    ("HAS_MEAN", "VALUE", "Fractional", "A rule that asserts on the mean of the feature"),
    ("HAS_DATATYPE", "ACCEPTED_TYPE", "String", ""),
    ("HAS_SUM", "VALUE", "Fractional", "A rule that asserts on the sum of the feature"),
    ("IS_LESS_THAN", "LEGAL_VALUES", "Fractional", ""),
    ("IS_GREATER_THAN_OR_EQUAL_TO", "LEGAL_VALUES", "Fractional", ""),
    ("HAS_STANDARD_DEVIATION", "VALUE", "Fractional", ""),
    ("HAS_PATTERN", "PATTERN", "String", ""),
    ("HAS_NUMBER_OF_DISTINCT_VALUES", "VALUE", "Integral", ""),
    ("HAS_MAX", "VALUE", "Fractional", "A rule that asserts on the max of the feature"),
    ("IS_CONTAINED_IN", "LEGAL_VALUES", "String", ""),
    ("IS_NON_NEGATIVE", "VALUE", "Fractional", ""),
    ("IS_POSITIVE", "VALUE", "Boolean", ""),
    ("HAS_MUTUAL_INFORMATION", "LEGAL_VALUES", "Fractional", ""),
    ("HAS_UNIQUE_VALUE_RATIO", "VALUE", "Fractional", ""),
    ("IS_GREATER_THAN", "LEGAL_VALUES", "Fractional", ""),
    ("HAS_COMPLETENESS", "VALUE", "Fractional", ""),
    ("HAS_ENTROPY", "VALUE", "Fractional", ""),
    ("HAS_MIN", "VALUE", "Fractional", "A rule that asserts on the min of the feature"),
    ("HAS_UNIQUENESS", "VALUE", "Fractional", ""),
    ("HAS_DISTINCTNESS", "VALUE", "Fractional", ""),
    ("HAS_CORRELATION", "LEGAL_VALUES", "Fractional", ""),
    ("HAS_APPROX_QUANTILE", "VALUE", "Fractional", ""),
    ("HAS_APPROX_COUNT_DISTINCT", "VALUE", "Fractional", ""),
    ("IS_LESS_THAN_OR_EQUAL_TO", "LEGAL_VALUES", "Fractional", ""),
]


class RuleDefinition:
    def __init__(self, name, predicate, value_type, description):
        self.name, self.predicate, self.value_type, self.description = name, predicate, value_type, description

    def to_dict(self):
        return {"name": self.name, "predicate": self.predicate, "valueType": self.value_type,
                "description": self.description}

    def __repr__(self):
        return str(self.to_dict())


RULES = {r[0]: RuleDefinition(*r) for r in RULE_DEFINITIONS}


class Rule:
    """A constraint on a feature: ``Rule(name='HAS_MIN', level='WARNING', min=0)``."""

    def __init__(self, name: str, level: str = "ERROR", min=None, max=None, pattern=None, accepted_type=None,
                 legal_values=None):
        name = name.upper()
        if name not in RULES:
            raise ValueError(f"unknown rule {name!r}")
        self.name, self.level = name, level.upper()
        self.min = None if min is None else float(min)
        self.max = None if max is None else float(max)
        self.pattern, self.accepted_type, self.legal_values = pattern, accepted_type, legal_values

    def to_dict(self):
        d = {"level": self.level, "name": self.name}
        for k in ("min", "max", "pattern"):
            if getattr(self, k) is not None:
                d[k] = getattr(self, k)
        if self.accepted_type is not None:
            d["acceptedType"] = self.accepted_type
        if self.legal_values is not None:
            d["legalValues"] = list(self.legal_values)
        return d

    @classmethod
    def from_dict(cls, d):
        return cls(d["name"], d.get("level", "ERROR"), d.get("min"), d.get("max"), d.get("pattern"),
                   d.get("acceptedType"), d.get("legalValues"))

    @staticmethod
    def createRule(name):  # noqa: N802  (JVM: Rule.createRule(RuleName.HAS_MIN).min(0).level(..).build())
        from .builders import RuleBuilder

        return RuleBuilder(name)

    def __repr__(self):
        return (f"Rule{{name={self.name}, level={self.level}, min={self.min}, max={self.max}, "
                f"pattern='{self.pattern}', acceptedType={self.accepted_type}, legalValues={self.legal_values}}}")


class Expectation:
    def __init__(self, name: str, features: list[str], rules: list[Rule], description: str = "", store=None):
        self.name, self.features, self.rules, self.description = name, list(features), list(rules), description
        self._store = store

    def save(self):
        if self._store is not None:
            self._store._save_expectation(self)
        return self

    def to_dict(self):
        return {"features": self.features, "rules": [r.to_dict() for r in self.rules],
                "description": self.description, "name": self.name}

    @classmethod
    def from_dict(cls, d, store=None):
        return cls(d["name"], d["features"], [Rule.from_dict(r) for r in d["rules"]], d.get("description", ""),
                   store)

    def __repr__(self):
        return f"Expectation{{name='{self.name}', features={self.features}, rules={self.rules}}}"


class ValidationResult:
    def __init__(self, status, message, value, feature, rule):
        self.status, self.message, self.value, self.feature, self.rule = status, message, value, feature, rule

    def to_dict(self):
        return {"feature": self.feature, "message": self.message, "rule": self.rule.to_dict(), "status": self.status,
                "value": self.value}


class ExpectationResult:
    def __init__(self, expectation, results):
        self.expectation, self.results = expectation, results
        self.status = _worst([r.status for r in results])

    def to_dict(self):
        return {"expectation": self.expectation.to_dict(), "results": [r.to_dict() for r in self.results],
                "status": self.status}


class FeatureGroupValidation:
    def __init__(self, validation_id, validation_time, expectation_results, commit_time=None):
        self.validation_id, self.validation_time = validation_id, validation_time
        self.expectation_results, self.commit_time = expectation_results, commit_time
        self.status = _worst([e.status for e in expectation_results]) if expectation_results else "SUCCESS"

    def to_dict(self):
        d = {"validationId": self.validation_id, "validationTime": self.validation_time,
             "expectationResults": [e.to_dict() for e in self.expectation_results]}
        if self.commit_time is not None:
            d["commitTime"] = self.commit_time
        d["status"] = self.status
        return d

    def __repr__(self):
        return str(self.to_dict())


_ORDER = {"SUCCESS": 0, "WARNING": 1, "FAILURE": 2}


def _worst(statuses):
    return max(statuses, key=lambda s: _ORDER[s]) if statuses else "SUCCESS"


class ValidationError(Exception):
    """Raised when STRICT/WARNING validation rejects an insert (the reference's HTTP 417)."""

    def __init__(self, validation: FeatureGroupValidation):
        fails = [f"ExpectationResult{{status={e.status.title()}, results=[" + ", ".join(
            f"ValidationResult{{status={r.status.title()}, message='{r.message}', value='{r.value}', "
            f"feature='{r.feature}', rule={r.rule!r}}}" for r in e.results) + f"], expectation={e.expectation!r}}}"
            for e in validation.expectation_results if e.status != "SUCCESS"]
        super().__init__("HTTP code: 417, HTTP reason: Expectation Failed, error msg: Feature group validation "
                         "checks did not pass, will not persist validation results., user msg: Results: [" +
                         ", ".join(fails) + "]")
        self.validation = validation


# ------------------------------------------------------------------ evaluator
def _num(s: pd.Series) -> np.ndarray:
    return pd.to_numeric(s, errors="coerce").to_numpy(np.float64)


def _entropy(s: pd.Series) -> float:
    p = s.value_counts(normalize=True, dropna=True).to_numpy()
    return float(-(p * np.log(p)).sum()) if len(p) else 0.0


GPU_MIN_ROWS = 100_000
_NUMERIC_RULES = ("HAS_MIN", "HAS_MAX", "HAS_MEAN", "HAS_SUM", "HAS_STANDARD_DEVIATION", "IS_NON_NEGATIVE",
                  "IS_POSITIVE")


def prefill_stats(df: pd.DataFrame, feats, stats_cache: dict, device=None) -> str:
    """Aggregates of every numeric feature in ``feats`` in one pass (GPU fp64 kernel on large frames);
    returns the device used ('gpu' / 'cpu')."""
    feats = [f for f in dict.fromkeys(feats) if f in df.columns and f not in stats_cache]
    if not feats:
        return stats_cache.get("_device", "cpu")
    x = np.stack([_num(df[f]) for f in feats], 1) if len(df) else np.zeros((0, len(feats)))
    use_gpu = False
    try:
        import torch

        use_gpu = torch.cuda.is_available() and (
            (device is not None and torch.device(device).type == "cuda") or (device is None and len(df) >= GPU_MIN_ROWS))
    except Exception:  # pragma: no cover
        pass
    if use_gpu and len(df):
        import torch

        from ..ops import kernels as K

        xt = torch.from_numpy(np.ascontiguousarray(x)).pin_memory().cuda(non_blocking=True)
        st = K.column_stats64(xt).cpu().numpy()
        dev = "gpu"
    else:
        valid = ~np.isnan(x)
        xz = np.where(valid, x, 0.0)
        st = np.stack([valid.sum(0), xz.sum(0), (xz * xz).sum(0), np.where(valid, x, np.inf).min(0, initial=np.inf),
                       np.where(valid, x, -np.inf).max(0, initial=-np.inf), (valid & (xz >= 0)).sum(0),
                       (valid & (xz > 0)).sum(0)], 1).astype(np.float64)
        dev = "cpu"
    for j, f in enumerate(feats):
        cnt, s, sq, mn, mx, nn, npos = (float(v) for v in st[j])
        mean = s / cnt if cnt else math.nan
        std = math.sqrt(max(sq / cnt - mean * mean, 0.0)) if cnt else math.nan
        stats_cache[f] = {"count": int(cnt), "n": len(df), "min": mn if cnt else math.nan,
                          "max": mx if cnt else math.nan, "sum": s, "mean": mean, "std": std,
                          "nonneg": nn / cnt if cnt else 1.0, "pos": npos / cnt if cnt else 1.0}
    stats_cache["_device"] = dev
    return dev


def _metric(rule: Rule, df: pd.DataFrame, feat: str, stats_cache: dict):
    """The measured value for rule on feature (None for row-wise predicates)."""
    n = rule.name
    s = df[feat] if feat in df.columns else None
    if n == "HAS_SIZE":
        return float(len(df))
    if s is None:
        raise KeyError(f"feature {feat!r} not in dataframe")
    if n == "HAS_COMPLETENESS":
        return float(s.notna().sum() / max(1, len(s)))
    if n in _NUMERIC_RULES:
        if feat not in stats_cache:
            prefill_stats(df, [feat], stats_cache)
        st = stats_cache[feat]
        return {"HAS_MIN": st["min"], "HAS_MAX": st["max"], "HAS_MEAN": st["mean"], "HAS_SUM": st["sum"],
                "HAS_STANDARD_DEVIATION": st["std"], "IS_NON_NEGATIVE": st["nonneg"], "IS_POSITIVE": st["pos"]}[n]
    if n == "HAS_NUMBER_OF_DISTINCT_VALUES" or n == "HAS_APPROX_COUNT_DISTINCT":
        return float(s.nunique(dropna=True))
    if n == "HAS_DISTINCTNESS":
        return float(s.nunique(dropna=True) / max(1, s.notna().sum()))
    if n == "HAS_UNIQUENESS":
        vc = s.value_counts(dropna=True)
        return float((vc == 1).sum() / max(1, s.notna().sum()))
    if n == "HAS_UNIQUE_VALUE_RATIO":
        vc = s.value_counts(dropna=True)
        return float((vc == 1).sum() / max(1, len(vc)))
    if n == "HAS_ENTROPY":
        return _entropy(s)
    if n == "HAS_APPROX_QUANTILE":
        q = 0.5 if rule.legal_values is None else float(rule.legal_values[0])
        return float(np.nanquantile(_num(s), q))
    if n == "HAS_PATTERN":
        pat = re.compile(rule.pattern or ".*")
        vals = s.dropna().astype(str)
        return float(vals.map(lambda v: bool(pat.fullmatch(v))).mean()) if len(vals) else 1.0
    if n == "HAS_DATATYPE":
        vals = s.dropna()
        t = (rule.accepted_type or "").lower()

        def ok(v):
            if t in ("integral", "integer", "int"):
                return float(v).is_integer() if isinstance(v, (int, float, np.number)) else str(v).lstrip("-").isdigit()
            if t in ("fractional", "float", "double"):
                try:
                    float(v)
                    return True
                except (TypeError, ValueError):
                    return False
            if t == "boolean":
                return str(v).lower() in ("true", "false", "0", "1")
            return isinstance(v, str)

        return float(vals.map(ok).mean()) if len(vals) else 1.0
    if n == "IS_CONTAINED_IN":
        legal = set(map(str, rule.legal_values or []))
        vals = s.dropna().astype(str)
        return float(vals.isin(legal).mean()) if len(vals) else 1.0
    if n in ("IS_LESS_THAN", "IS_LESS_THAN_OR_EQUAL_TO", "IS_GREATER_THAN", "IS_GREATER_THAN_OR_EQUAL_TO",
             "HAS_CORRELATION", "HAS_MUTUAL_INFORMATION"):
        other = (rule.legal_values or [None])[0]
        if other is None or other not in df.columns:
            raise ValueError(f"{n} needs legal_values=[<other feature>]")
        a, b = _num(s), _num(df[other])
        m = ~(np.isnan(a) | np.isnan(b))
        a, b = a[m], b[m]
        if n == "HAS_CORRELATION":
            return float(np.corrcoef(a, b)[0, 1]) if len(a) > 1 else math.nan
        if n == "HAS_MUTUAL_INFORMATION":
            ja = pd.Series(list(zip(s.astype(str), df[other].astype(str))))
            return _entropy(s.astype(str)) + _entropy(df[other].astype(str)) - _entropy(ja)
        op = {"IS_LESS_THAN": np.less, "IS_LESS_THAN_OR_EQUAL_TO": np.less_equal, "IS_GREATER_THAN": np.greater,
              "IS_GREATER_THAN_OR_EQUAL_TO": np.greater_equal}[n]
        return float(op(a, b).mean()) if len(a) else 1.0
    raise NotImplementedError(n)


def check(rule: Rule, value) -> bool:
    if value is None or (isinstance(value, float) and math.isnan(value)):
        return False
    if rule.min is not None and value < rule.min:
        return False
    if rule.max is not None and value > rule.max:
        return False
    return True


def validate(df: pd.DataFrame, expectations: list[Expectation], validation_id: int,
             commit_time=None) -> FeatureGroupValidation:
    cache: dict = {}
    # one aggregate pass (GPU fp64 kernel on large frames) over every feature a numeric rule reads
    prefill_stats(df, [f for e in expectations for r in e.rules if r.name in _NUMERIC_RULES for f in e.features],
                  cache)
    results = []
    for e in expectations:
        rs = []
        # rules are evaluated rule-major like the reference output (all features for a rule)
        for rule in sorted(e.rules, key=lambda r: r.name, reverse=True):
            feats = e.features if rule.name != "HAS_SIZE" else (e.features[:1] or ["*"])
            for f in feats:
                v = _metric(rule, df, f, cache)
                if rule.min is None and rule.max is None and rule.name in ("IS_NON_NEGATIVE", "IS_POSITIVE",
                                                                           "HAS_PATTERN", "HAS_DATATYPE",
                                                                           "IS_CONTAINED_IN", "IS_LESS_THAN",
                                                                           "IS_LESS_THAN_OR_EQUAL_TO",
                                                                           "IS_GREATER_THAN",
                                                                           "IS_GREATER_THAN_OR_EQUAL_TO"):
                    ok = v >= 1.0  # row predicates: all rows must satisfy unless a fraction is given
                else:
                    ok = check(rule, v)
                status = "SUCCESS" if ok else ("WARNING" if rule.level == "WARNING" else "FAILURE")
                msg = "Success" if ok else f"Value: {v} does not meet the constraint requirement! {rule.name}"
                rs.append(ValidationResult(status, msg, str(v), f, rule))
        results.append(ExpectationResult(e, rs))
    v = FeatureGroupValidation(validation_id, int(time.time() * 1000), results, commit_time)
    v.aggregates_device = cache.get("_device", "cpu")
    return v
