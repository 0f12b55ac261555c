"""Builder-style (JVM hsfs) feature-store API, so the Scala notebooks and the FS-tour job read the
same in Python.

Reference call shapes (re-provided here, not translated):
* ``fs.createFeatureGroup().name(..).version(..).description(..).timeTravelFormat(TimeTravelFormat.HUDI)
  .primaryKeys(Seq(..)).partitionKeys(..).hudiPrecombineKey(..).onlineEnabled(true)
  .statisticsConfig(new StatisticsConfig(true, true, true)).build()``
  (featurestore_tour/src/main/scala/io/hops/examples/featurestore_tour/featuregroups/ComputeFeatures.scala:108-133;
  notebooks/featurestore/hsfs/time_travel/time_travel_scala.ipynb:148-161)
* ``fs.createOnDemandFeatureGroup().name(..).query(..).storageConnector(sc).build()`` (ComputeFeatures.scala:179-191)
* ``fs.createTrainingDataset().name(..).dataFormat(DataFormat.TFRECORD).build(); td.save(query)`` (:312-328)
* ``Rule.createRule(RuleName.HAS_MIN).min(0).level(Level.WARNING).build()``,
  ``fs.createExpectation().name(..).features(..).rules(..).build()``,
  ``fg.getValidation(ts, ValidationTimeType.COMMIT_TIME)``
  (notebooks/featurestore/hsfs/data_validation/feature_validation_scala.ipynb:264-331,741-765)

Every builder ends in the same Python constructors the pythonic API uses; ``CamelCaseAPI``
gives the entity classes their camelCase method names (``commitDetails``, ``readChanges``,
``asOf``, ``selectAll`` …) by mapping them onto the snake_case implementations.
"""
from __future__ import annotations

import re

from . import rules as R
from .statistics import StatisticsConfig


def _snake(name: str) -> str:
    return re.sub(r"(?<!^)(?=[A-Z])", "_", name).lower()


class CamelCaseAPI:
    """``obj.commitDetails(...)`` -> ``obj.commit_details(...)`` for any snake_case method."""

    def __getattr__(self, name):
        if name.startswith("_") or not any(c.isupper() for c in name):
            raise AttributeError(name)
        sn = _snake(name)
        if sn == name:
            raise AttributeError(name)
        try:
            return object.__getattribute__(self, sn)
        except AttributeError:
            raise AttributeError(f"{type(self).__name__} has no attribute {name!r} (nor {sn!r})") from None


# ----------------------------------------------------------------------- enums
class TimeTravelFormat:
    HUDI = "HUDI"
    NONE = "NONE"


class DataFormat:
    CSV, TSV, TFRECORD, TFRECORDS, PARQUET, AVRO, ORC, NPY, HDF5, PETASTORM = (
        "csv", "tsv", "tfrecord", "tfrecords", "parquet", "avro", "orc", "npy", "hdf5", "petastorm")


class Level:
    WARNING, ERROR = "WARNING", "ERROR"


class ValidationTimeType:
    VALIDATION_TIME, COMMIT_TIME = "VALIDATION_TIME", "COMMIT_TIME"


class _RuleNames:
    def __getattr__(self, name):
        if name.upper() in R.RULES:
            return name.upper()
        raise AttributeError(f"unknown rule {name!r}; known: {sorted(R.RULES)}")

    def values(self):
        return sorted(R.RULES)


RuleName = _RuleNames()


# -------------------------------------------------------------------- builders
class _Builder:
    _fields: tuple = ()

    def __init__(self, **defaults):
        self._v = dict(defaults)

    def __getattr__(self, name):
        if name.startswith("_"):
            raise AttributeError(name)
        key = _snake(name)
        if key not in self._fields:
            raise AttributeError(f"{type(self).__name__} has no setter {name!r}")

        def setter(value=True):
            self._v[key] = list(value) if isinstance(value, (tuple, set)) else value
            return self

        return setter


class FeatureGroupBuilder(_Builder):
    _fields = ("name", "version", "description", "time_travel_format", "primary_keys", "partition_keys",
               "hudi_precombine_key", "online_enabled", "statistics_config", "validation_type", "expectations",
               "features", "event_time")

    def __init__(self, fs):
        super().__init__()
        self._fs = fs

    def build(self):
        v = self._v
        if "name" not in v:
            raise ValueError("createFeatureGroup(): .name(...) is required")
        return self._fs.create_feature_group(
            v["name"], version=v.get("version"), description=v.get("description", ""),
            online_enabled=bool(v.get("online_enabled", False)), time_travel_format=v.get("time_travel_format"),
            partition_key=v.get("partition_keys"), primary_key=v.get("primary_keys"),
            hudi_precombine_key=v.get("hudi_precombine_key"), features=v.get("features"),
            statistics_config=v.get("statistics_config"), validation_type=v.get("validation_type", "NONE"),
            expectations=v.get("expectations"), event_time=v.get("event_time"))


class OnDemandFeatureGroupBuilder(_Builder):
    _fields = ("name", "version", "description", "query", "storage_connector", "statistics_config", "features",
               "data_format", "path")

    def __init__(self, fs):
        super().__init__()
        self._fs = fs

    def build(self):
        v = self._v
        return self._fs.create_on_demand_feature_group(
            v["name"], v["storage_connector"], query=v.get("query"), version=v.get("version"),
            description=v.get("description", ""), features=v.get("features"),
            statistics_config=v.get("statistics_config"), data_format=v.get("data_format"), path=v.get("path"))


class TrainingDatasetBuilder(_Builder):
    _fields = ("name", "version", "description", "data_format", "coalesce", "storage_connector", "splits",
               "location", "seed", "statistics_config", "label")

    def __init__(self, fs):
        super().__init__()
        self._fs = fs

    def build(self):
        v = self._v
        return self._fs.create_training_dataset(
            v["name"], version=v.get("version"), description=v.get("description", ""),
            data_format=v.get("data_format", "tfrecords"), coalesce=bool(v.get("coalesce", False)),
            storage_connector=v.get("storage_connector"), splits=v.get("splits"), location=v.get("location", ""),
            seed=v.get("seed"), statistics_config=v.get("statistics_config"), label=v.get("label"))


class ExpectationBuilder(_Builder):
    _fields = ("name", "description", "features", "rules")

    def __init__(self, fs):
        super().__init__()
        self._fs = fs

    def build(self):
        v = self._v
        return self._fs.create_expectation(v["name"], description=v.get("description", ""),
                                           features=v.get("features"), rules=v.get("rules"))


class RuleBuilder(_Builder):
    _fields = ("level", "min", "max", "pattern", "accepted_type", "legal_values")

    def __init__(self, name):
        super().__init__(name=name)

    def build(self) -> R.Rule:
        v = self._v
        return R.Rule(v["name"], level=v.get("level", "ERROR"), min=v.get("min"), max=v.get("max"),
                      pattern=v.get("pattern"), accepted_type=v.get("accepted_type"),
                      legal_values=v.get("legal_values"))


def create_rule(name) -> RuleBuilder:
    """``Rule.createRule(RuleName.HAS_MIN)`` (feature_validation_scala.ipynb:312-331)."""
    return RuleBuilder(name)


def statistics_config(enabled=True, histograms=False, correlations=False, columns=None) -> StatisticsConfig:
    """``new StatisticsConfig(true, true, true)`` (ComputeFeatures.scala:114)."""
    return StatisticsConfig(enabled, histograms, correlations, columns)
