"""hsfs-compatible feature store (``import hops_examples_amd.featurestore as hsfs``).

See core.py for the reference call sites each piece re-provides.
"""
from .builders import DataFormat, Level, RuleName, ValidationTimeType, statistics_config
from .core import (Feature, FeatureGroup, FeatureStoreException, Filter, JoinType, Logic, OnDemandFeatureGroup,
                   Query, VersionWarning)
from .rules import RULES, Expectation, FeatureGroupValidation, Rule, ValidationError
from .statistics import StatisticsConfig
from .store import Connection, FeatureStore, StorageConnector, connection
from .training_dataset import TrainingDataset

__all__ = ["connection", "Connection", "FeatureStore", "FeatureGroup", "OnDemandFeatureGroup", "Feature", "Query",
           "Filter", "Logic", "JoinType", "TrainingDataset", "StorageConnector", "Rule", "Expectation",
           "FeatureGroupValidation", "ValidationError", "RULES", "StatisticsConfig", "VersionWarning",
           "FeatureStoreException", "TimeTravelFormat", "DataFormat", "Level", "RuleName", "ValidationTimeType",
           "HopsworksConnection", "statistics_config"]


from .builders import TimeTravelFormat  # noqa: E402
from .store import Connection as HopsworksConnection  # noqa: E402  (JVM name: HopsworksConnection.builder...build)


class ValidationType:
    STRICT, WARNING, ALL, NONE = "STRICT", "WARNING", "ALL", "NONE"
