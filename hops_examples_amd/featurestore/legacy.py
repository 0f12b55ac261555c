"""The pre-hsfs ``hops.featurestore`` functions the inference / petastorm notebooks use
(notebooks/featurestore/petastorm/PetastormHelloWorld.ipynb: ``create_training_dataset(df, name,
data_format='petastorm', petastorm_args={'schema': …})``, ``get_training_dataset(name)``;
notebooks/ml/Inference/*: ``get_training_dataset_path``).

Training datasets live under ``<project>_Training_Datasets/<name>_<version>/``; the
petastorm format stores Unischema-encoded Parquet readable with ``make_reader``; other
formats (csv, parquet, tfrecords, npy) go through the hsfs-style training dataset writer.
"""
from __future__ import annotations

from pathlib import Path

import pandas as pd

from .. import hdfs


def _td_root() -> Path:
    p = Path(hdfs.project_path()) / f"{hdfs.project_name()}_Training_Datasets"
    p.mkdir(parents=True, exist_ok=True)
    return p


def _fs():
    from .store import connection_quiet

    return connection_quiet().get_feature_store()


def _latest(name: str) -> int:
    vs = [int(p.name.rsplit("_", 1)[1]) for p in _td_root().glob(f"{name}_*") if p.name.rsplit("_", 1)[1].isdigit()]
    return max(vs, default=0)


def create_training_dataset(df, training_dataset: str, description: str = "", featurestore=None,
                            data_format: str = "tfrecords", training_dataset_version: int | None = None,
                            petastorm_args: dict | None = None, **kw) -> str:
    v = training_dataset_version or _latest(training_dataset) + 1
    if data_format == "petastorm":
        from ..petastorm.etl.dataset_metadata import write_rows
        from ..petastorm.unischema import Unischema

        schema: Unischema = (petastorm_args or {})["schema"]
        path = _td_root() / f"{training_dataset}_{v}"
        rows = df.to_dict("records") if isinstance(df, pd.DataFrame) else list(df)
        rows = [{k: r[k] for k in schema.fields} for r in rows]
        write_rows(str(path), schema, rows)
        return str(path)
    td = _fs().create_training_dataset(training_dataset, version=v, description=description,
                                       data_format=data_format, **kw)
    td.save(df)
    return td.location


def get_training_dataset_path(training_dataset: str, featurestore=None, training_dataset_version: int | None = None
                              ) -> str:
    v = training_dataset_version or _latest(training_dataset)
    p = _td_root() / f"{training_dataset}_{v}"
    if p.exists():
        return str(p)
    return _fs().get_training_dataset(training_dataset, v).location


def get_training_dataset(training_dataset: str, featurestore=None, training_dataset_version: int | None = None,
                         dataframe_type: str = "pandas") -> pd.DataFrame:
    path = Path(get_training_dataset_path(training_dataset, featurestore, training_dataset_version))
    if (path / "_common_metadata").exists():
        from ..petastorm.reader import make_reader

        with make_reader(str(path), shuffle_row_groups=False, workers_count=4) as r:
            return pd.DataFrame([row._asdict() for row in r])
    return _fs().get_training_dataset(training_dataset, training_dataset_version).read()


def get_featuregroup(featuregroup: str, featurestore=None, featuregroup_version: int = 1,
                     dataframe_type: str = "pandas") -> pd.DataFrame:
    return _fs().get_feature_group(featuregroup, featuregroup_version).read()


def create_featuregroup(df: pd.DataFrame, featuregroup: str, primary_key=None, description: str = "",
                        featuregroup_version: int = 1, online: bool = False, **kw):
    fg = _fs().create_feature_group(featuregroup, version=featuregroup_version, description=description,
                                    primary_key=[primary_key] if isinstance(primary_key, str) else primary_key,
                                    online_enabled=online)
    fg.save(df)
    return fg


def insert_into_featuregroup(df: pd.DataFrame, featuregroup: str, featuregroup_version: int = 1,
                             mode: str = "append", **kw):
    fg = _fs().get_feature_group(featuregroup, featuregroup_version)
    fg.insert(df, overwrite=(mode == "overwrite"))
    return fg


def get_features(features: list[str], featurestore=None, featuregroups_version_dict: dict | None = None,
                 join_key=None, dataframe_type: str = "pandas") -> pd.DataFrame:
    """Join the feature groups that hold ``features`` on their common primary key."""
    fs = _fs()
    groups = featuregroups_version_dict or {}
    if not groups:
        raise ValueError("pass featuregroups_version_dict={fg_name: version} to locate the features")
    q = None
    for name, ver in groups.items():
        fg = fs.get_feature_group(name, ver)
        cols = [f for f in features if f in [x.name for x in fg.features]]
        sel = fg.select(cols + [k for k in fg.primary_key if k not in cols])
        q = sel if q is None else q.join(sel, on=[join_key] if isinstance(join_key, str) else join_key)
    return q.read()[features]
