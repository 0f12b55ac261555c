"""TFX-style Chicago-taxi pipeline on MI355X: ExampleGen -> StatisticsGen -> SchemaGen -> Transform ->
Trainer -> Evaluator -> Pusher, run as an ``orchestration.DAG`` whose stages are ROCm jobs.

The reference README names a ``chicago_taxi_tfx_hopsworks`` notebook, pipeline notebooks and an
Airflow DAG ``chicago_tfx_airflow_pipeline.py`` (README.md:99-112) that are absent from the snapshot
(SURVEY §0.4), and BASELINE.json's north star asks for "the TFX Chicago-taxi Transform/Trainer stages
run as ROCm jobs instead of Spark/TF".  The feature engineering follows the public TFX taxi
example's ``preprocessing_fn``; see :mod:`.transform` for the analyze/apply split and
:mod:`.pipeline` for the components.
"""
from .taxi import RAW_COLUMNS, synth_raw_trips  # noqa: F401
from .transform import TaxiTransform, analyze, apply_numpy  # noqa: F401
