# %% [markdown]
# # Chicago-taxi TFX pipeline on MI355X
# The reference README describes a TFX Chicago-taxi pipeline (Transform + Trainer, an Airflow DAG
# `chicago_tfx_airflow_pipeline.py`; README.md:99-112) whose notebooks are not in the snapshot.
# Here the same stages run as ROCm jobs chained by an `orchestration.DAG`:
# ExampleGen -> StatisticsGen -> SchemaGen -> Transform (GPU analyze + apply) -> Trainer (wide&deep,
# one kernel per step, data streamed Parquet -> HBM) -> Evaluator -> Pusher (model registry).
# Raw trips are synthetic with the public dataset's column names (no network for the extract).
# %%
import json
import os

from hops_examples_amd import hdfs
from hops_examples_amd.tfx import pipeline, synth_raw_trips

FAST = os.environ.get("HOPSX_FAST") == "1"
n_trips = 6_000 if FAST else 200_000
raw = os.path.join(hdfs.project_path(), "Resources", "chicago_taxi_raw.csv")
os.makedirs(os.path.dirname(raw), exist_ok=True)
synth_raw_trips(n_trips, seed=1).to_csv(raw, index=False)

# %%
dag, root = pipeline.build_dag(raw, train_steps=300 if FAST else 5000, threshold=0.6)
state = dag.run()
print(state)
assert all(v == "success" for v in state.values()), getattr(dag, "errors", {})

# %%
for stage in ("transform/transform_stats.json", "trainer/metrics.json", "evaluator/metrics.json",
              "pusher/result.json"):
    print(stage, json.loads((root / stage).read_text()))
