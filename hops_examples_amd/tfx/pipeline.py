"""The Chicago-taxi TFX pipeline as ROCm jobs chained by an ``orchestration.DAG``.

Components (TFX names; artifacts under ``<project>/Resources/tfx/<pipeline>/``):

=================  ==========================================================================
ExampleGen         raw trips (CSV or Parquet) -> ``examples/{train,eval}.parquet``; split by a hash of
                   ``trip_start_timestamp`` into 2:1 buckets (TFX's default 3 hash buckets)
StatisticsGen      feature statistics of the train split (``featurestore.statistics``: stats.hip
                   column statistics, histograms, correlations on the GPU)
SchemaGen          types, value domains and required-ness inferred from the statistics
Transform          analyze on train, apply to both splits (:mod:`.transform`; transform.hip) ->
                   ``transform/transform_fn.json`` + ``transformed/{train,eval}.parquet``
Trainer            wide&deep trainer (``models.widedeep``: the whole step in one kernel) fed by the
                   transformed Parquet streamed into HBM (``io.parquet``) -> ``trainer/model.pt``
Evaluator          accuracy / AUC / log-loss on the eval split; blesses the model above a threshold
Pusher             exports a blessed model + its transform_fn to the model registry (``model.export``)
=================  ==========================================================================

Transform and Trainer run as jobs (``jobs.create_job`` / ``HopsworksLaunchOperator``: separate
processes with their own GPU), the light stages as ``PythonOperator`` tasks — the shape of the
reference README's Airflow DAG ``chicago_tfx_airflow_pipeline.py`` (README.md:99-112, absent from
the snapshot).  ``python -m hops_examples_amd.tfx.pipeline <component> --root DIR`` is
each job's program (``tfx/job_main.py``).
"""
from __future__ import annotations

import argparse
import json
import sys
import time
import zlib
from pathlib import Path

import numpy as np
import pandas as pd

from .. import hdfs


def pipeline_root(name: str = "chicago_taxi") -> Path:
    return Path(hdfs.project_path()) / "Resources" / "tfx" / name


def _write_json(p: Path, obj) -> str:
    p.parent.mkdir(parents=True, exist_ok=True)
    p.write_text(json.dumps(obj, indent=1, default=float))
    return str(p)


# ------------------------------------------------------------------ components
def example_gen(root, raw_path) -> dict:
    root = Path(root)
    raw_path = str(raw_path)
    df = pd.read_parquet(raw_path) if raw_path.endswith(".parquet") else pd.read_csv(raw_path)
    h = np.array([zlib.crc32(str(v).encode()) % 3 for v in df["trip_start_timestamp"].to_numpy()])
    out = {}
    for split, mask in (("train", h < 2), ("eval", h == 2)):
        p = root / "examples" / f"{split}.parquet"
        p.parent.mkdir(parents=True, exist_ok=True)
        df[mask].reset_index(drop=True).to_parquet(p, index=False, row_group_size=65536)
        out[split] = {"path": str(p), "rows": int(mask.sum())}
    _write_json(root / "examples" / "splits.json", out)
    return out


def statistics_gen(root) -> dict:
    from ..featurestore import statistics

    root = Path(root)
    df = pd.read_parquet(root / "examples" / "train.parquet")
    st = statistics.compute(df, statistics.StatisticsConfig(enabled=True, histograms=True, correlations=True))
    _write_json(root / "statistics" / "train_stats.json", st)
    return st


def schema_gen(root) -> dict:
    root = Path(root)
    st = json.loads((root / "statistics" / "train_stats.json").read_text())
    feats = []
    for c in st["columns"]:
        f = {"name": c["column"], "type": "FLOAT" if c["dataType"] == "Fractional" else "BYTES",
             "presence": {"min_fraction": round(float(c["completeness"]), 4)}}
        if c["dataType"] == "Fractional":
            f["domain"] = {"min": c["minimum"], "max": c["maximum"]}
        feats.append(f)
    schema = {"feature": feats}
    _write_json(root / "schema" / "schema.json", schema)
    return schema


def transform(root, device=None) -> dict:
    from .transform import analyze, transformed_frame

    root = Path(root)
    t0 = time.perf_counter()
    train = pd.read_parquet(root / "examples" / "train.parquet")
    tf = analyze(train, device=device)
    tf.save(root / "transform" / "transform_fn.json")
    out = {"analyze_s": round(time.perf_counter() - t0, 3)}
    for split in ("train", "eval"):
        df = train if split == "train" else pd.read_parquet(root / "examples" / "eval.parquet")
        t1 = time.perf_counter()
        dense, cat, label = tf.apply(df, device=device)
        p = root / "transformed" / f"{split}.parquet"
        p.parent.mkdir(parents=True, exist_ok=True)
        transformed_frame(dense, cat, label).to_parquet(p, index=False, row_group_size=65536)
        out[split] = {"path": str(p), "rows": len(df), "apply_s": round(time.perf_counter() - t1, 3)}
    out["device"] = str(dense.device)
    _write_json(root / "transform" / "transform_stats.json", out)
    return out


def _load_transformed(root: Path, split: str, device):
    """Transformed examples -> HBM (Parquet row groups through the pinned staging ring)."""
    import torch

    from ..io.parquet import ParquetDeviceReader
    from ..models.widedeep import DENSE_FLOAT_FEATURE_KEYS, N_WIDE

    nd = len(DENSE_FLOAT_FEATURE_KEYS)
    cols = [f"dense_{j}" for j in range(nd)] + [f"wide_{j}" for j in range(N_WIDE)] + ["label"]
    x = ParquetDeviceReader(root / "transformed" / f"{split}.parquet", cols, device=device).read()
    dense = x[:, :nd].contiguous()
    cat = x[:, nd:nd + N_WIDE].round().to(torch.int64).contiguous()
    label = x[:, nd + N_WIDE:].contiguous()
    return dense, cat, label


def trainer(root, steps: int = 2000, batch: int = 40, device=None) -> dict:
    import torch

    from ..models.widedeep import FusedWideDeepStep, TaxiWideDeep, make_optimizer
    from ..runtime.arena import ParamArena
    from ..runtime.step import TrainStep

    root = Path(root)
    dev = torch.device(device) if device is not None else (
        torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu"))
    torch.manual_seed(0)
    dense, cat, label = _load_transformed(root, "train", dev)
    nb = dense.shape[0] // batch
    if nb < 1:
        raise ValueError(f"{dense.shape[0]} transformed training rows < one batch of {batch}")
    model = TaxiWideDeep().to(dev)
    ParamArena.from_module(model, dev)
    opt = make_optimizer(model)
    xs = (dense[:nb * batch].view(nb, batch, -1).contiguous(), cat[:nb * batch].view(nb, batch, -1).contiguous())
    ys = label[:nb * batch].view(nb, batch, 1).contiguous()
    fused = FusedWideDeepStep(model, opt) if dev.type == "cuda" else None
    t0 = time.perf_counter()
    if fused is not None and fused.ok(batch):
        r = fused.run_resident(xs, ys, steps)
        path = "fused"
    else:
        st = TrainStep(model, opt, "bce_logits", graph=dev.type == "cuda", forward_fn=lambda m, x: m(*x))
        for i in range(steps):
            j = i % nb
            r = st((xs[0][j], xs[1][j]), ys[j])
        path = "layerwise"
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    p = root / "trainer" / "model.pt"
    p.parent.mkdir(parents=True, exist_ok=True)
    torch.save({k: v.detach().cpu() for k, v in model.state_dict().items()}, p)
    res = {"model": str(p), "steps": steps, "batch": batch, "train_rows": int(dense.shape[0]), "step": path,
           "steps_per_sec": round(steps / el, 1), "final_loss": round(float(r["loss"].reshape(-1)[0]), 4),
           "device": str(dev)}
    _write_json(root / "trainer" / "metrics.json", res)
    return res


def _auc(score: np.ndarray, y: np.ndarray) -> float:
    pos, neg = y > 0.5, y <= 0.5
    if not pos.any() or not neg.any():
        return float("nan")
    ranks = pd.Series(score).rank().to_numpy()
    return float((ranks[pos].sum() - pos.sum() * (pos.sum() + 1) / 2) / (pos.sum() * neg.sum()))


def evaluator(root, threshold: float = 0.6, device=None) -> dict:
    import torch

    from ..models.widedeep import TaxiWideDeep
    from ..runtime.arena import ParamArena

    root = Path(root)
    dev = torch.device(device) if device is not None else (
        torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu"))
    dense, cat, label = _load_transformed(root, "eval", dev)
    model = TaxiWideDeep()
    model.load_state_dict(torch.load(root / "trainer" / "model.pt", map_location="cpu", weights_only=True))
    model.to(dev)
    ParamArena.from_module(model, dev)
    with torch.no_grad():
        logits = torch.cat([model(dense[i:i + 4096], cat[i:i + 4096]).float()
                            for i in range(0, dense.shape[0], 4096)])
    p = torch.sigmoid(logits).cpu().numpy()[:, 0]
    y = label.cpu().numpy()[:, 0]
    acc = float(((p > 0.5) == (y > 0.5)).mean())
    eps = 1e-7
    ll = float(-(y * np.log(p + eps) + (1 - y) * np.log(1 - p + eps)).mean())
    res = {"accuracy": acc, "auc": _auc(p, y), "log_loss": ll, "eval_rows": int(len(y)),
           "baseline_accuracy": float(max(y.mean(), 1 - y.mean())), "blessed": acc >= threshold}
    _write_json(root / "evaluator" / "metrics.json", res)
    return res


def pusher(root, model_name: str = "chicago_taxi_wide_deep") -> dict:
    from .. import model as registry

    root = Path(root)
    ev = json.loads((root / "evaluator" / "metrics.json").read_text())
    if not ev.get("blessed"):
        return {"pushed": False, "reason": "model not blessed by the evaluator"}
    stage = root / "pusher" / "export"
    stage.mkdir(parents=True, exist_ok=True)
    for src in (root / "trainer" / "model.pt", root / "transform" / "transform_fn.json"):
        (stage / src.name).write_bytes(src.read_bytes())
    registry.export(str(stage), model_name, metrics={k: ev[k] for k in ("accuracy", "auc")})
    best = registry.get_best_model(model_name, "accuracy", registry.Metric.MAX)
    res = {"pushed": True, "model": model_name, "version": best["version"]}
    _write_json(root / "pusher" / "result.json", res)
    return res


# ------------------------------------------------------------------ DAG
_COMPONENTS = ("example_gen", "statistics_gen", "schema_gen", "transform", "trainer", "evaluator", "pusher")


def build_dag(raw_path, name: str = "chicago_taxi", train_steps: int = 2000, batch: int = 40,
              threshold: float = 0.6, jobs_for_heavy_stages: bool = True):
    """The pipeline DAG: ExampleGen >> StatisticsGen >> SchemaGen >> Transform >> Trainer >> Evaluator >>
    Pusher.  With ``jobs_for_heavy_stages`` Transform and Trainer are jobs (own process + GPU)."""
    from .. import jobs
    from ..orchestration import DAG, HopsworksLaunchOperator, PythonOperator

    root = pipeline_root(name)
    dag = DAG(f"{name}_tfx_pipeline", schedule_interval="@once")
    prog = str(Path(__file__).resolve().parent / "job_main.py")
    t_eg = PythonOperator(dag, "ExampleGen", example_gen, op_kwargs={"root": root, "raw_path": raw_path})
    t_sg = PythonOperator(dag, "StatisticsGen", statistics_gen, op_kwargs={"root": root})
    t_sc = PythonOperator(dag, "SchemaGen", schema_gen, op_kwargs={"root": root})
    if jobs_for_heavy_stages:
        for comp, extra in (("transform", ""), ("trainer", f" --steps {train_steps} --batch {batch}")):
            jobs.create_job(f"{name}_{comp}", {"appPath": prog, "jobType": "PYTHON", "spark.executor.gpus": 1,
                                               "defaultArgs": f"{comp} --root {root}{extra}"})
        t_tf = HopsworksLaunchOperator(dag, "Transform", job_name=f"{name}_transform",
                                       job_arguments=f"transform --root {root}")
        t_tr = HopsworksLaunchOperator(dag, "Trainer", job_name=f"{name}_trainer",
                                       job_arguments=f"trainer --root {root} --steps {train_steps} --batch {batch}")
    else:
        t_tf = PythonOperator(dag, "Transform", transform, op_kwargs={"root": root})
        t_tr = PythonOperator(dag, "Trainer", trainer, op_kwargs={"root": root, "steps": train_steps, "batch": batch})
    t_ev = PythonOperator(dag, "Evaluator", evaluator, op_kwargs={"root": root, "threshold": threshold})
    t_pu = PythonOperator(dag, "Pusher", pusher, op_kwargs={"root": root})
    t_eg >> t_sg >> t_sc >> t_tf >> t_tr >> t_ev >> t_pu
    return dag, root


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="hops_examples_amd.tfx.pipeline")
    ap.add_argument("component", choices=_COMPONENTS)
    ap.add_argument("--root", required=True)
    ap.add_argument("--raw", default=None)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--batch", type=int, default=40)
    a = ap.parse_args(argv)
    fn = {"example_gen": lambda: example_gen(a.root, a.raw), "statistics_gen": lambda: statistics_gen(a.root),
          "schema_gen": lambda: schema_gen(a.root), "transform": lambda: transform(a.root),
          "trainer": lambda: trainer(a.root, a.steps, a.batch), "evaluator": lambda: evaluator(a.root),
          "pusher": lambda: pusher(a.root)}[a.component]
    print(json.dumps(fn(), default=float)[:2000], flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
